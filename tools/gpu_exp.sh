# timing experiments on the C2 gossip plane (SWIM_EXP knobs give wrong results; timing only)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/exp
mkdir -p $O
for e in 0 1 2; do
  SWIM_EXP=$e timeout -k 10 300 python -u tools/exp_c2.py 10000 14 > $O/exp$e.log 2>&1 || { tail -20 $O/exp$e.log; exit 1; }
  echo "SWIM_EXP=$e"; tail -4 $O/exp$e.log
done
