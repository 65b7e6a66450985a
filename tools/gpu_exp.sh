# gossip-send work counters (SWIM_EXP=4 only counts; results are exact)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/exp
mkdir -p $O
SWIM_EXP=4 timeout -k 10 300 python -u tools/exp_c2.py 10000 13 > $O/exp4.log 2>&1 || { tail -20 $O/exp4.log; exit 1; }
tail -6 $O/exp4.log
