# round 3: the C4 schedule (two halves partitioned from period 0, unblockAll at period 200, run to 320) at growing N
# on one GPU: wall time per 10-period chunk and the storm counters (tools/exp_c4.py)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3c4}
mkdir -p $O
for n in ${2:-2000 4000 8000}; do
  C4_RING=${5:-0} C4_CHUNK=${4:-10} timeout -k 10 ${3:-500} python -u tools/exp_c4.py $n 200 320 > $O/c4_$n.log 2>&1 || { tail -5 $O/c4_$n.log; exit 1; }
  tail -2 $O/c4_$n.log
done
