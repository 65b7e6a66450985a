# timing experiment at C2: the largest per-member cycles of each member-kernel phase (SWIM_EXP=128), per step
cd $GRAFT_REPO_ROOT
O=gpurun_out/expc2max
mkdir -p $O
SWIM_EXP=128 timeout -k 10 300 python -u bench.py --workload c2 --steps 3 --warmup 12 --no-cpu-baseline > $O/max.log 2>&1
grep "exp:" $O/max.log | tail -4
SWIM_EXP=128 timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > $O/max_c3.log 2>&1
grep "exp:" $O/max_c3.log | tail -2
