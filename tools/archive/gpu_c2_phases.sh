# C2: member-kernel shader cycles per phase (SWIM_EXP=16 timing experiment; results are not a bench line)
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-c2phases}
mkdir -p $O
SWIM_EXP=16 timeout -k 10 300 python -u bench.py --workload c2 --steps 3 --warmup 12 --no-cpu-baseline > $O/phases.log 2>&1
grep "exp:" $O/phases.log | tail -4
