# iteration: the whole -m gpu suite, then the C2 line and its member-kernel phase cycles (SWIM_EXP=16)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r2iter}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${2:+-k "$2"} > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --workload c2 --steps 6 --warmup 12 --no-cpu-baseline > $O/bench_c2.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench_c2.log
SWIM_EXP=16 timeout -k 10 300 python -u bench.py --workload c2 --steps 3 --warmup 12 --no-cpu-baseline > $O/phases.log 2>&1
grep "exp:" $O/phases.log | tail -1
