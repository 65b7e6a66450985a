# iteration check: the whole -m gpu suite, then the default bench line (no CPU baseline) with its kernel trace
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/iter
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1
grep metric $O/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline > $O/trace_bench.log 2>&1
find $O/trace -name "*kernel_stats.csv" -exec head -8 {} \;
