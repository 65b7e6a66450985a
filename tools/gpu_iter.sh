# one iteration on the GPU box: all GPU tests, then the 100k bench and its kernel-trace summary
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/iter
mkdir -p $O
SWIM_TEST_LOGDIR=$GRAFT_REPO_ROOT/$O timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -4 $O/pytest.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep metric $O/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline > $O/prof_bench.log 2>&1
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
head -25 $O/kernel_stats.csv | cut -c1-160
