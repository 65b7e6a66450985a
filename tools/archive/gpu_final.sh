# end-of-round check of the sampled k_sync_diff timing: bench lines (events / no events), -m gpu suite, smoke, kernel stats
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/bench_ev.log 2>&1
timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-events > $O/bench_noev.log 2>&1
grep -h '^{' $O/bench_ev.log $O/bench_noev.log | python -c "import sys,json;[print(json.loads(l)['ms_per_step'], json.loads(l)['roofline']) for l in sys.stdin]"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c3 -- python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/prof_bench.log 2>&1
grep '^{' $O/prof_bench.log | python -c "import sys,json;[print(json.loads(l)['ms_per_step'], json.loads(l)['roofline']['avg_launch_us']) for l in sys.stdin]"
