# C3 per-tick gaps: bench with and without the k_sync_diff HIP events, and a kernel trace with timestamps
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gaps
mkdir -p $O
timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/bench_ev.log 2>&1
timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-events > $O/bench_noev.log 2>&1
grep -h '^{' $O/bench_ev.log $O/bench_noev.log | python -c "import sys,json;[print(json.loads(l)['ms_per_step']) for l in sys.stdin]"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o c3 -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-events > $O/trace.log 2>&1
find $O/trace -name '*kernel_trace.csv' | head -3
