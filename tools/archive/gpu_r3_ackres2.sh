# round 3: SYNC_ACK resolution, second cut — -m gpu suite, the C3 line and its kernel trace
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3ackres3}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider ${2:-} > $O/tests.log 2>&1 || true
tail -n 1 $O/tests.log
grep -E "^FAILED|^ERROR" $O/tests.log | head -30 || true
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/c3.json 2> $O/c3.err
grep -o '"ms_per_step": [0-9.]*\|"avg_launch_us": [0-9.]*' $O/c3.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/trace_bench.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/trace_bench.log
