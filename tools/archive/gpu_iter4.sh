# fused member kernel (triage + control + end-of-tick flag in one launch): the whole -m gpu suite, the default bench
# line with its kernel trace, then the gossip-heavy C2 and C5-shaped lines with their CPU baselines and traces
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/iter4
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c3 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/trace_c3.log 2>&1
timeout -k 10 500 python -u bench.py --workload c2 --steps 8 --warmup 12 > $O/bench_c2.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench_c2.log
timeout -k 10 500 python -u bench.py --workload c5 --steps 10 --warmup 25 > $O/bench_c5.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench_c5.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace_c2 -o run --output-format csv -- python3 bench.py --workload c2 --steps 4 --warmup 12 --no-cpu-baseline > $O/trace_c2.log 2>&1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace_c5 -o run --output-format csv -- python3 bench.py --workload c5 --steps 5 --warmup 25 --no-cpu-baseline > $O/trace_c5.log 2>&1
ls $O
