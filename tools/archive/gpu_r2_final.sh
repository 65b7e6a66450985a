# round-2 closing run: smoke, the whole -m gpu suite, then the secondary lines (c3dyn, C2, C5-shaped) with kernel traces
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -n 1 $O/gpu_tests.log
L=gpurun_out/lines
mkdir -p $L
timeout -k 10 400 python -u bench.py --workload c3dyn --steps 20 --warmup 3 --no-cpu-baseline > $L/bench_c3dyn.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $L/trace_c3dyn -o run --output-format csv -- python3 bench.py --workload c3dyn --steps 10 --warmup 3 --no-cpu-baseline > $L/trace_c3dyn.log 2>&1
timeout -k 10 500 python -u bench.py --workload c2 --steps 8 --warmup 12 > $L/bench_c2.log 2>&1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $L/trace_c2 -o run --output-format csv -- python3 bench.py --workload c2 --steps 4 --warmup 12 --no-cpu-baseline > $L/trace_c2.log 2>&1
timeout -k 10 500 python -u bench.py --workload c5 --steps 10 --warmup 25 > $L/bench_c5.log 2>&1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $L/trace_c5 -o run --output-format csv -- python3 bench.py --workload c5 --steps 5 --warmup 25 --no-cpu-baseline > $L/trace_c5.log 2>&1
grep -ho '"ms_per_step": [0-9.]*' $L/bench_*.log
