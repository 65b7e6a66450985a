# round-2 evidence: the headline profile (tools/gpu_profile_round.sh: bench line with CPU baseline, kernel trace,
# k_sync_diff FETCH_SIZE / WRITE_SIZE passes), then the secondary lines (c3dyn, C2, C5-shaped) with kernel traces
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_profile_round.sh
O=gpurun_out/lines
mkdir -p $O
timeout -k 10 400 python -u bench.py --workload c3dyn --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c3dyn.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c3dyn -o run --output-format csv -- python3 bench.py --workload c3dyn --steps 10 --warmup 3 --no-cpu-baseline > $O/trace_c3dyn.log 2>&1
timeout -k 10 500 python -u bench.py --workload c2 --steps 8 --warmup 12 > $O/bench_c2.log 2>&1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace_c2 -o run --output-format csv -- python3 bench.py --workload c2 --steps 4 --warmup 12 --no-cpu-baseline > $O/trace_c2.log 2>&1
timeout -k 10 500 python -u bench.py --workload c5 --steps 10 --warmup 25 > $O/bench_c5.log 2>&1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace_c5 -o run --output-format csv -- python3 bench.py --workload c5 --steps 5 --warmup 25 --no-cpu-baseline > $O/trace_c5.log 2>&1
grep -ho '"ms_per_step": [0-9.]*' gpurun_out/round/bench.json $O/bench_*.log
