# the gossip-heavy C2 and C5-shaped bench lines (with their CPU baselines) and kernel traces
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gossip
mkdir -p $O
timeout -k 10 500 python -u bench.py --workload c2 --steps 8 --warmup 12 > $O/bench_c2.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench_c2.log
timeout -k 10 500 python -u bench.py --workload c5 --steps 10 --warmup 25 > $O/bench_c5.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench_c5.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace_c2 -o run --output-format csv -- python3 bench.py --workload c2 --steps 4 --warmup 12 --no-cpu-baseline > $O/trace_c2.log 2>&1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace_c5 -o run --output-format csv -- python3 bench.py --workload c5 --steps 5 --warmup 25 --no-cpu-baseline > $O/trace_c5.log 2>&1
ls $O
