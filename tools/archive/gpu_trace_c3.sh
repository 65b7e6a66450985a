# kernel-trace summary of the default C3 bench (per-kernel averages)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/trace_c3
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench.log
head -6 $O/t/run_kernel_stats.csv
