# per-kernel times at a shard's share of C3 (100k / 8 = 12.5k observers' worth of members), single GPU
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/trace_small
mkdir -p $O
for n in 12500 25000; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t$n -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --members $n > $O/bench$n.log 2>&1
echo "$n: $(grep -o '"ms_per_step": [0-9.]*' $O/bench$n.log)"
head -4 $O/t$n/run_kernel_stats.csv | cut -c1-140
done
