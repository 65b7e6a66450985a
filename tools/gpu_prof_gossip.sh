# kernel-trace summaries of the gossip-heavy workloads (C5-shaped rumor mode at 100k, C2 at 10k)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pg
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c5 -o run --output-format csv -- python3 bench.py --workload c5 --warmup 20 --steps 4 --no-cpu-baseline > $O/c5.log 2>&1
find $O/c5 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/c5_kernel_stats.csv
head -10 $O/c5_kernel_stats.csv | cut -c1-150
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c2 -o run --output-format csv -- python3 bench.py --workload c2 --warmup 10 --steps 4 --no-cpu-baseline > $O/c2.log 2>&1
find $O/c2 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/c2_kernel_stats.csv
head -10 $O/c2_kernel_stats.csv | cut -c1-150
