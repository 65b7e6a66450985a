# round evidence for the gossip-heavy configs: C5-shaped and C2 bench lines (with CPU baselines), kernel traces
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gr
mkdir -p $O
timeout -k 10 500 python -u bench.py --workload c5 --warmup 25 --steps 10 > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
tail -1 $O/c5.log | cut -c1-200
timeout -k 10 500 python -u bench.py --workload c2 --warmup 12 --steps 8 > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
tail -1 $O/c2.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c5 -o run --output-format csv -- python3 bench.py --workload c5 --warmup 20 --steps 4 --no-cpu-baseline > $O/c5p.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c2 -o run --output-format csv -- python3 bench.py --workload c2 --warmup 10 --steps 4 --no-cpu-baseline > $O/c2p.log 2>&1
find $O -name "*kernel_stats.csv"
