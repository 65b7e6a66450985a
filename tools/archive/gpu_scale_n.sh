cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sn
for n in 10000 30000 100000; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sn/p$n -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-events --members $n > gpurun_out/sn/b$n.log 2>&1
f=$(find gpurun_out/sn/p$n -name "*kernel_stats.csv" | head -1)
echo "N=$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sn/b$n.log)"; grep -E "k_member_tick|k_sync_diff|k_tick_flag" $f | cut -d, -f1-4
done
