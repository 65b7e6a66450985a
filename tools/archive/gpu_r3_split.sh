# round 3: the split member tick (triage + classes 1-3 beside k_sync_diff, class 0 after it) in speculative batches:
# C3 bench with and without it (SWIM_NO_SPLIT), a kernel trace, then a -m gpu selection
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3split}
mkdir -p $O
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_split.log 2>&1
echo "split $(grep -o '"ms_per_step": [0-9.]*\|"avg_launch_us": [0-9.]*' $O/bench_split.log | tr '\n' ' ')"
SWIM_NO_SPLIT=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_nosplit.log 2>&1
echo "nosplit $(grep -o '"ms_per_step": [0-9.]*\|"avg_launch_us": [0-9.]*' $O/bench_nosplit.log | tr '\n' ' ')"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t_c3 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-events > $O/b_c3.log 2>&1
grep -h "k_member\|k_sync_diff" $O/t_c3/run_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${2:-c1 or golden or parity or partition or join or leave or metadata or user_gossip or dyn or fuzz or delay or fallback}" > $O/tests.log 2>&1
tail -n 1 $O/tests.log
