# parity subset + the dynamic 100k line (c3dyn) with its kernel trace + C2 line
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-dyn}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${2:-c1 or partition or fuzz_single or same_tick or kill_many or user_gossips or joins}" > $O/tests.log 2>&1
tail -n 1 $O/tests.log
timeout -k 10 400 python -u bench.py --workload c3dyn --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c3dyn.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench_c3dyn.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c3dyn -o run --output-format csv -- python3 bench.py --workload c3dyn --steps 6 --warmup 3 --no-cpu-baseline > $O/trace_c3dyn.log 2>&1
grep -h "k_member_tick\|k_gossip_send\|k_gossip_apply" $O/trace_c3dyn/run_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 300 python -u bench.py --workload c2 --steps 6 --warmup 12 --no-cpu-baseline > $O/bench_c2.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench_c2.log
