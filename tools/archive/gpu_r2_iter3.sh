# round 2 iteration: a -k selection of the -m gpu suite, the C3 bench line with its kernel trace, the C2 bench line
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-it3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${2:-c1 or preconverged or partition or fuzz_single or member_configs or rumor_mode_sharded}" > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/bench_c3.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench_c3.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c3 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/trace_c3.log 2>&1
grep -h "k_sync_diff\|k_member_tick" $O/trace_c3/run_kernel_stats.csv | cut -c1-160
timeout -k 10 300 python -u bench.py --workload c2 --steps 6 --warmup 12 --no-cpu-baseline > $O/bench_c2.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench_c2.log
