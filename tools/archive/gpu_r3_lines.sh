# round 3 measurement pass: the C3 headline (default bench, 20 steps) with a kernel trace and per-tick breakdown, then
# the gossip-plane lines (C2, C5-shaped, c3dyn) with kernel traces
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3lines}
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c3.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench_c3.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t_c3 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-events > $O/b_c3.log 2>&1
python3 tools/tick_breakdown.py $O/t_c3/run_kernel_trace.csv 20 | tail -2
for ww in ${2:-c2:12 c5:25 c3dyn:3}; do
  w=${ww%%:*}
  timeout -k 10 300 python -u bench.py --workload $w --steps 8 --warmup ${ww##*:} --no-cpu-baseline > $O/bench_$w.log 2>&1
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$w.log)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 3 --warmup ${ww##*:} --no-cpu-baseline > $O/b_$w.log 2>&1
  python3 tools/tick_breakdown.py $O/t_$w/run_kernel_trace.csv 4 | tail -1
done
