# round 3: the C3 headline line (default bench) with a kernel trace and its per-tick timeline, and the member-kernel
# class timing experiments (SWIM_EXP=32: class-0 bodies skipped, 64: classes 1-3 skipped; wrong results, timing only)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3c3}
mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/t_c3 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-events > $O/b_c3.log 2>&1
python3 tools/tick_breakdown.py $O/t_c3/run_kernel_trace.csv 20 | tail -1
for e in ${2:-32 64}; do
  SWIM_EXP=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t$e -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-events > $O/l$e.log 2>&1
  echo "exp=$e $(grep -h k_member_tick $O/t$e/run_kernel_stats.csv | cut -d, -f4-6)"
done
