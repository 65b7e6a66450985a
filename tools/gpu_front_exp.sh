# timing experiment of the fused tick (SWIM_FRONT_EXP, wrong results): k_tick_front without its member bodies (1),
# without its diff (2), and as built (0); per-kernel average durations over the last ticks
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4f}
mkdir -p $O
for e in 0 1 2; do
  SWIM_FRONT_EXP=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t$e -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-events > $O/l$e.log 2>&1
  echo "exp=$e $(python3 tools/tick_breakdown.py $O/t$e/run_kernel_trace.csv 10 | tail -1)"
done
