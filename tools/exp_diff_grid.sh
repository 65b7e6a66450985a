mkdir -p gpurun_out/r5p
for g in 1024 1536 2048 3072 4096; do
  SWIM_DIFF_GRID=$g timeout -k 10 200 python3 bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r5p/grid_$g.log 2>&1 || exit 1
  echo "grid $g $(grep -o '"ms_per_step": [0-9.]*\|"avg_launch_us": [0-9.]*\|"frac": [0-9.]*' gpurun_out/r5p/grid_$g.log | tr '\n' ' ')"
done
