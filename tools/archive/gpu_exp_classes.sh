# timing experiment: k_member_tick with the bodies of class 0 (SWIM_EXP=32) or classes 1-3 (64) skipped
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-expcls}
mkdir -p $O
for e in ${2:-0 32 64}; do
  SWIM_EXP=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t$e -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/l$e.log 2>&1
  echo "exp=$e $(grep -h k_member_tick $O/t$e/run_kernel_stats.csv | cut -d, -f4-6)"
done
