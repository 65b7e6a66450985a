# timing experiments at C2 (wrong results): member-kernel phase cycles (SWIM_EXP=16) and class-skip kernel times
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-expc2}
mkdir -p $O
SWIM_EXP=16 timeout -k 10 300 python -u bench.py --workload c2 --steps 3 --warmup 12 --no-cpu-baseline > $O/phases.log 2>&1
grep "exp:" $O/phases.log | tail -2
for e in 0 32 64; do
  SWIM_EXP=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t$e -o run --output-format csv -- python3 bench.py --workload c2 --steps 2 --warmup 12 --no-cpu-baseline > $O/l$e.log 2>&1
  echo "exp=$e $(grep -h k_member_tick $O/t$e/run_kernel_stats.csv | cut -d, -f4-7)"
done
