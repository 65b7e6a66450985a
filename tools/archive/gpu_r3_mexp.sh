# round 3: C3 member-kernel timing experiments (wrong results, timing only): rocprof kernel averages with the bodies of
# class 0 skipped (32), classes 1-3 skipped (64), all bodies skipped (96), and the per-wave timeline (512)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3mx}
mkdir -p $O
for e in 0 32 64 96; do
  SWIM_EXP=$e timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t$e -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-events > $O/l$e.log 2>&1
  echo "exp=$e $(grep -h 'k_member_tick\|k_sync_diff' $O/t$e/run_kernel_stats.csv | cut -d, -f3-4 | tr '\n' ' ')"
done
SWIM_EXP=512 timeout -k 10 200 python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-events > $O/l512.log 2>&1
grep -h "exp512" $O/l512.log | tail -12
