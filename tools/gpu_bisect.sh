# perf bisect of the C3 line across trees under _bisect/ (not committed; drop ./_bisect from .gpurunignore for the
# run): the bench line of each and its kernel averages (rocprofv3, no HIP events)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bisect
mkdir -p $O
for c in HEAD $(ls _bisect); do
  if [ $c = HEAD ]; then D=$R; else D=$R/_bisect/$c; fi
  cd $D
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/b_$c.log 2>&1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t_$c -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-events > $O/tl_$c.log 2>&1
  echo "== $c $(grep -o '"ms_per_step": [0-9.]*' $O/b_$c.log) $(grep -o '"ms_per_step": [0-9.]*' $O/tl_$c.log) $(grep -h 'k_sync_diff\|k_member_tick' $O/t_$c/run_kernel_stats.csv | cut -d, -f3-4 | tr '\n' ' ')"
done
