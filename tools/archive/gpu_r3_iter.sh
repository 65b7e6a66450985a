# round 3 iteration: a -k selection of the -m gpu suite (stop at the first failure), then the gossip-heavy lines
# with kernel traces and the per-tick breakdown of the last ticks
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3i}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${2:-c1 or golden or dissemination or partition or loss or user_gossip or rumor or fuzz or fallback or tiny or memory}" > $O/tests.log 2>&1
tail -n 1 $O/tests.log
for ww in ${3:-c2:12 c5:25 c3dyn:3}; do
  w=${ww%%:*}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/t_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 4 --warmup ${ww##*:} --no-cpu-baseline > $O/b_$w.log 2>&1
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $O/b_$w.log)"
  python3 tools/tick_breakdown.py $O/t_$w/run_kernel_trace.csv 4 | tail -2
done
