# round 3: the target-major gossip plane. The gossip-heavy -m gpu cases first (stop at the first failure), then the
# rest of the suite, then the C2 / C5-shaped / c3dyn lines with kernel traces
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3g}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${2:-c1 or golden or dissemination or partition or loss or user_gossip or rumor or fuzz or leaves or joins}" > $O/tests.log 2>&1
tail -n 1 $O/tests.log
for ww in c2:12 c5:25 c3dyn:3; do
  w=${ww%%:*}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/t_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 4 --warmup ${ww##*:} --no-cpu-baseline > $O/b_$w.log 2>&1
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $O/b_$w.log)"
done
