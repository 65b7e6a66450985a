# gossip-plane change check: the gossip-heavy -m gpu cases, then the C2, C5-shaped and c3dyn lines with traces
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-gsp}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${2:-partition or loss or dissemination or fuzz or rumor or golden or kill_many or user_gossips or joins or leaves or c1}" > $O/tests.log 2>&1
tail -n 1 $O/tests.log
for ww in c2:12 c5:25 c3dyn:3; do
  w=${ww%%:*}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/t_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 4 --warmup ${ww##*:} --no-cpu-baseline > $O/b_$w.log 2>&1
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $O/b_$w.log) $(grep -h 'k_gossip_apply\|k_gossip_scan' $O/t_$w/run_kernel_stats.csv | cut -d, -f4 | tr '\n' ' ')"
done
