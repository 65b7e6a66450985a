# round 3: the whole -m gpu suite (no -x: every failure listed), smoke, then the gossip-heavy lines with traces and
# the C2 send-work counters (SWIM_EXP=4)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3f}
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || true
tail -n 1 $O/tests.log
grep -E "^FAILED|^ERROR" $O/tests.log | head -20 || true
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
for ww in c2:12 c5:25 c3dyn:3; do
  w=${ww%%:*}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/t_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 4 --warmup ${ww##*:} --no-cpu-baseline > $O/b_$w.log 2>&1
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $O/b_$w.log)"
done
SWIM_EXP=4 timeout -k 10 300 python -u bench.py --workload c2 --steps 3 --warmup 14 --no-cpu-baseline > $O/c2_exp4.log 2>&1
grep "exp:" $O/c2_exp4.log | tail -3
