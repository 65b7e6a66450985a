# round 3: SYNC_ACK resolution — the whole -m gpu suite, then C3 / c3dyn lines with and without it
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3ackres}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider ${2:-} > $O/tests.log 2>&1 || true
tail -n 1 $O/tests.log
grep -E "^FAILED|^ERROR" $O/tests.log | head -30 || true
for w in c3 c3dyn; do
  timeout -k 10 300 python3 -u bench.py --workload $w --steps 30 --warmup 3 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err
  grep -o '"ms_per_step": [0-9.]*' $O/bench_$w.json
  SWIM_NO_ACKRES=1 timeout -k 10 300 python3 -u bench.py --workload $w --steps 30 --warmup 3 --no-cpu-baseline > $O/bench_${w}_noack.json 2> $O/bench_${w}_noack.err
  grep -o '"ms_per_step": [0-9.]*' $O/bench_${w}_noack.json
done
