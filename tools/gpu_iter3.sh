# split member tick (busy members beside k_sync_diff on a second stream): the whole -m gpu suite, then the default
# bench line under a few k_sync_diff grid sizes and with the split disabled
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/iter3
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for g in 1024 512 768 2048; do
  SWIM_DIFF_GRID=$g timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/bench_g$g.log 2>&1
  echo "grid $g: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_g$g.log) $(grep -o '"avg_launch_us": [0-9.]*' $O/bench_g$g.log)"
done
SWIM_NO_SPLIT=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/bench_nosplit.log 2>&1
echo "nosplit: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_nosplit.log) $(grep -o '"avg_launch_us": [0-9.]*' $O/bench_nosplit.log)"
