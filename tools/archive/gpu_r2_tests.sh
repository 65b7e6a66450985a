# round 2: the new parity cases first (same-tick SYNC, device known answers, fast-SYNC fuzz), then smoke, the whole
# -m gpu suite and one short default bench line
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  -k "same_tick or known_answers or fast_sync" > $O/new_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1
tail -3 $O/gpu_tests.log; grep metric $O/bench.log
