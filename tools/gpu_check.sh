set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/chk
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/chk/pytest.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/chk/smoke.log 2>&1
timeout -k 10 500 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/chk/bench.log 2>&1
tail -3 gpurun_out/chk/pytest.log; cat gpurun_out/chk/smoke.log; grep metric gpurun_out/chk/bench.log
