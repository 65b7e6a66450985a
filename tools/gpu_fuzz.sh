cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/fz
timeout -k 10 800 python -u -m pytest tests/test_gpu_fuzz.py tests/test_golden.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/fz/pytest.log 2>&1
grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/fz/pytest.log | cut -c1-400 | tail -30
