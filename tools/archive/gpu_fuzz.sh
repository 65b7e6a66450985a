cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/fz
timeout -k 10 800 python -u -m pytest tests/test_gpu_fuzz.py tests/test_golden.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/fz/pytest.log 2>&1
grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/fz/pytest.log | grep -v PASSED | cut -c1-600 | tail -30
