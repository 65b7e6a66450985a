set -e
cd $GRAFT_REPO_ROOT
rocm-smi --showproductname 2>&1 | head -5 || true
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider 2>&1 | tee gpurun_out/parity1.log
