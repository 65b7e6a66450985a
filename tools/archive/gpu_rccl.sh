set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rccl
SWIM_TEST_LOGDIR=$GRAFT_REPO_ROOT/gpurun_out/rccl timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_rccl.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/rccl/pytest.log 2>&1 || { tail -60 gpurun_out/rccl/pytest.log; exit 1; }
tail -5 gpurun_out/rccl/pytest.log
