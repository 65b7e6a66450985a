set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/shard
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/shard/pytest_shard.log 2>&1 || { tail -40 gpurun_out/shard/pytest_shard.log; exit 1; }
tail -15 gpurun_out/shard/pytest_shard.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/shard/pytest_parity.log 2>&1 || { tail -40 gpurun_out/shard/pytest_parity.log; exit 1; }
tail -3 gpurun_out/shard/pytest_parity.log
