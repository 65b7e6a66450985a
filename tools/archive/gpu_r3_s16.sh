# round 3: 16-bit holder entries. The long runs past the 13-bit tick window, then the whole -m gpu suite, then the
# gossip-heavy lines and the lone C5 slot shard at 10^6 members at steady state (periods 25-27)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3s16}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_long_runs.py -x -v --timeout 500 --timeout-method thread -p no:cacheprovider > $O/long.log 2>&1
tail -n 1 $O/long.log
