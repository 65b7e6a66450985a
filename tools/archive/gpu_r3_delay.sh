# round 3: link delays and emulator counters (tests/test_gpu_delay.py), then a regression selection of -m gpu
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3d}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_delay.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/delay.log 2>&1 || true
tail -n 25 $O/delay.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${2:-parity or golden or c1 or fallback or user_gossip}" --deselect tests/test_gpu_delay.py > $O/tests.log 2>&1
tail -n 1 $O/tests.log
