# parity (parity, fuzz, golden, sharded) then C2 with the gossip-send work counters (SWIM_EXP=4; exact results)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/c2x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_golden.py tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -2 $O/parity.log
SWIM_EXP=4 timeout -k 10 300 python -u tools/exp_c2.py 10000 14 > $O/exp4.log 2>&1 || { tail -20 $O/exp4.log; exit 1; }
tail -16 $O/exp4.log
