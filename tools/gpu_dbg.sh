cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/dbg
timeout -k 10 400 python -u tools/dbg_poison.py 125 > gpurun_out/dbg/poison.log 2>&1; tail -3 gpurun_out/dbg/poison.log
echo "== parity file poison"; SWIM_POISON=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | grep -E "passed|failed|Error" | cut -c1-700
