# parity incl. RUMOR mode, then the C5-shaped (rumor-only, 1 % churn) and C2 bench lines
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/rumor
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_golden.py tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 400 python -u bench.py --workload c5 --members ${C5N:-100000} --warmup 25 --steps 10 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
tail -1 $O/c5.log | cut -c1-400
timeout -k 10 400 python -u bench.py --workload c2 --warmup 12 --steps 8 --no-cpu-baseline > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
tail -1 $O/c2.log | cut -c1-300
