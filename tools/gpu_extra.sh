# restated-scenario parity, then the C5-shaped and C2 bench lines with their CPU baselines
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/extra
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fast_config or metadata or joins" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 500 python -u bench.py --workload c5 --warmup 25 --steps 10 > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
tail -1 $O/c5.log | cut -c1-200
timeout -k 10 500 python -u bench.py --workload c2 --warmup 12 --steps 8 > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
tail -1 $O/c2.log | cut -c1-200
