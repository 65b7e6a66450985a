# C2 (10k members, 5 % loss, full views) on one GPU: parity spot check, throughput and kernel-trace summary
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/c2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_golden.py tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 400 python -u tools/exp_c2.py ${C2N:-10000} ${C2P:-25} > $O/c2.log 2>&1 || { tail -30 $O/c2.log; exit 1; }
cat $O/c2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/exp_c2.py ${C2N:-10000} 14 > $O/prof_c2.log 2>&1
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
head -25 $O/kernel_stats.csv | cut -c1-160
