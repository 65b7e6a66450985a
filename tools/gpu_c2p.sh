# C2 kernel breakdown: a short run under rocprofv3 kernel trace
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/c2p
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/exp_c2.py ${C2N:-10000} ${C2P:-6} > $O/prof_c2.log 2>&1 || { tail -30 $O/prof_c2.log; exit 1; }
grep period $O/prof_c2.log
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
head -25 $O/kernel_stats.csv | cut -c1-160
