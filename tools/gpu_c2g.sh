# C2 send-group tuning: steady-state ms/period per SWIM_SEND_GROUP, then a kernel-trace summary at the default
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/c2g
mkdir -p $O
for g in 1 4; do
  SWIM_SEND_GROUP=$g timeout -k 10 300 python -u tools/exp_c2.py 10000 13 > $O/g$g.log 2>&1 || { tail -20 $O/g$g.log; exit 1; }
  echo "group $g: $(tail -1 $O/g$g.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/exp_c2.py 10000 12 > $O/prof_c2.log 2>&1
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
head -12 $O/kernel_stats.csv | cut -c1-140
