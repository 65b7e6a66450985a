# round profile: the default bench line (with the CPU baseline), its kernel-trace summary, and the HBM PMC passes
# for k_sync_diff (FETCH_SIZE and WRITE_SIZE in separate runs, MI355X_MICROARCH.md HBM/rocprofv3 section); then
# tools/make_profiles.py <tag> copies the summaries into profiles/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O

timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
grep metric $O/bench.log > $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/trace_bench.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_sync_diff" -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_sync_diff" -d $O/pmc_write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1
find $O -name "*.csv" | head -20
cat $O/bench.json
