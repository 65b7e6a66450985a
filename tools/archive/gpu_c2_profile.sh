# C2 (10k members, 5 % loss) gossip-plane profile: bench line, kernel-trace summary, and separate HBM PMC passes
# (FETCH_SIZE, WRITE_SIZE) over the gossip kernels and the member kernel (MI355X_MICROARCH.md HBM/rocprofv3 section)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-c2prof}
mkdir -p $O
timeout -k 10 300 python -u bench.py --workload c2 --steps 6 --warmup 12 --no-cpu-baseline > $O/bench_c2.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench_c2.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --workload c2 --steps 3 --warmup 12 --no-cpu-baseline > $O/trace.log 2>&1
K="k_gossip_send|k_gossip_scan|k_member_tick|k_gossip_apply|k_seg_sort|k_scatter_rc|k_count_rc|k_gossip_replay"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --workload c2 --steps 1 --warmup 12 --no-cpu-baseline > $O/pmc_fetch.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/pmc_write -o run --output-format csv -- python3 bench.py --workload c2 --steps 1 --warmup 12 --no-cpu-baseline > $O/pmc_write.log 2>&1
find $O -name "*.csv" | head
