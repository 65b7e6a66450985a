# round 3, final gossip-plane evidence: for C2 and C5-shape, a kernel trace, the SWIM_EXP=4 work units and three PMC
# passes (FETCH_SIZE, WRITE_SIZE, TCC_ATOMIC_sum; one counter group per run, MI355X_MICROARCH.md HBM section) of the same
# deterministic command; then the lone C5 slot shard of 8 at 10^6 members
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3pmc2}
mkdir -p $O
K="k_gossip|k_round|k_contact|k_rx_build|k_member_tick|k_tin_scatter|k_seg_sort|k_scatter_rc|k_count_rc"
for ww in c2:12 c5:25; do
  w=${ww%%:*}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 2 --warmup ${ww##*:} --no-cpu-baseline > $O/trace_$w.log 2>&1
  SWIM_EXP=4 timeout -k 10 300 python3 bench.py --workload $w --steps 2 --warmup ${ww##*:} --no-cpu-baseline > $O/exp4_$w.log 2>&1
  for c in FETCH_SIZE WRITE_SIZE TCC_ATOMIC_sum; do
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "$K" -d $O/pmc_${w}_$c -o run --output-format csv -- python3 bench.py --workload $w --steps 2 --warmup ${ww##*:} --no-cpu-baseline > $O/pmc_${w}_$c.log 2>&1
    echo "$w $c done"
  done
done
# (the lone 10^6-member C5 shard is measured by tools/gpu_r3_c5m.sh)
