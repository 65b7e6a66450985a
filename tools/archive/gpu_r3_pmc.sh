# round 3: HBM and atomic PMC passes over the gossip plane at C2 and C5 (one counter group per pass, each its own
# run, MI355X_MICROARCH.md HBM section), then C3 timing experiments: 256 = no per-tick event / host wait (gossip
# plane never launched: C3 has no gossips), 128 / 16 = member-kernel cycles per phase (max / sum)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3pmc}
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "TCC_[A-Z0-9_]*ATOMIC[A-Z0-9_]*" $O/avail.txt | sort -u > $O/atomic_names.txt || true
K="k_gossip|k_round|k_contact|k_rx_build|k_member_tick|k_tin_scatter|k_seg_sort|k_scatter_rc|k_count_rc"
for ww in c2:12 c5:25; do
  w=${ww%%:*}
  CS="FETCH_SIZE WRITE_SIZE"
  grep -qx TCC_ATOMIC $O/atomic_names.txt && CS="$CS TCC_ATOMIC_sum"
  for c in $CS; do
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "$K" -d $O/pmc_${w}_$c -o run --output-format csv -- python3 bench.py --workload $w --steps 2 --warmup ${ww##*:} --no-cpu-baseline > $O/pmc_${w}_$c.log 2>&1
    echo "$w $c done"
  done
done
for e in 256 128 16; do
  SWIM_EXP=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t$e -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-events > $O/l$e.log 2>&1
  echo "exp=$e $(grep -h k_member_tick $O/t$e/run_kernel_stats.csv | cut -d, -f4-6)"
done
python3 tools/tick_breakdown.py $O/t256/run_kernel_trace.csv 20 | tail -3
grep -h "exp:" $O/l128.log | tail -3
grep -h "exp:" $O/l16.log | tail -3
