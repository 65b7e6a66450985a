# round 3: speculative batches (no host wait per tick while the gossip plane is idle). A -m gpu selection, the C3
# line, its kernel trace and per-tick gaps, and the per-wave wall clock of the member kernel (SWIM_EXP=512)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3s}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${2:-c1 or golden or parity or partition or join or leave or metadata or user_gossip or dyn}" > $O/tests.log 2>&1
tail -n 1 $O/tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/t_c3 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-events > $O/b_c3.log 2>&1
python3 tools/tick_breakdown.py $O/t_c3/run_kernel_trace.csv 20 | tail -3
SWIM_EXP=512 timeout -k 10 300 python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-events > $O/l512.log 2>&1
grep -h "exp512" $O/l512.log | tail -9
