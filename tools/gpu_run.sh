# The one GPU runner (run through gpurun from the repository root): each argument is a step, run in order under its
# own time limit; the first failing step ends the call (no GPU step runs after a fault, abort or time limit).
#   suite[:EXPR]      -m gpu tests (optionally -k EXPR), log in $O/tests.log
#   smoke             __graft_entry__.smoke()
#   bench:W[:S[:WU]]  bench.py --workload W (c3 | c3dyn | c2 | c5), S steps, WU warm-up, no CPU baseline
#   benchcpu          the default bench line with its CPU baseline (the driver's command)
#   benchc:W[:S[:WU]] bench.py --workload W with its CPU baseline leg
#   trace:W[:S[:WU]]  rocprofv3 kernel trace + stats of the same bench command, and its per-tick breakdown
#   pmc:W:COUNTER[:S] one rocprofv3 --pmc pass (one counter) over a bench run of workload W with S steps (default 3)
#   pmcg:W[:S[:WU]]   the gossip plane's HBM bytes and L2 atomics per kernel and tick: FETCH_SIZE, WRITE_SIZE and
#                     TCC_ATOMIC_sum passes + a SWIM_EXP=4 work-unit run of the same command (tools/pmc_gossip.py);
#                     run a trace:W step with the same S / WU first for the kernel times
#   rehearse:R:N[:W]  bench.py --gpus R on this one GPU (R ranks over RCCL sockets), N members, workload W (default c3)
#   c4:N              the C4 schedule at N members (tools/exp_c4.py: partition, unblockAll at period 200, run to 320)
#   tapes             record the oracle tapes of the @pytest.mark.tape tests into $O/tapes
#   golden:NAME[:P[:T]] record box-sized golden NAME (P periods at most, T seconds) into $O/golden
#   c5m               rank 0 of 8 C5 slot shards at 10^6 members alone (bench.py --rehearse-shard 8), default caps
# Example:  gpurun --timeout 1200 -- 'bash tools/gpu_run.sh r4a suite:fullsize smoke bench:c3'
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for step in "$@"; do
  IFS=: read -r what a b c <<< "$step"
  echo "== $step $(date +%T)"
  case $what in
    suite)
      k=()
      [ -n "$a" ] && k=(-k "$a")
      rc=0
      timeout -k 10 1100 python -u -m pytest tests -m gpu -v --durations=${DURATIONS:-25} --timeout 600 --timeout-method thread -p no:cacheprovider \
        "${k[@]}" > $O/tests.log 2>&1 || rc=$?
      tail -n 1 $O/tests.log
      grep -E "^FAILED|^ERROR" $O/tests.log | head -30 || true
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc  # 1 = test failures (listed above); anything else ends the call
      ;;
    tapes)
      # record the oracle tapes of the @pytest.mark.tape tests (tests/tape.py): the tests run against the live oracle
      rc=0
      SWIM_ORACLE_TAPE=record SWIM_TAPE_OUT=$O/tapes timeout -k 10 1000 python -u -m pytest tests -m "gpu and tape" -v \
        --durations=0 --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tapes.log 2>&1 || rc=$?
      tail -n 1 $O/tapes.log
      grep -E "^FAILED|^ERROR" $O/tapes.log | head -30 || true
      [ $rc -eq 0 ] || exit $rc
      ;;
    golden)
      # a box-sized golden fixture from the oracle on this host (tools/record_golden_box.py); b = max periods
      rc=0
      timeout -k 10 ${c:-1000} python3 -u tools/record_golden_box.py $a ${b:+--max-periods $b} --out $O/golden \
        > $O/golden_$a.log 2>&1 || rc=$?
      tail -n 3 $O/golden_$a.log
      [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc  # 3: the memory guard stopped it (finished periods are saved)
      ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      tail -1 $O/smoke.log
      ;;
    bench)
      timeout -k 10 400 python -u bench.py --workload $a --steps ${b:-20} --warmup ${c:-3} --no-cpu-baseline \
        > $O/bench_$a.log 2>&1
      grep metric $O/bench_$a.log > $O/bench_$a.json
      grep -o '"ms_per_step": [0-9.]*' $O/bench_$a.json
      ;;
    benchc)
      # a secondary line (c3dyn / c2 / c5) with its CPU baseline leg
      timeout -k 10 900 python -u bench.py --workload $a --steps ${b:-20} --warmup ${c:-3} > $O/benchc_$a.log 2>&1
      grep metric $O/benchc_$a.log > $O/benchc_$a.json
      grep -o '"ms_per_step": [0-9.]*\|"cpu_baseline": {"value": [0-9.e+]*' $O/benchc_$a.json
      ;;
    benchcpu)
      timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
      grep metric $O/bench.log > $O/bench.json
      grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*' $O/bench.json
      ;;
    exp512)
      # per-wave wall-clock trace of the member kernel (SWIM_EXP=512, a timing experiment: not a result)
      SWIM_EXP=512 timeout -k 10 300 python3 bench.py --workload ${a:-c3} --steps 2 --warmup 3 --no-cpu-baseline \
        > $O/exp512_${a:-c3}.log 2>&1
      grep "exp512" $O/exp512_${a:-c3}.log | tail -14
      ;;
    trace)
      [ -n "$TRACE_ENV" ] && export $TRACE_ENV
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/t_$a -o run --output-format csv -- \
        python3 bench.py --workload $a --steps ${b:-5} --warmup ${c:-3} --no-cpu-baseline > $O/trace_$a.log 2>&1
      python3 tools/tick_breakdown.py $O/t_$a/run_kernel_trace.csv 10 | tail -3
      ;;
    pmc)
      timeout -s KILL 300 rocprofv3 --pmc $b -d $O/pmc_${a}_${b}_${c:-3} -o run --output-format csv -- \
        python3 bench.py --workload $a --steps ${c:-3} --warmup 1 --no-cpu-baseline > $O/pmc_${a}_${b}_${c:-3}.log 2>&1
      ;;
    pmcg)
      for ctr in FETCH_SIZE WRITE_SIZE TCC_ATOMIC_sum; do
        timeout -s KILL 300 rocprofv3 --pmc $ctr -d $O/pmc_${a}_$ctr -o run --output-format csv -- \
          python3 bench.py --workload $a --steps ${b:-2} --warmup ${c:-12} --no-cpu-baseline > $O/pmc_${a}_$ctr.log 2>&1
      done
      SWIM_EXP=4 timeout -k 10 300 python3 bench.py --workload $a --steps ${b:-2} --warmup ${c:-12} --no-cpu-baseline \
        > $O/exp4_$a.log 2>&1
      python3 tools/pmc_gossip.py $O $a $((${b:-2} * 10)) $O/pmc_gossip_$a.json > /dev/null
      python3 -c "import json; d = json.load(open('$O/pmc_gossip_$a.json')); print({k: d.get(k) for k in ('gossip_plane_hbm_bytes_per_tick', 'algorithmic_bytes_per_tick', 'wasted_traffic_ratio')})"
      ;;
    rehearse)
      timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $a --master-addr 127.0.0.1 \
        --master-port $((29500 + a)) bench.py --workload ${c:-c3} --gpus $a --steps 5 --warmup 2 --members $b \
        --rehearse-one-gpu > $O/rehearse_${c:-c3}_w${a}_$b.log 2>&1
      grep metric $O/rehearse_${c:-c3}_w${a}_$b.log > $O/rehearse_${c:-c3}_w${a}_$b.json
      grep -o '"ms_per_step": [0-9.]*\|"exchange_ms_per_step": [0-9.]*\|"diff_msgs_total": [0-9]*\|"ack_resolved_total": [0-9]*\|"sync_merges": [0-9]*' \
        $O/rehearse_${c:-c3}_w${a}_$b.json | tr '\n' ' '; echo
      ;;
    c4)
      timeout -k 10 900 python3 -u tools/exp_c4.py $a 200 320 > $O/c4_$a.log 2>&1 || { tail -3 $O/c4_$a.log; exit 1; }
      tail -2 $O/c4_$a.log
      ;;
    c4s)
      # the C4 partition phase at a members, one line per period to period b, with sampled SUSPECT coverage (exit 2: a
      # capacity or allocation error ended it, reported in the log)
      rc=0
      C4_CHUNK=1 C4_SUSPECT=1 timeout -k 10 ${c:-900} python3 -u tools/exp_c4.py $a 200 $b > $O/c4s_$a.log 2>&1 || rc=$?
      tail -n 4 $O/c4s_$a.log
      [ $rc -eq 0 ] || [ $rc -eq 2 ] || exit $rc
      ;;
    c5m)
      timeout -k 10 900 python3 -u bench.py --workload c5 --members 1000000 --rehearse-shard 8 --steps 3 --warmup 25 \
        --no-cpu-baseline > $O/c5_1M_shard.log 2>&1 || { grep -v amdgpu $O/c5_1M_shard.log | tail -5; exit 1; }
      grep metric $O/c5_1M_shard.log > $O/c5_1M_shard.json
      grep -o '"ms_per_step": [0-9.]*\|"device_bytes": [0-9]*' $O/c5_1M_shard.json | tr '\n' ' '; echo
      ;;
    *)
      echo "unknown step $step"
      exit 2
      ;;
  esac
done
echo "== done $(date +%T)"
