# round 3: the sharded paths after the speculative sharded batch: the in-process / two-process parity suites, then the
# 2- and 4-rank C3 rehearsal (RCCL over sockets on one GPU) with their exchange time per step
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3sh}
mkdir -p $O
[ -n "$2" ] || SWIM_TEST_LOGDIR=$O/rccl timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_rccl.py tests/test_gpu_sharded.py tests/test_gpu_multi_device_handle.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || true
if [ -z "$2" ]; then tail -n 3 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head || true; fi
for WN in 2:20000 4:4000; do
  W=${WN%%:*}; N=${WN##*:}
  for NS in "" 1; do
    if [ -n "$NS" ]; then export SWIM_NO_SPECULATION=1; else unset SWIM_NO_SPECULATION; fi
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 2957$W bench.py --gpus $W --steps 5 --warmup 1 --members $N --rehearse-one-gpu > $O/bench_c3_w$W$NS.log 2>&1 || { tail -30 $O/bench_c3_w$W$NS.log; exit 1; }
    echo "C3 $N W=$W no_spec=$NS $(grep -o '"ms_per_step": [0-9.]*\|"exchange_ms_per_step": [0-9.]*' $O/bench_c3_w$W$NS.log | tr '\n' ' ')"
  done
done
