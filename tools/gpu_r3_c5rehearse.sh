# round 3: bench.py --workload c5 on W ranks (slot-sharded RUMOR mode, RCCL) rehearsed on one GPU, W = 2 and 4, and
# W = 1 for comparison; then the two-process parity tests (row-sharded and slot-sharded) against the oracle
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3c5r}
mkdir -p $O
N=${2:-20000}
for W in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 2958$W bench.py --workload c5 --gpus $W --steps 5 --warmup 25 --members $N --rehearse-one-gpu > $O/bench_c5_w$W.log 2>&1 || { tail -40 $O/bench_c5_w$W.log; exit 1; }
  echo "W=$W $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c5_w$W.log)"
done
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 25 --members $N --no-cpu-baseline > $O/bench_c5_w1.log 2>&1
echo "W=1 $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c5_w1.log)"
SWIM_TEST_LOGDIR=$O/rccl timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded_rccl.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/rccl_tests.log 2>&1 || true
tail -n 3 $O/rccl_tests.log
