# round 3: bench.py --workload c5 on W ranks (slot-sharded RUMOR mode, RCCL) rehearsed on one GPU, W = 2 and 4, and
# W = 1 for comparison
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3c5r}
mkdir -p $O
# (the ranks share the one GPU's HBM: 4 ranks at 8 000 members)
for WN in 2:20000 4:8000; do
  W=${WN%%:*}; N=${WN##*:}
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 2958$W bench.py --workload c5 --gpus $W --steps 5 --warmup 25 --members $N --rehearse-one-gpu > $O/bench_c5_w$W.log 2>&1 || { tail -40 $O/bench_c5_w$W.log; exit 1; }
  echo "N=$N W=$W $(grep -o '"ms_per_step": [0-9.]*\|"exchange_ms_per_step": [0-9.]*' $O/bench_c5_w$W.log | tr '\n' ' ')"
  timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 25 --members $N --no-cpu-baseline > $O/bench_c5_w1_$N.log 2>&1
  echo "N=$N W=1 $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c5_w1_$N.log)"
done
