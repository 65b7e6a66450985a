# round 3: functional rehearsal of the driver's multi-GPU bench at W = 8 on one GPU (8 ranks, RCCL over sockets):
# C3 shape at 4 000 members, and the gossip-active sharded path (c3dyn at W = 2, exchange B every tick)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3w8}
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29598 bench.py --gpus 8 --steps 5 --warmup 1 --members 4000 --rehearse-one-gpu > $O/bench_c3_w8.log 2>&1 || { tail -30 $O/bench_c3_w8.log; exit 1; }
echo "C3 4000 W=8 $(grep -o '"ms_per_step": [0-9.]*\|"exchange_ms_per_step": [0-9.]*' $O/bench_c3_w8.log | tr '\n' ' ')"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29599 bench.py --workload c3dyn --gpus 2 --steps 5 --warmup 3 --members 20000 --rehearse-one-gpu > $O/bench_c3dyn_w2.log 2>&1 || { tail -30 $O/bench_c3dyn_w2.log; exit 1; }
echo "c3dyn 20000 W=2 $(grep -o '"ms_per_step": [0-9.]*\|"exchange_ms_per_step": [0-9.]*' $O/bench_c3dyn_w2.log | tr '\n' ' ')"
timeout -k 10 300 python -u bench.py --workload c3dyn --steps 5 --warmup 3 --members 20000 --no-cpu-baseline > $O/bench_c3dyn_w1.log 2>&1
echo "c3dyn 20000 W=1 $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c3dyn_w1.log)"
