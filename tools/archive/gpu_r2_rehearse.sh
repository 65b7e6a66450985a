# closing rehearsal of the driver's multi-GPU bench path on one GPU: 2 and 4 ranks over RCCL (--rehearse-one-gpu)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/rehearse
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29577 bench.py --gpus 2 --steps 5 --warmup 1 --members 20000 --rehearse-one-gpu > $O/bench2.log 2>&1 || { tail -40 $O/bench2.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench2.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29578 bench.py --gpus 4 --steps 5 --warmup 1 --members 4000 --rehearse-one-gpu > $O/bench4.log 2>&1 || { tail -40 $O/bench4.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench4.log
