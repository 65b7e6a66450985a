# 4-rank rehearsal of the sharded bench on the one GPU (RCCL over its socket transport; functional, not xGMI timing)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/reh4
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29577 bench.py --gpus 4 --steps 5 --warmup 1 --members 4000 --rehearse-one-gpu > $O/bench4.log 2>&1 || { tail -40 $O/bench4.log; exit 1; }
grep metric $O/bench4.log
