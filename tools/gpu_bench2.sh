set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/b2
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29577 bench.py --gpus 2 --steps 3 --warmup 1 --members 20000 --rehearse-one-gpu > gpurun_out/b2/bench2.log 2>&1 || { tail -40 gpurun_out/b2/bench2.log; exit 1; }
grep metric gpurun_out/b2/bench2.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --members 20000 --no-cpu-baseline > gpurun_out/b2/bench1.log 2>&1
grep metric gpurun_out/b2/bench1.log
