# iteration check after a sharded-path change: the whole -m gpu suite, the default bench line, and a 2-rank
# rehearsal of the sharded bench on the one GPU (RCCL over its socket transport; functional, not an xGMI timing)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/iter2
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1
grep metric $O/bench.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29577 bench.py --gpus 2 --steps 5 --warmup 1 --members 20000 --rehearse-one-gpu > $O/bench2.log 2>&1 || { tail -40 $O/bench2.log; exit 1; }
grep metric $O/bench2.log
