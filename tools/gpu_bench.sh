set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u __graft_entry__.py smoke 2>&1 | tail -3
timeout -k 10 300 python -u bench.py --members 20000 --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | tee gpurun_out/bench20k.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 2 2>&1 | tee gpurun_out/bench100k.log
