set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench100k.log
mkdir -p gpurun_out/prof2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof2_bench.log 2>&1
