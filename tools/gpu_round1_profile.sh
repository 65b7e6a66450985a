set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r1
timeout -k 10 600 python -u bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r1/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r1/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline > gpurun_out/r1/trace_bench.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_sync_diff" -d gpurun_out/r1/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r1/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_sync_diff" -d gpurun_out/r1/pmc_write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r1/pmc_write.log 2>&1
ls -R gpurun_out/r1 | head -30
