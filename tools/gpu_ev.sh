cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ev
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/ev/on.log 2>&1; grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*' gpurun_out/ev/on.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-events > gpurun_out/ev/off.log 2>&1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/ev/off.log
