cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/nt
for v in 1 0 1; do SWIM_DIFF_NT=$v timeout -k 10 300 python -u bench.py --steps 15 --warmup 2 --no-cpu-baseline > gpurun_out/nt/b$v.log 2>&1; echo "NT=$v $(grep metric gpurun_out/nt/b$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,2), 'M', round(d['ms_per_step'],3), 'ms', round(d['roofline']['avg_launch_us'],1), 'us', round(d['roofline']['frac'],3))")"; done
