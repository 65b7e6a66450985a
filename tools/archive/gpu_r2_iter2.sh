# iteration: the whole -m gpu suite, the C2 line, and a C2 kernel-trace summary
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r2iter}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${2:+-k "$2"} > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --workload c2 --steps 6 --warmup 12 --no-cpu-baseline > $O/bench_c2.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench_c2.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --workload c2 --steps 3 --warmup 12 --no-cpu-baseline > $O/trace.log 2>&1
python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/trace/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:10]:
    print(f"{r['Name'][:34]:36s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:10.1f} us {r['Percentage'][:5]}")
PY
