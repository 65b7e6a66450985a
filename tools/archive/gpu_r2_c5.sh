# RUMOR at-scale paths: parity tests, then a short C5 slot-shard rehearsal at 10^6 members (rank 0 of 8 alone)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r2c5}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "rumor or golden or c5_shard or multi_device" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u bench.py --workload c5 --members 1000000 --rehearse-shard 8 --slots 40000 --warmup ${2:-3} --steps ${3:-2} --no-cpu-baseline > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"device_bytes": [0-9]*\|"counters": {[^}]*}' $O/c5.log
