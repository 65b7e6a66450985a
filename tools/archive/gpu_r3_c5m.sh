# round 3: the lone C5 slot shard of 8 at 10^6 members at steady state (periods 25-27), then the bench lines
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3c5m2}
mkdir -p $O
timeout -k 10 900 python3 -u bench.py --workload c5 --members 1000000 --rehearse-shard 8 --slots 45056 --ring 32768 --steps 3 --warmup 25 --no-cpu-baseline > $O/c5_1M_shard.log 2>&1 || { grep -v amdgpu $O/c5_1M_shard.log | tail -5; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"device_bytes": [0-9]*' $O/c5_1M_shard.log
