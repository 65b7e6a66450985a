# round 2 (session 3): C2 gossip-plane profile (tools/gpu_c2_profile.sh), member-kernel phase cycles at C2 and C3
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r2p2}
mkdir -p $O
bash tools/gpu_c2_profile.sh ${1:-r2p2}
SWIM_EXP=16 timeout -k 10 300 python -u bench.py --workload c2 --steps 3 --warmup 12 --no-cpu-baseline > $O/phases_c2.log 2>&1
SWIM_EXP=16 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/phases_c3.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c3 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/trace_c3.log 2>&1
grep "exp:" $O/phases_c2.log $O/phases_c3.log | tail -8
