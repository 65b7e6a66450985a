# round 3: C2 timing experiments: gossip-send / replay work counters per step (SWIM_EXP=4: window items, contact-path
# bits, items that reach the contact replay, first-receipt candidates, sends the replay blocked) and the member
# kernel's largest per-member cycles per phase (SWIM_EXP=128)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3c2x}
mkdir -p $O
SWIM_EXP=4 timeout -k 10 300 python -u bench.py --workload c2 --steps 3 --warmup 12 --no-cpu-baseline > $O/c2_exp4.log 2>&1
grep "exp:" $O/c2_exp4.log | tail -3
SWIM_EXP=128 timeout -k 10 300 python -u bench.py --workload c2 --steps 3 --warmup 12 --no-cpu-baseline > $O/c2_exp128.log 2>&1
grep "exp:" $O/c2_exp128.log | tail -4
