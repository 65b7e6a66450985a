# round 3, first GPU pass: the new parity cases (forced capacity fallbacks, COLD_JOIN member configs, small-cap
# drains, parallel user-gossip creation through the user-gossip / RUMOR cases), then the full-size C2 one-vs-two-shard
# property check and a C5-shaped line
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "fallback or tiny_caps or member_configs or drain_small or user_gossip or rumor or cold_join_inbound or contact_replay" \
  > $O/new_tests.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale_props.py -x -v --timeout 850 --timeout-method thread \
  -p no:cacheprovider > $O/scale_props.log 2>&1
timeout -k 10 400 python -u bench.py --workload c5 --steps 10 --warmup 25 --no-cpu-baseline > $O/bench_c5.log 2>&1
tail -3 $O/new_tests.log; tail -3 $O/scale_props.log; grep metric $O/bench_c5.log
# C2 gossip-send work counters (SWIM_EXP=4: window items, contact bits, replays, first-receipt candidates per step)
SWIM_EXP=4 timeout -k 10 300 python -u bench.py --workload c2 --steps 3 --warmup 14 --no-cpu-baseline > $O/c2_exp4.log 2>&1
grep -c "exp:" $O/c2_exp4.log
