# C2 gossip-plane profile of the current engine, the new accounting test, and the one-off 100k CPU baseline
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r2j}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  -k "sampled_diff" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_c2_profile.sh ${1:-r2j}/c2
timeout -k 10 900 python -u tools/cpu_baseline_full.py 100000 2 $O/cpu_baseline_full.json > $O/cpu_full.log 2>&1
tail -3 $O/cpu_full.log
