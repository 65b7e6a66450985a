# the whole -m gpu suite, then the C2 gossip-plane profile (tools/gpu_c2_profile.sh)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r2f}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
bash tools/gpu_c2_profile.sh ${1:-r2f}
