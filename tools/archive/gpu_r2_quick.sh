# round 2: a -k selection of the -m gpu suite (fast feedback on new parity cases)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r2q}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "$2" > $O/tests.log 2>&1
tail -3 $O/tests.log
