# round 3: the whole -m gpu suite (no -x: every failure listed) and smoke
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3suite}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider ${2:-} > $O/tests.log 2>&1 || true
tail -n 1 $O/tests.log
grep -E "^FAILED|^ERROR" $O/tests.log | head -30 || true
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
