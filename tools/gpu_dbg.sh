cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for s in c1 c2_small c4_small c3_small; do timeout -k 10 300 python -u tools/dbg_golden.py $s 2>&1 | tail -1; done
