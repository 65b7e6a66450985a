# C4-shaped runs (partition healed at period 200, to period 320) at reduced N, to size a C4 bench line
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/c4
mkdir -p $O
timeout -k 10 300 python -u tools/exp_c4.py 2000 > $O/c4_2000.log 2>&1 || { tail -5 $O/c4_2000.log; exit 1; }
tail -4 $O/c4_2000.log
timeout -k 10 400 python -u tools/exp_c4.py 5000 > $O/c4_5000.log 2>&1 || { tail -5 $O/c4_5000.log; exit 1; }
tail -4 $O/c4_5000.log
