cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-dbgsc}
mkdir -p $O
SWIM_EXP=256 timeout -k 10 200 python -u tools/dbg_scalars.py 3 55 880 > $O/k.log 2>&1
grep DBG $O/k.log | head -30; tail -n 3 $O/k.log
