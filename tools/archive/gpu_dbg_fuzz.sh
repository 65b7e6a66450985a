# fuzz seed 204 (fast SYNC) under the engine's debugging switches: which mechanism makes the chunked run diverge
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-dbgfuzz}
mkdir -p $O
run() { echo "== $1"; timeout -k 10 200 python -u tools/dbg_fuzz.py 204 fast; }
run default > $O/a.log 2>&1
SWIM_NO_PIPELINE=1 run nopipe > $O/b.log 2>&1
SWIM_NO_GOSSIP_SKIP=1 run noskip > $O/c.log 2>&1
SWIM_EXP=8 run nofilter > $O/d.log 2>&1
cat $O/[abcd].log | cut -c1-600
