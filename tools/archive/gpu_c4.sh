# C4-shaped runs at reduced N (partition healed at period 200, run to period 320): wall time per 10 periods and the
# storm counters; each size under its own time limit
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-c4}
mkdir -p $O
for n in ${2:-1000 2000}; do
  timeout -k 10 ${3:-400} python -u tools/exp_c4.py $n > $O/c4_$n.log 2>&1
  echo "N=$n rc=$?"; tail -3 $O/c4_$n.log
done
