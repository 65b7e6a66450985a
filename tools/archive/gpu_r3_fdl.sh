# round 3: batched FD-list inserts (fd_flush): parity cases with many ADDED events, then the C3 line and the C4
# schedule at 4 000 and 8 000 members (the heal re-adds half the cluster at every member)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3fdl}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "c1 or golden or join or partition or fuzz or leave or delay or cold or member_config or fallback" > $O/tests.log 2>&1
tail -n 1 $O/tests.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c3.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench_c3.log
for n in 4000 8000; do
  C4_RING=$([ $n = 8000 ] && echo 2097152 || echo 0) C4_CHUNK=1 timeout -k 10 400 python -u tools/exp_c4.py $n 200 320 > $O/c4_$n.log 2>&1 || { tail -5 $O/c4_$n.log; exit 1; }
  tail -1 $O/c4_$n.log
done
