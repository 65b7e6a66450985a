# round 3: k_sync_diff grid size at C3 with SYNC_ACK resolution (half the payloads streamed)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3grid}
mkdir -p $O
for g in 2048 1024 1536 4096; do
  SWIM_DIFF_GRID=$g timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/c3_g$g.json 2> $O/c3_g$g.err
  echo "grid $g $(grep -o '"ms_per_step": [0-9.]*\|"avg_launch_us": [0-9.]*' $O/c3_g$g.json | tr '\n' ' ')"
done
