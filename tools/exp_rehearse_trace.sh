# Per-rank kernel traces of a row-sharded C3 rehearsal on ONE GPU (each rank under its own rocprofv3, RCCL over
# sockets): bash tools/exp_rehearse_trace.sh OUTDIR W MEMBERS [STEPS]. The ranks share the GPU, so kernel times are
# upper bounds of what one rank's kernels take on a GPU of its own; the exchange time is the socket transport's.
set -e
O=$1; W=$2; N=$3; S=${4:-5}
mkdir -p $O
export MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29600 + W)) WORLD_SIZE=$W TMPDIR=/tmp
pids=()
for r in $(seq 0 $((W - 1))); do
  RANK=$r LOCAL_RANK=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r$r -o run --output-format csv -- \
    python3 bench.py --gpus $W --members $N --steps $S --warmup 2 --rehearse-one-gpu --no-cpu-baseline > $O/r$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
grep -h metric $O/r0.log > $O/line.json || true
exit $rc
