#!/bin/bash
# bench.py on every workload (1 GPU), then a 2-rank rehearsal of the multi-process
# path on the one GPU (gloo transport; ranks share the device).  Each GPU step has
# its own time limit; anything but success stops the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
for W in clay104 rs124 lrc clay42; do
  timeout -k 10 300 python bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 5 > "$OUT/bench_$W.log" 2>&1
  rc=$?; echo "bench $W rc=$rc"; tail -1 "$OUT/bench_$W.log" | cut -c1-300; [ $rc -ne 0 ] && exit $rc
done
ECX_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --pool 4096 \
    --stripes-per-step 8192 --no-probes > "$OUT/bench_2rank.log" 2>&1
rc=$?; echo "bench 2-rank rc=$rc"; grep '^{' "$OUT/bench_2rank.log" | cut -c1-300
exit $rc
