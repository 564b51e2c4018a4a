#!/bin/bash
# The end-to-end leg (bench.py e2e: pinned host -> H2D -> kernel -> D2H, host_pipe.cpp) of the
# headline over the host pipe's deployment knobs: chunk bytes per H2D (host_chunk_kib) and
# device buffer sets in the ring (host_buffers).  One JSON line per run into gpurun_out/e2e_sweep.jsonl.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
W=${1:-clay42}
for CH in 16384 65536 262144; do
  for NB in 2 3 4; do
    L="$OUT/e2e_${W}_${CH}_${NB}.log"
    timeout -k 10 200 python bench.py --workload $W --steps 1 --warmup 0 --cpu-seconds 0 --no-probes --e2e-seconds 3 \
        --tune host_chunk_kib=$CH --tune host_buffers=$NB > "$L" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench $W $CH $NB rc=$rc"; tail -3 "$L"; exit $rc; }
    python -c "
import json
l=json.loads(open('$L').read().strip().splitlines()[-1]); e=l['e2e']
print(json.dumps({'workload':'$W','host_chunk_kib':$CH,'host_buffers':$NB,'GiBps':e['GiBps'],'h2d_GBps':e['h2d_GBps'],'d2h_GBps':e['d2h_GBps'],'verified':e['verified']}))" | tee -a "$OUT/e2e_sweep.jsonl"
  done
done
