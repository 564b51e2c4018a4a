#!/bin/bash
# A/B of ecx_tune "pad_first" (padding loads re-read the tile's first input vs the shared zero page)
# on the workloads whose tiles are padded (rs173: 17 -> 24 entries, rs124 / lrcenc: 12 -> 16, lrc:
# 3 -> 4), interleaved A B B A, one bench line each (no probes, no CPU baseline, no e2e leg).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
for W in ${*:-rs173 rs124 lrcenc lrc}; do
  for P in 1 0 0 1; do
    timeout -k 10 200 python bench.py --workload $W --steps 5 --warmup 2 --no-probes --cpu-seconds 0 --e2e-seconds 0 \
        --tune pad_first=$P > "$OUT/pad_ab_${W}_$P.log" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench $W pad_first=$P rc=$rc"; tail -3 "$OUT/pad_ab_${W}_$P.log"; exit $rc; }
    python -c "
import json,sys
l=json.loads(open('$OUT/pad_ab_${W}_$P.log').read().strip().splitlines()[-1])
print(json.dumps({'workload':'$W','pad_first':$P,'frac':l['roofline']['frac'],'avg_launch_ms':l['roofline']['avg_launch_ms'],'shape':l['roofline']['launch_shape'].get('name')}))" | tee -a "$OUT/pad_ab.jsonl"
  done
done
