#!/bin/bash
# A/B of ecx_tune "units" (k_gf_apply_multi: several (stripe, chunk) units per workgroup, one load
# ring across them) on the single-tile workloads, interleaved 1 2 4 4 2 1, one bench line each (no
# probes, no CPU baseline, no e2e leg); one JSON summary line per run into gpurun_out/units_ab.jsonl.
# The kernel lives in the diagnostic library (make DIAG=1): run with ECX_LIB_PATH=.../libecx_diag.so.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
for W in ${*:-clay42 rs173 rs124 lrcenc lrc}; do
  for U in 1 2 4 4 2 1; do
    timeout -k 10 200 python bench.py --workload $W --steps 5 --warmup 2 --no-probes --cpu-seconds 0 --e2e-seconds 0 \
        --tune units=$U --tune layout_select=0 > "$OUT/units_ab_${W}_$U.log" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench $W units=$U rc=$rc"; tail -3 "$OUT/units_ab_${W}_$U.log"; exit $rc; }
    python -c "
import json
l=json.loads(open('$OUT/units_ab_${W}_$U.log').read().strip().splitlines()[-1])
print(json.dumps({'workload':'$W','units':$U,'frac':l['roofline']['frac'],'avg_launch_ms':l['roofline']['avg_launch_ms'],'shape':l['roofline']['launch_shape'].get('name'),'verified':l['verified']}))" | tee -a "$OUT/units_ab.jsonl"
  done
done
