#!/bin/bash
# Interleaved A/B of one ecx_tune key on the bench workloads: tune_ab.sh KEY "A B" [workload...].
# Values run A B B A A B per workload, one bench line each (no probes, no CPU baseline, no e2e leg,
# layout selection off so both arms run the static shape unless EXTRA_TUNE says otherwise); one
# JSON summary line per run into gpurun_out/tune_ab_KEY.jsonl.  Diagnostic keys need the
# diagnostic library: ECX_LIB_PATH=repair-pipelining_amd/libecx_diag.so ECX_DIAGNOSTIC=1.
set -u
KEY=$1; read -r A B <<< "$2"; shift 2
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
EXTRA=(--tune layout_select=0)
for kv in ${EXTRA_TUNE:-}; do EXTRA+=(--tune "$kv"); done
for W in ${*:-clay42 rs173 lrcenc}; do
  i=0
  for V in $A $B $B $A $A $B; do
    L="$OUT/tune_ab_${KEY}_${W}_${i}.log"
    timeout -k 10 200 python bench.py --workload $W --steps 5 --warmup 2 --no-probes --cpu-seconds 0 --e2e-seconds 0 \
        --tune "$KEY=$V" "${EXTRA[@]}" > "$L" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench $W $KEY=$V rc=$rc"; tail -3 "$L"; exit $rc; }
    python -c "
import json
l=json.loads(open('$L').read().strip().splitlines()[-1])
print(json.dumps({'workload':'$W','$KEY':$V,'frac':l['roofline']['frac'],'avg_launch_ms':l['roofline']['avg_launch_ms'],'shape':l['roofline']['launch_shape'].get('name'),'verified':l['verified']}))" | tee -a "$OUT/tune_ab_${KEY}.jsonl"
    i=$((i + 1))
  done
done
