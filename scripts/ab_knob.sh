#!/bin/bash
# A/B of one ecx_tune knob (KNOB, default bitslice) per workload, interleaved A B B A.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
WL="${WL:-clay104}"
EXTRA="${EXTRA:-}"
for W in $WL; do
  for V in ${VALS:-0 1 1 0}; do
    timeout -k 10 300 python bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 --no-probes \
        --tune ${KNOB:-bitslice}=$V $EXTRA > "$OUT/ab_${W}_$V.log" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc"; tail -5 "$OUT/ab_${W}_$V.log"; exit $rc; }
    python - "$OUT/ab_${W}_$V.log" "$W" "$V" "${KNOB:-bitslice}" <<'PY' | tee -a "$OUT/ab_knob.jsonl"
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print(json.dumps({"workload": sys.argv[2], "knob": sys.argv[4], "value_set": int(sys.argv[3]), "value": d["value"],
                  "frac": d["roofline"]["frac"], "kernel": d["roofline"]["kernel"],
                  "avg_launch_ms": d["roofline"]["avg_launch_ms"], "verified": d["verified"]}))
PY
  done
done
