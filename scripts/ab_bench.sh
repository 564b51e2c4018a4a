#!/bin/bash
# Interleaved bench.py A/B over tune sets: WL=<workload> SETS="k=v,k=v;k=v" [ROUNDS=2] ab_bench.sh
# Each round runs every set once (order reversed on odd rounds); one JSON line per run.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
WL="${WL:-rs124}"
IFS=';' read -r -a S <<< "${SETS:-}"
ROUNDS="${ROUNDS:-2}"
for ((r = 0; r < ROUNDS; r++)); do
  idx=$(seq 0 $((${#S[@]} - 1)))
  [ $((r % 2)) -eq 1 ] && idx=$(seq $((${#S[@]} - 1)) -1 0)
  for i in $idx; do
    args=()
    IFS=',' read -r -a kv <<< "${S[$i]}"
    for t in "${kv[@]}"; do [ -n "$t" ] && args+=(--tune "$t"); done
    log="$OUT/ab_${WL}_${r}_$i.log"
    timeout -k 10 300 python bench.py --workload "$WL" --steps 3 --warmup 1 --cpu-seconds 0 --no-probes \
        "${args[@]}" > "$log" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc"; tail -5 "$log"; exit $rc; }
    python - "$log" "$WL" "${S[$i]}" <<'PY' | tee -a "$OUT/ab_bench.jsonl"
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(json.dumps({"workload": sys.argv[2], "tune": sys.argv[3], "value": d["value"], "frac": d["roofline"]["frac"],
                  "kernel": d["roofline"]["kernel"], "avg_launch_ms": d["roofline"]["avg_launch_ms"],
                  "verified": d["verified"]}))
PY
  done
done
