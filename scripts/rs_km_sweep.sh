#!/bin/bash
# RS(k, m) encodeParity over 256 KiB shards (aligned) and 200,000-B shards, ~16 GiB of
# stripes each: how the rate depends on the map's input / output counts (is RS(17,3)'s
# rate its 17 streams, its 3 rows, or its ring padding -- 17 entries padded to 24?).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/rs_km.jsonl"
for KM in "8 3" "12 3" "16 3" "17 3" "20 3" "12 4" "16 4" "17 2" "10 2"; do
  set -- $KM
  for SH in 262144 200000; do
    timeout -k 10 120 python "$ROOT/scripts/rs173_knobs.py" --set shapes --k $1 --m $2 --shard $SH --gib 16 \
        --rounds 2 --reps 4 >> "$OUT/rs_km.jsonl" 2> "$OUT/rs_km.err" || { echo "k=$1 m=$2 shard $SH failed"; exit 1; }
  done
done
cat "$OUT/rs_km.jsonl"
