#!/bin/bash
# RS(17,3) encodeParity: does the 200,000-B shard pitch set its rate?  Default launch and the
# two fixed workgroup sizes over a range of shard sizes, ~16 GiB of stripes each.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/rs173_pitch.jsonl"
for SH in 200000 200064 196608 204800 262144 266240 1048576 1052672 4198400; do
  timeout -k 10 120 python "$ROOT/scripts/rs173_knobs.py" --set shapes --shard $SH --gib 16 --rounds 2 --reps 4 \
      >> "$OUT/rs173_pitch.jsonl" 2> "$OUT/rs173_pitch.err" || { echo "shard $SH failed"; exit 1; }
done
cat "$OUT/rs173_pitch.jsonl"
