#!/bin/bash
# Interleaved same-box A/B of the Clay(10,4) line: the round-4 HEAD
# (352308b), the round-5 HEAD (633630c) and the round-5 HEAD with the launch registry
# (note_device_launch) short-circuited, each its own tree under ab_trees/ (made by
# `git archive`, built in place).  REPS rounds of r4, r5, r5nn.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/clay104_ab"
mkdir -p "$OUT"
REPS="${REPS:-3}"
for rep in $(seq 1 "$REPS"); do
  for v in r4 r5 r5nn; do
    extra=""
    [ "$v" != r4 ] && extra="--e2e-seconds 0"
    (cd "$ROOT/ab_trees/$v" && timeout -k 10 300 python bench.py --workload clay104 --steps 8 --warmup 2 \
        --cpu-seconds 0 --no-probes $extra) > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err"
    rc=$?
    echo "$v rep $rep rc=$rc $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline']['kernel'])" "$OUT/${v}_$rep.json" 2>/dev/null)"
    [ $rc -ne 0 ] && { tail -5 "$OUT/${v}_$rep.err"; exit $rc; }
  done
done
exit 0
