#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the Clay(10,4) repair kernel under each block order
# (one workgroup per tile vs tile groups), one counter per rocprofv3 pass.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for X in tiles waves; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc104_x${X}_$C" -o run \
        -- python3 "$ROOT/scripts/multitile_bench.py" --only clay104 --mode $X --reps 2 --rounds 1 \
        > "$OUT/pmc104_x${X}_$C.log" 2>&1
    rc=$?; echo "pmc x$X $C rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
