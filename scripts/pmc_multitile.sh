#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of a multi-tile map's apply kernel under each launch shape
# of scripts/multitile_bench.py, one counter per rocprofv3 pass; summarised by
# scripts/pmc_cases.py.
#   scripts/pmc_multitile.sh [case (default clay104)] [modes (default "tiles waves")]
set -u
CASE="${1:-clay104}"
MODES="${2:-tiles waves}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for X in $MODES; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmcmt_${CASE}_${X}_$C" -o run \
        -- python3 "$ROOT/scripts/multitile_bench.py" --only "$CASE" --mode $X --reps 2 --rounds 1 \
        > "$OUT/pmcmt_${CASE}_${X}_$C.log" 2>&1
    rc=$?; echo "pmc $CASE $X $C rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
