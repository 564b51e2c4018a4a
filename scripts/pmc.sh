#!/bin/bash
# HBM traffic of the headline kernel from rocprofv3 PMC counters, one counter
# per pass (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o run \
      -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --stripes-per-step 32768 --no-verify --no-probes \
      > "$OUT/pmc_$C.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
find "$OUT" -path '*pmc_*' -name '*.csv' | head
exit 0
