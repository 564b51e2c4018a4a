#!/bin/bash
# The LDS lookup-table kernel (k_gf_lut, ecx_tune "lds_lut") against the split-table
# kernel on the headline workload (Clay(4,2) repair, 32 KiB, 2^15 stripes resident):
#   1. one bench.py line per variant (default, lds_lut=1 log/antilog, lds_lut=2 product rows);
#   2. LDS / VALU shader counters per variant, one rocprofv3 pass each.
# Every GPU step has its own time limit; a failure stops the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
VARIANTS=("lds_lut=0" "lds_lut=1" "lds_lut=2")
for V in "${VARIANTS[@]}"; do
  timeout -k 10 300 python3 "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --tune "$V" \
      > "$OUT/lut_bench_$V.log" 2>&1
  rc=$?; echo "bench $V rc=$rc"; [ $rc -ne 0 ] && exit $rc
  tail -1 "$OUT/lut_bench_$V.log" >> "$OUT/lut_bench.jsonl"
done
SET="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES"
for V in "${VARIANTS[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d "$OUT/lut_sq_$V" -o run -- \
      python3 "$ROOT/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --stripes-per-step 32768 --no-verify \
      --no-probes --tune "$V" > "$OUT/lut_sq_$V.log" 2>&1
  rc=$?; echo "sq $V rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
