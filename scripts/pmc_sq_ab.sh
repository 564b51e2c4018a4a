#!/bin/bash
# Shader counters of the bench's kernel for one workload under two tunings (A/B),
# one rocprofv3 pass per counter set.  Usage: WL=clay104 A="bitslice=0" B="bitslice=1" pmc_sq_ab.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
WL="${WL:-clay104}"
case $WL in clay42) POOL=32768 ;; clay104) POOL=2048 ;; rs124) POOL=512 ;; lrc) POOL=32768 ;; esac
SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
      "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
      "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS")
for TAG in A B; do
  TUNE="${!TAG}"
  i=0
  for S in "${SETS[@]}"; do
    D="$OUT/sqab_${WL}_${TAG}_$i"; mkdir -p "$D"
    timeout -s KILL 240 rocprofv3 --pmc $S --output-format csv -d "$D" -o run \
        -- python3 "$ROOT/bench.py" --workload "$WL" --steps 1 --warmup 0 --cpu-seconds 0 \
           --stripes-per-step "$POOL" --no-probes --tune "$TUNE" --meta "$D/meta.json" > "$D.log" 2>&1
    rc=$?; echo "sq $WL $TAG set$i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$D.log"; exit $rc; }
    i=$((i + 1))
  done
done
exit 0
