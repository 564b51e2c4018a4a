#!/bin/bash
# Shader-side counters (VALU / SALU / scalar-cache / wait cycles) of the apply
# kernel on two maps: the headline Clay(4,2) repair (one tile, 20 entries) and
# the shortened Clay(10,4) repair (32 tiles, 1,280 entries).  One rocprofv3
# pass per counter set, each under its own time limit; a pass that fails on an
# unknown counter name (rc 1) is reported and skipped, anything else stops.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
SETS=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU"
  "SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES"
)
CASES="${CASES:-clay104 clay42}"
for C in $CASES; do
  if [[ $C == clay42 ]]; then
    CMD=(python3 "$ROOT/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --stripes-per-step 32768 --no-verify --no-probes)
  else
    CMD=(python3 "$ROOT/scripts/multitile_bench.py" --only "$C" --mode tiles --reps 2 --rounds 1)
  fi
  i=0
  for S in "${SETS[@]}"; do
    timeout -s KILL 120 rocprofv3 --pmc $S --output-format csv -d "$OUT/sq_${C}_$i" -o run -- "${CMD[@]}" \
        > "$OUT/sq_${C}_$i.log" 2>&1
    rc=$?; echo "sq $C set$i rc=$rc"
    case $rc in 0) ;; 1) tail -3 "$OUT/sq_${C}_$i.log" ;; *) exit $rc ;; esac
    i=$((i + 1))
  done
done
exit 0
