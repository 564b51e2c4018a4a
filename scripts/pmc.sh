#!/bin/bash
# HBM traffic and shader counters of the bench's dominant kernel, per --workload
# (default: all four), from rocprofv3 PMC passes: FETCH_SIZE and WRITE_SIZE in passes
# of their own (they do not fit one TCC pass on gfx950), then one SQ pass (VALU
# instructions, wave/busy/wait cycles, GRBM clock).  Every pass runs the bench for one
# step of 16 launches over its resident pool (the per-layout shape selection's timed first
# calls of the RS / LRC-encode maps run before it, so the timed launches outnumber them) and writes its launch metadata (--meta: kernel instance,
# pool, algorithmic bytes, kernel-source hash) next to the counters;
# scripts/pmc_summary.py turns them into profiles/pmc_traffic.json.
# A pass that fails stops the script (no retries).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
# --candidates: instead, every launch shape the per-layout selection can keep for the many-stream
# RS / LRC-encode maps (kernels.hip kLayoutCand), each forced by its ecx_tune keys, FETCH and
# WRITE passes only; pmc_summary.py files them under the workload's by_shape profiles, keyed by
# the full launch shape (kernel instance + stagger + XCD runs) bench.py reports.
CANDIDATES=0
if [ "${1:-}" = "--candidates" ]; then CANDIDATES=1; shift; fi
if [ $CANDIDATES = 1 ]; then
  WORKLOADS="${*:-rs124 rs173 lrcenc}"
else
  WORKLOADS="${*:-clay42 clay104 rs124 lrc clay42x2 rs173 lrcenc rs173check}"
fi
# the selection's candidates (kLayoutCand order): static rules, 256-thread / 4 KiB, skewed chunks,
# one wave / 1 KiB, one wave + stagger 2, one wave + stagger 8, 256-thread + stagger 4
CAND_TUNES=("layout_select=0" "block_threads=256 skew_chunks=0" "block_threads=256 skew_chunks=4"
            "block_threads=64 skew_chunks=0" "block_threads=64 skew_chunks=0 stagger=2"
            "block_threads=64 skew_chunks=0 stagger=8" "block_threads=256 skew_chunks=0 stagger=4")
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
# Variants of a workload (bench.py profile_key): <workload>_blocked (--layout blocked),
# <workload>_pitch<P> (--pitch P, e.g. _pitchrecommended), clay104_sub<B> (--sub-bytes B).
variant_args() {
  local w=$1 base=${1%%_*} v=${1#*_}
  [ "$w" = "$base" ] && { echo "--workload $w"; return; }
  case $v in
    blocked) echo "--workload $base --layout blocked" ;;
    pitch*) echo "--workload $base --pitch ${v#pitch}" ;;
    sub*) echo "--workload $base --sub-bytes ${v#sub}" ;;
    *) echo "unknown variant $w" >&2; exit 2 ;;
  esac
}
for W in $WORKLOADS; do
  case ${W%%_*} in
    clay42|clay42x2) POOL=32768 ;; clay104) POOL=2048 ;; rs124) POOL=512 ;; rs173|rs173check) POOL=4096 ;; lrcenc) POOL=32768 ;; lrc) POOL=32768 ;;
    *) echo "unknown workload $W"; exit 2 ;;
  esac
  [ "$W" = clay104_sub1048576 ] && POOL=16  # bench.py's pool for 1 MiB sub-chunks
  if [ $CANDIDATES = 1 ]; then NC=${#CAND_TUNES[@]}; else NC=1; fi
  for ((c = 0; c < NC; c++)); do
    TUNE=(); TAG=""
    if [ $CANDIDATES = 1 ]; then
      for kv in ${CAND_TUNES[$c]}; do TUNE+=(--tune "$kv"); done
      TAG="_c$c"
      PASSES=(FETCH_SIZE WRITE_SIZE)
    else
      PASSES=(FETCH_SIZE WRITE_SIZE "$SQ")
    fi
    i=0
    for C in "${PASSES[@]}"; do
      D="$OUT/pmc_${W}${TAG}_$i"; mkdir -p "$D"
      timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$D" -o run \
          -- python3 "$ROOT/bench.py" $(variant_args "$W") --steps 1 --warmup 0 --cpu-seconds 0 --e2e-seconds 0 \
             --stripes-per-step $((POOL * 16)) --no-probes --meta "$D/meta.json" "${TUNE[@]}" > "$D.log" 2>&1
      rc=$?; echo "pmc $W$TAG pass$i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$D.log"; exit $rc; }
      i=$((i + 1))
    done
  done
done
exit 0
