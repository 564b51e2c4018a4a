#!/bin/bash
# Occupancy experiment (ecx_tune occ_lds: dummy LDS per k_gf_apply workgroup caps the
# workgroups resident per CU at floor(160 KiB / occ_lds)): interleaved bench.py A/B per workload.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
: > "$ROOT/gpurun_out/ab_bench.jsonl"
WL=rs173 SETS="occ_lds=0;occ_lds=32768;occ_lds=40960;occ_lds=53248;occ_lds=65536" ROUNDS=2 bash "$ROOT/scripts/ab_bench.sh" || exit $?
WL=rs124 SETS="occ_lds=0;occ_lds=10240;occ_lds=13653;occ_lds=20480;occ_lds=32768" ROUNDS=2 bash "$ROOT/scripts/ab_bench.sh" || exit $?
WL=lrc SETS="occ_lds=0;occ_lds=32768;occ_lds=40960;occ_lds=53248" ROUNDS=2 bash "$ROOT/scripts/ab_bench.sh" || exit $?
WL=clay42 SETS="occ_lds=0;occ_lds=65536" ROUNDS=2 bash "$ROOT/scripts/ab_bench.sh" || exit $?
