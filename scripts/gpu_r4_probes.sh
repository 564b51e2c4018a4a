#!/bin/bash
# Round-4 probes: the RS rotation shapes, the Clay(10,4) one-wave ring, RS(17,3) unit orders.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out
mkdir -p $O
timeout -k 10 200 ./scripts/addr_probe rot > $O/addr_rot2.jsonl 2>&1 || { echo "rot rc=$?"; exit 1; }
timeout -k 10 200 ./scripts/clay104_probe > $O/clay104_probe_r4.jsonl 2>&1 || { echo "clay104 rc=$?"; exit 1; }
timeout -k 10 400 python -u scripts/layout_sweep.py --set misaligned --cases rs173 > $O/lsweep_misaligned.jsonl 2> $O/lsweep_mis.err || { echo "sweep rc=$?"; tail -3 $O/lsweep_mis.err; exit 1; }
echo done
