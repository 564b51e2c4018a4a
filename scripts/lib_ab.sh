#!/bin/bash
# Two library builds on the same box, interleaved A B B A per workload: A = scripts/ab/libecx_base.so
# (a build of the previous sources), B = the in-tree repair-pipelining_amd/libecx.so.  One bench line
# each (no CPU baseline, no probes); prints {workload, lib, frac, avg_launch_ms} lines.
#   WLS="clay42 rs173" ROUNDS=2 bash scripts/lib_ab.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
O=gpurun_out
mkdir -p $O
: > $O/lib_ab.jsonl
A="$ROOT/scripts/ab/libecx_base.so"
B="$ROOT/repair-pipelining_amd/libecx.so"
for W in ${WLS:-clay42 rs173}; do
  for r in $(seq 1 "${ROUNDS:-2}"); do
    for L in A B B A; do
      LIB=$A; [ $L = B ] && LIB=$B
      ECX_LIB_PATH=$LIB timeout -k 10 200 python bench.py --workload $W --steps 4 --warmup 1 --cpu-seconds 0 \
          --no-probes --no-verify > $O/ab_${W}_$L.log 2>&1 || { echo "$W $L rc=$?"; tail -3 $O/ab_${W}_$L.log; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/ab_${W}_$L.log').read().strip().splitlines()[-1]); print(json.dumps({'workload': '$W', 'lib': '$L', 'frac': d['roofline']['frac'], 'avg_launch_ms': d['roofline']['avg_launch_ms'], 'kernel': d['roofline']['kernel']}))" >> $O/lib_ab.jsonl
    done
  done
done
cat $O/lib_ab.jsonl
