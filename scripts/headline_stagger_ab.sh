#!/bin/bash
# The headline (Clay(4,2) e=1, 2^15 resident stripes) under the stagger unit order
# (ecx_tune "stagger": 0 = stripe-major default, G = G stripes interleaved at G chunk
# offsets), interleaved A B C D D C B A, one bench line each (no CPU baseline, no probes).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out
mkdir -p $O
: > $O/headline_stagger.jsonl
for G in 0 2 4 8 8 4 2 0; do
  timeout -k 10 200 python bench.py --steps 4 --warmup 1 --cpu-seconds 0 --no-probes --no-verify --tune stagger=$G \
      > $O/hs_$G.log 2>&1 || { echo "stagger $G rc=$?"; tail -3 $O/hs_$G.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/hs_$G.log').read().strip().splitlines()[-1]); print(json.dumps({'stagger': $G, 'frac': d['roofline']['frac'], 'value': d['value'], 'avg_launch_ms': d['roofline']['avg_launch_ms']}))" >> $O/headline_stagger.jsonl
done
cat $O/headline_stagger.jsonl
