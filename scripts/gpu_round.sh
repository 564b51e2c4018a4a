#!/bin/bash
# One GPU session on the MI355X box: smoke, GPU parity tests, bench, rocprofv3.
# Every GPU step has its own time limit; a fault/abort/timeout stops the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
MODE="${1:-all}"

fatal() { case "$1" in 0|1) return 1;; *) echo "step exited with $1: stopping" ; return 0;; esac; }

if [[ "$MODE" == all || "$MODE" == test ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; fatal $rc && exit $rc
  timeout -k 10 900 python -m pytest tests -m gpu -q -rf > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; tail -15 "$OUT/pytest_gpu.log"; fatal $rc && exit $rc
fi
if [[ "$MODE" == all || "$MODE" == bench ]]; then
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 --cpu-seconds 10 > "$OUT/bench.log" 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench.log"; fatal $rc && exit $rc
fi
if [[ "$MODE" == all || "$MODE" == prof ]]; then
  export TMPDIR=/tmp
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
      -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-seconds 0) > "$OUT/prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/prof.log"; fatal $rc && exit $rc
  find "$OUT/prof" -name '*stats*' | head
fi
exit 0
