#!/bin/bash
# One GPU session on the MI355X box.  Modes (any of; run in this order): test diag pmc bench gloo2 workloads refcpu prof
# Every GPU step has its own time limit; a fault/abort/timeout stops the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
MODES="${*:-test bench}"
has() { [[ " $MODES " == *" $1 "* ]]; }
stop() { echo "step '$1' exited with $2: stopping"; exit "$2"; }

if has test; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -ne 0 ] && stop smoke $rc
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; tail -5 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && stop pytest $rc
fi
if has diag; then
  # the measured-and-rejected kernels, in the diagnostic library (make DIAG=1): the tests marked
  # `diag` and the lab variants of the mixed tests
  ECX_LIB_PATH="$ROOT/repair-pipelining_amd/libecx_diag.so" timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf \
      --timeout 120 --timeout-method thread -k "diag or bitslice or lds_lut or multitile_launch or random_maps or clay_rtc_kernel or two_slice or skew_chunks or stagger_unit or multi_unit" \
      > "$OUT/pytest_gpu_diag.log" 2>&1
  rc=$?; echo "pytest gpu diag rc=$rc"; tail -3 "$OUT/pytest_gpu_diag.log"; [ $rc -ne 0 ] && stop pytest_diag $rc
fi
if has pmc; then
  bash "$ROOT/scripts/pmc.sh" || stop pmc $?
  # refresh this copy's profiles/pmc_traffic.json, so a bench later in the same call reports
  # the traffic just measured (re-run scripts/pmc_summary.py on the merged gpurun_out/ to keep it)
  python "$ROOT/scripts/pmc_summary.py" "$OUT" "$OUT/pmc_workloads_box.json" > "$OUT/pmc_summary.log" 2>&1 \
      || stop pmc_summary $?
fi
if has bench; then
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 > "$OUT/bench.log" 2>&1
  rc=$?; echo "bench rc=$rc"; tail -2 "$OUT/bench.log"; [ $rc -ne 0 ] && stop bench $rc
fi
if has gloo2; then
  # the multi-rank path without an external launcher, 2 ranks sharing the one GPU
  ECX_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --pool 4096 --steps 2 --warmup 1 \
      --cpu-seconds 4 --no-probes > "$OUT/bench_gloo2.log" 2>&1
  rc=$?; echo "bench gloo2 rc=$rc"; tail -2 "$OUT/bench_gloo2.log"; [ $rc -ne 0 ] && stop gloo2 $rc
fi
if has workloads; then
  for W in clay104 rs124 lrc clay42x2 rs173 lrcenc rs173check; do
    timeout -k 10 300 python bench.py --workload $W --steps 3 --warmup 1 > "$OUT/bench_$W.log" 2>&1
    rc=$?; echo "bench $W rc=$rc"; tail -1 "$OUT/bench_$W.log"; [ $rc -ne 0 ] && stop "bench $W" $rc
  done
fi
if has refcpu; then
  # the headline line with BASELINE.md section 4's CPU protocol (2 warm-ups + 10 x 2 s)
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 --cpu-protocol reference > "$OUT/bench_refcpu.log" 2>&1
  rc=$?; echo "bench refcpu rc=$rc"; tail -1 "$OUT/bench_refcpu.log"; [ $rc -ne 0 ] && stop "bench refcpu" $rc
fi
if has prof; then
  export TMPDIR=/tmp
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
      -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-seconds 0 --e2e-seconds 0) > "$OUT/prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -2 "$OUT/prof.log"; [ $rc -ne 0 ] && stop prof $rc
  find "$OUT/prof" -name '*stats*'
fi
exit 0
