# Copy traces of the end-to-end leg (round-5 verdict weak 8): Clay(10,4)'s 128 strided DMA runs per
# stripe against the headline's 8 -- rocprofv3 memory-copy + kernel trace (no counters), one
# bench run each with a short timed region and the e2e leg.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
for W in clay104 clay42; do
  (cd /tmp && timeout -k 10 400 rocprofv3 --memory-copy-trace --kernel-trace --stats --output-format csv \
      -d "$GRAFT_REPO_ROOT/gpurun_out/r06_e2e_trace_$W" -o run \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload $W --steps 1 --warmup 0 --cpu-seconds 0 --no-probes --e2e-seconds 1) \
      > gpurun_out/r06_e2e_trace_$W.log 2>&1; rc=$?; echo "$W rc=$rc"; tail -1 gpurun_out/r06_e2e_trace_$W.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
