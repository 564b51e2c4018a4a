# Final round-6 record on the final sources: the default bench line (the driver's command), then the
# rocprofv3 kernel statistics of a short bench run (its HIP-event average printed beside them).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r06_bench_final.json 2> gpurun_out/r06_bench_final.err || { tail -20 gpurun_out/r06_bench_final.err; exit 1; }
tail -1 gpurun_out/r06_bench_final.json | cut -c1-400
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r06_final_prof" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --e2e-seconds 0) > gpurun_out/r06_final_prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -1 gpurun_out/r06_final_prof.log | cut -c1-300; exit $rc
