set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
rm -rf gpurun_out/pmc_* 
bash scripts/pmc.sh clay42 clay104 rs124 lrc clay42x2 rs173 lrcenc rs173check || exit $?
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r06_prof" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --e2e-seconds 0) > gpurun_out/r06_prof.log 2>&1; rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/r06_prof.log; exit $rc
