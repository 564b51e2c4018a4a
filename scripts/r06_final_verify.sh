# Round-6 final verification on the final sources: the GPU suite, the diagnostic-library tests, smoke().
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_final_gpu.log 2>&1 || { tail -30 gpurun_out/r06_final_gpu.log; exit 1; }
tail -1 gpurun_out/r06_final_gpu.log
ECX_LIB_PATH=$PWD/repair-pipelining_amd/libecx_diag.so timeout -k 10 600 python -u -m pytest tests -m "gpu and diag" -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_final_diag.log 2>&1 || { tail -30 gpurun_out/r06_final_diag.log; exit 1; }
tail -1 gpurun_out/r06_final_diag.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
