set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/rs_layout_contract.py > gpurun_out/r06_rs_layout_contract.jsonl 2> gpurun_out/r06_rs_layout_contract.err; rc=$?; echo "layout rc=$rc"; cat gpurun_out/r06_rs_layout_contract.jsonl | cut -c1-200; [ $rc -ne 0 ] && { tail -5 gpurun_out/r06_rs_layout_contract.err; exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/r06_pytest_gpu_first.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r06_pytest_gpu_first.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --workload clay104 --sub-bytes 1048576 > gpurun_out/r06_clay104_1mib.json 2> gpurun_out/r06_clay104_1mib.err; rc=$?; echo "clay104 1MiB rc=$rc"; tail -c 1500 gpurun_out/r06_clay104_1mib.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/r06_clay104_1mib.err; exit $rc; }
exit 0
