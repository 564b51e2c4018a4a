set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
line() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['unit'], r['frac'], r['kernel'], (d.get('e2e') or {}).get('GiBps'))" "$1"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "clay104 or layout_selection or is_parity_correct_batch or blocked" > gpurun_out/r06_pytest_gpu_sel.log 2>&1; rc=$?; echo "pytest sel rc=$rc"; tail -3 gpurun_out/r06_pytest_gpu_sel.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for w in 0 1; do
timeout -k 10 300 python bench.py --workload clay104 --steps 6 --warmup 2 --cpu-seconds 0 --e2e-seconds 0 --no-probes --tune rtc_wide=$w > gpurun_out/r06_clay104_wide$w.$rep.json 2>/dev/null; rc=$?; echo "clay104 wide=$w rc=$rc $(line gpurun_out/r06_clay104_wide$w.$rep.json)"; [ $rc -ne 0 ] && exit $rc
done; done
timeout -k 10 600 python bench.py --workload clay104 --sub-bytes 1048576 > gpurun_out/r06_clay104_1mib.json 2> gpurun_out/r06_clay104_1mib.err; rc=$?; echo "clay104 1MiB rc=$rc $(line gpurun_out/r06_clay104_1mib.json)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r06_clay104_1mib.err; exit $rc; }
timeout -k 10 400 python -u scripts/rs_layout_contract.py > gpurun_out/r06_rs_layout_contract2.jsonl 2> gpurun_out/r06_rs_layout_contract2.err; rc=$?; echo "layout rc=$rc"; cut -c1-120 gpurun_out/r06_rs_layout_contract2.jsonl; [ $rc -ne 0 ] && exit $rc
for W in rs173 rs124; do for L in "--layout natural" "--pitch recommended" "--layout blocked"; do
tag=$(echo "$W$L" | tr -d ' -'); timeout -k 10 300 python bench.py --workload $W $L --steps 4 --warmup 1 --cpu-seconds 0 --e2e-seconds 1 > gpurun_out/r06_$tag.json 2> gpurun_out/r06_$tag.err; rc=$?; echo "$W $L rc=$rc $(line gpurun_out/r06_$tag.json)"; [ $rc -ne 0 ] && { tail -3 gpurun_out/r06_$tag.err; exit $rc; }
done; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/r06_pytest_gpu_second.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06_pytest_gpu_second.log; exit $rc
