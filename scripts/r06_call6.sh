set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/r06_pytest_gpu_third.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06_pytest_gpu_third.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r06_bench_second.json 2> gpurun_out/r06_bench_second.err; rc=$?; echo "bench rc=$rc"; python -c "import json; d=json.loads(open('gpurun_out/r06_bench_second.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['e2e']['GiBps'], d['cpu_baseline']['value'])"; exit $rc
