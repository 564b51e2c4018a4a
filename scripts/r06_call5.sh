set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
line() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['unit'], r['frac'], r['kernel'], (d.get('e2e') or {}).get('GiBps'))" "$1"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_percall.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "blocked or percall or concurrent" > gpurun_out/r06_pytest_gpu_sel2.log 2>&1; rc=$?; echo "pytest sel rc=$rc"; tail -3 gpurun_out/r06_pytest_gpu_sel2.log; [ $rc -ne 0 ] && exit $rc
for T in 1 16; do timeout -k 10 400 tests/native/_build/percall_threshold --threads $T > gpurun_out/r06_percall_threads$T.jsonl 2> gpurun_out/r06_percall_threads$T.err; rc=$?; echo "percall T=$T rc=$rc"; grep crossover gpurun_out/r06_percall_threads$T.jsonl; [ $rc -ne 0 ] && exit $rc; done
for W in rs173 rs124; do for L in "--pitch recommended" "--layout blocked"; do
tag=$(echo "$W$L" | tr -d ' -'); timeout -k 10 300 python bench.py --workload $W $L --steps 4 --warmup 1 --cpu-seconds 0 --e2e-seconds 0 > gpurun_out/r06_$tag.json 2> gpurun_out/r06_$tag.err; rc=$?; echo "$W $L rc=$rc $(line gpurun_out/r06_$tag.json)"; [ $rc -ne 0 ] && { tail -3 gpurun_out/r06_$tag.err; exit $rc; }
done; done
exit 0
