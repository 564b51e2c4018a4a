# The blocked RS batches from host memory (ecx_rs_*_blocked_batch_host): parity tests (direct and
# through the JNI forwarders) and the blocked bench lines' end-to-end legs, which now call them.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_jni_runtime.py -m gpu -x -q --timeout 120 --timeout-method thread -k "blocked" > gpurun_out/r06_blocked_host_tests.log 2>&1 || { tail -40 gpurun_out/r06_blocked_host_tests.log; exit 1; }
tail -2 gpurun_out/r06_blocked_host_tests.log
: > gpurun_out/r06_blocked_e2e.jsonl
for W in rs173 rs124; do
  timeout -k 10 400 python bench.py --workload $W --layout blocked --steps 5 --warmup 2 --cpu-seconds 0 --e2e-seconds 3 > gpurun_out/r06_blocked_$W.json 2> gpurun_out/r06_blocked_$W.err || { tail -20 gpurun_out/r06_blocked_$W.err; exit 1; }
  tail -1 gpurun_out/r06_blocked_$W.json >> gpurun_out/r06_blocked_e2e.jsonl
  python -c "import json; d=json.loads(open('gpurun_out/r06_blocked_$W.json').read().strip().splitlines()[-1]); print('$W', d['value'], d['unit'], d['roofline']['frac'], d.get('verified'), json.dumps(d['e2e'])[:400])"
done
