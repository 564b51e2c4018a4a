# Host-batch parity tests and the e2e legs of the two many-run workloads on the final host_pipe.cpp.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "host" > gpurun_out/r06_hostpipe_tests.log 2>&1 || { tail -30 gpurun_out/r06_hostpipe_tests.log; exit 1; }
tail -2 gpurun_out/r06_hostpipe_tests.log
: > gpurun_out/r06_minrows_final.jsonl
for W in clay104 clay42x2 clay42; do
  timeout -k 10 300 python bench.py --workload $W --steps 1 --warmup 0 --cpu-seconds 0 --no-probes --e2e-seconds 3 > gpurun_out/r06_mr.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/r06_mr.json').read().strip().splitlines()[-1]); e=d['e2e']; print(json.dumps({'workload': '$W', 'min_rows': 160, 'e2e_GiBps': e.get('GiBps'), 'h2d_GBps': e.get('h2d_GBps'), 'd2h_GBps': e.get('d2h_GBps'), 'stripes_per_call': e.get('stripes_per_call'), 'verified': e.get('verified')}))" >> gpurun_out/r06_minrows_final.jsonl
  tail -1 gpurun_out/r06_minrows_final.jsonl
done
