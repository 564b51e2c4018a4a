# The e2e legs on the final host pipe (3D copies, copy-keyed chunk floor): host-batch parity tests,
# then every workload's and layout variant's end-to-end rate (no timed region, no CPU baseline).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "host or blocked" > gpurun_out/r06_e2e_final_tests.log 2>&1 || { tail -40 gpurun_out/r06_e2e_final_tests.log; exit 1; }
tail -1 gpurun_out/r06_e2e_final_tests.log
: > gpurun_out/r06_e2e_final.jsonl
for spec in "--workload clay42" "--workload clay104" "--workload clay42x2" "--workload lrc" "--workload lrcenc" "--workload rs124" "--workload rs173" "--workload rs173check" "--workload rs124 --pitch recommended" "--workload rs173 --pitch recommended" "--workload rs124 --layout blocked" "--workload rs173 --layout blocked" "--workload clay104 --sub-bytes 1048576"; do
  timeout -k 10 300 python bench.py $spec --steps 1 --warmup 0 --cpu-seconds 0 --no-probes --e2e-seconds 3 > gpurun_out/r06_ef.json 2>/dev/null; rc=$?
  [ $rc -ne 0 ] && { echo "$spec rc=$rc"; exit $rc; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/r06_ef.json').read().strip().splitlines()[-1]); e=d['e2e']; print(json.dumps({'spec': '$spec', 'e2e_GiBps': e.get('GiBps'), 'h2d_GBps': e.get('h2d_GBps'), 'd2h_GBps': e.get('d2h_GBps'), 'MBps': e.get('MBps'), 'stripes_per_call': e.get('stripes_per_call'), 'verified': e.get('verified')}))" >> gpurun_out/r06_e2e_final.jsonl
  tail -1 gpurun_out/r06_e2e_final.jsonl
done
