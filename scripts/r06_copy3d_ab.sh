# (the ECX_AB_* override existed only for this A/B; the measured winner is now fixed in host_pipe.cpp.)
# 3D copies in the host pipe (host_pipe.cpp plan_copies; ECX_AB_3D=0 turned them off for this A/B
# only): the host-batch parity tests (pageable and pinned, 3D on), then the e2e legs A B B A.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "host or blocked" > gpurun_out/r06_copy3d_tests.log 2>&1 || { tail -40 gpurun_out/r06_copy3d_tests.log; exit 1; }
tail -1 gpurun_out/r06_copy3d_tests.log
: > gpurun_out/r06_copy3d_ab.jsonl
for W in clay104 clay42; do for F in 1 0 0 1; do
  ECX_AB_3D=$F timeout -k 10 300 python bench.py --workload $W --steps 1 --warmup 0 --cpu-seconds 0 --no-probes --e2e-seconds 3 > gpurun_out/r06_c3.json 2>/dev/null; rc=$?
  [ $rc -ne 0 ] && { echo "$W 3d=$F rc=$rc"; exit $rc; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/r06_c3.json').read().strip().splitlines()[-1]); e=d['e2e']; print(json.dumps({'workload': '$W', 'copies_3d': $F, 'e2e_GiBps': e.get('GiBps'), 'h2d_GBps': e.get('h2d_GBps'), 'd2h_GBps': e.get('d2h_GBps'), 'stripes_per_call': e.get('stripes_per_call'), 'verified': e.get('verified')}))" >> gpurun_out/r06_copy3d_ab.jsonl
  tail -1 gpurun_out/r06_copy3d_ab.jsonl
done; done
