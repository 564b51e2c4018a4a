# (the ECX_AB_* override existed only for this A/B; the measured winner is now fixed in host_pipe.cpp.)
# After 3D copies: does the many-run chunk floor still pay?  ECX_AB_FLOOR=1 (this A/B only) keys the
# 160-stripe floor on the planned copies per chunk instead of the runs per stripe, which drops it for
# Clay(10,4) (3 copies) and Clay(4,2) {0,3} (1 copy).  A B B A.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
: > gpurun_out/r06_floor_ab.jsonl
for W in clay104 clay42x2; do for F in 0 1 1 0; do
  ECX_AB_FLOOR=$F timeout -k 10 300 python bench.py --workload $W --steps 1 --warmup 0 --cpu-seconds 0 --no-probes --e2e-seconds 3 > gpurun_out/r06_fl.json 2>/dev/null; rc=$?
  [ $rc -ne 0 ] && { echo "$W floor=$F rc=$rc"; exit $rc; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/r06_fl.json').read().strip().splitlines()[-1]); e=d['e2e']; print(json.dumps({'workload': '$W', 'floor_by_copies': $F, 'e2e_GiBps': e.get('GiBps'), 'h2d_GBps': e.get('h2d_GBps'), 'd2h_GBps': e.get('d2h_GBps'), 'verified': e.get('verified')}))" >> gpurun_out/r06_floor_ab.jsonl
  tail -1 gpurun_out/r06_floor_ab.jsonl
done; done
