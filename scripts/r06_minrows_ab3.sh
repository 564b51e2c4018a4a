# (ECX_AB_MINROWS was a temporary override in host_pipe.cpp for these A/Bs; the floor is now fixed at 160.)
# The many-run chunk floor above 160 rows (ECX_AB_MINROWS, this A/B only) on Clay(4,2) {0,3}.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
: > gpurun_out/r06_minrows_ab3.jsonl
for W in clay42x2; do for V in 160 256 512 512 256 160; do
  ECX_AB_MINROWS=$V timeout -k 10 300 python bench.py --workload $W --steps 1 --warmup 0 --cpu-seconds 0 --no-probes --e2e-seconds 3 > gpurun_out/r06_mr.json 2>/dev/null; rc=$?
  [ $rc -ne 0 ] && { echo "$W $V rc=$rc"; exit $rc; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/r06_mr.json').read().strip().splitlines()[-1]); e=d['e2e']; print(json.dumps({'workload': '$W', 'min_rows': $V, 'e2e_GiBps': e.get('GiBps'), 'h2d_GBps': e.get('h2d_GBps'), 'd2h_GBps': e.get('d2h_GBps'), 'stripes_per_call': e.get('stripes_per_call'), 'verified': e.get('verified')}))" >> gpurun_out/r06_minrows_ab3.jsonl
  echo "$(tail -1 gpurun_out/r06_minrows_ab3.jsonl)"
done; done
