# (ECX_AB_MINROWS was a temporary override in host_pipe.cpp for these A/Bs; the floor is now fixed at 160.)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
: > gpurun_out/r06_minrows_ab.jsonl
for W in clay104; do for V in "64 0" "160 0" "160 1" "64 1" "160 1" "160 0" "64 0" "96 1" "96 0"; do
  set -- $V
  ECX_AB_MINROWS=$1 ECX_AB_BALANCE=$2 timeout -k 10 300 python bench.py --workload $W --steps 1 --warmup 0 --cpu-seconds 0 --no-probes --e2e-seconds 3 > gpurun_out/r06_mr.json 2>/dev/null; rc=$?
  [ $rc -ne 0 ] && { echo "$W $V rc=$rc"; exit $rc; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/r06_mr.json').read().strip().splitlines()[-1]); e=d['e2e']; print(json.dumps({'workload': '$W', 'min_rows': $1, 'balance': $2, 'e2e_GiBps': e['GiBps'], 'h2d_GBps': e['h2d_GBps'], 'd2h_GBps': e['d2h_GBps'], 'verified': e['verified']}))" >> gpurun_out/r06_minrows_ab.jsonl
  echo "$(tail -1 gpurun_out/r06_minrows_ab.jsonl)"
done; done
