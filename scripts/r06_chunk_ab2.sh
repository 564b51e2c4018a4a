# host_chunk_kib on the final host pipe (3D copies, copy-keyed floor): 32 / 64 / 128 MiB, A B C C B A.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
: > gpurun_out/r06_chunk_ab2.jsonl
for W in clay104 clay42; do for C in 32768 65536 131072 131072 65536 32768; do
  timeout -k 10 300 python bench.py --workload $W --steps 1 --warmup 0 --cpu-seconds 0 --no-probes --e2e-seconds 3 --tune host_chunk_kib=$C > gpurun_out/r06_ck.json 2>/dev/null; rc=$?
  [ $rc -ne 0 ] && { echo "$W chunk=$C rc=$rc"; exit $rc; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/r06_ck.json').read().strip().splitlines()[-1]); e=d['e2e']; print(json.dumps({'workload': '$W', 'host_chunk_kib': $C, 'e2e_GiBps': e.get('GiBps'), 'h2d_GBps': e.get('h2d_GBps'), 'plan': e.get('plan')}))" >> gpurun_out/r06_chunk_ab2.jsonl
  tail -1 gpurun_out/r06_chunk_ab2.jsonl | cut -c1-140
done; done
