# End-to-end leg at three host_chunk_kib settings (ecx_tune), interleaved A B C C B A: does a larger
# chunk (fewer, larger strided copies per call) pay for the per-copy gaps the memory-copy trace
# shows (profiles/r06_e2e_trace/summary.jsonl)?
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
: > gpurun_out/r06_chunk_ab.jsonl
for W in clay104 clay42 rs124; do for C in 65536 262144 524288 524288 262144 65536; do
  timeout -k 10 300 python bench.py --workload $W --steps 1 --warmup 0 --cpu-seconds 0 --no-probes --e2e-seconds 3 --tune host_chunk_kib=$C > gpurun_out/r06_chunk.json 2>/dev/null; rc=$?
  [ $rc -ne 0 ] && { echo "$W chunk=$C rc=$rc"; exit $rc; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/r06_chunk.json').read().strip().splitlines()[-1]); e=d['e2e']; print(json.dumps({'workload': '$W', 'host_chunk_kib': $C, 'e2e_GiBps': e['GiBps'], 'h2d_GBps': e['h2d_GBps'], 'd2h_GBps': e['d2h_GBps'], 'stripes_per_call': e['stripes_per_call'], 'verified': e['verified']}))" >> gpurun_out/r06_chunk_ab.jsonl
  echo "$W chunk=$C $(tail -1 gpurun_out/r06_chunk_ab.jsonl)"
done; done
exit 0
