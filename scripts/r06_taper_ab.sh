# (host_taper was removed after this A/B; the script records how profiles/r06_taper_ab.jsonl was taken.)
# e2e leg with and without the tapered last chunk (ecx_tune host_taper), interleaved A B B A.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
: > gpurun_out/r06_taper_ab.jsonl
for W in clay104 clay42 rs124; do for T in 1 4 4 1; do
  timeout -k 10 300 python bench.py --workload $W --steps 1 --warmup 0 --cpu-seconds 0 --no-probes --e2e-seconds 3 --tune host_taper=$T > gpurun_out/r06_taper.json 2>/dev/null; rc=$?
  python -c "import json,sys; d=json.loads(open('gpurun_out/r06_taper.json').read().strip().splitlines()[-1]); e=d['e2e']; print(json.dumps({'workload': '$W', 'host_taper': $T, 'e2e_GiBps': e['GiBps'], 'h2d_GBps': e['h2d_GBps'], 'd2h_GBps': e['d2h_GBps'], 'stripes_per_call': e['stripes_per_call'], 'verified': e['verified']}))" >> gpurun_out/r06_taper_ab.jsonl
  echo "$W taper=$T rc=$rc $(tail -1 gpurun_out/r06_taper_ab.jsonl)"; [ $rc -ne 0 ] && exit $rc
done; done
exit 0
