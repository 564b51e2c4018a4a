# Column slices for one-chunk batches (host_pipe.cpp): the host-batch parity tests, then the
# config-4 1 MiB-sub-chunk line's e2e leg (one 3.5 GiB stripe per call) and the headline's.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "host or blocked or slices" > gpurun_out/r06_slices_tests.log 2>&1 || { tail -40 gpurun_out/r06_slices_tests.log; exit 1; }
tail -1 gpurun_out/r06_slices_tests.log
: > gpurun_out/r06_slices_e2e.jsonl
for spec in "--workload clay104 --sub-bytes 1048576" "--workload clay104" "--workload clay42"; do
  timeout -k 10 300 python bench.py $spec --steps 1 --warmup 0 --cpu-seconds 0 --no-probes --e2e-seconds 3 > gpurun_out/r06_sl.json 2>/dev/null; rc=$?
  [ $rc -ne 0 ] && { echo "$spec rc=$rc"; exit $rc; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/r06_sl.json').read().strip().splitlines()[-1]); e=d['e2e']; print(json.dumps({'spec': '$spec', 'e2e_GiBps': e.get('GiBps'), 'h2d_GBps': e.get('h2d_GBps'), 'd2h_GBps': e.get('d2h_GBps'), 'stripes_per_call': e.get('stripes_per_call'), 'verified': e.get('verified')}))" >> gpurun_out/r06_slices_e2e.jsonl
  tail -1 gpurun_out/r06_slices_e2e.jsonl
done
