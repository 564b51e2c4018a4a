# The round's per-workload bench lines (default CPU protocol), appended to gpurun_out/$OUT (default
# r06_workloads.jsonl; give each gpurun call its own file: a call's merge replaces the file).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
OUT="${OUT:-r06_workloads.jsonl}"
for spec in "$@"; do
  args=$(echo "$spec" | tr ':' ' ')
  tag=$(echo "$spec" | tr -d ' :-')
  timeout -k 10 400 python bench.py $args --steps 3 --warmup 1 > gpurun_out/r06_wl_$tag.json 2> gpurun_out/r06_wl_$tag.err; rc=$?
  echo "$spec rc=$rc $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['unit'], r['frac'], r['traffic'] and round(r['traffic']/r['algorithmic_bytes_per_launch'],5), (d.get('e2e') or {}).get('GiBps'), (d.get('cpu_baseline') or {}).get('value'))" gpurun_out/r06_wl_$tag.json 2>&1 | tail -1)"
  [ $rc -ne 0 ] && { tail -3 gpurun_out/r06_wl_$tag.err; exit $rc; }
  tail -1 gpurun_out/r06_wl_$tag.json >> "gpurun_out/$OUT"
done
exit 0
