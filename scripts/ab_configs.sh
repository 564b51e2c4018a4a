#!/bin/bash
# In-run A/B of two builds of libecx.so on every BASELINE config: the in-tree build
# (B) against scripts/ab/libecx_base.so (A, built from another commit), in the order
# A B B A so that clock and thermal drift hit both alike.  Each step has its own
# time limit; any failure stops the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
run_a() { ECX_LIB_PATH="$ROOT/scripts/ab/libecx_base.so" timeout -k 10 300 python scripts/configs_bench.py --rounds 3 \
    > "$OUT/ab_A$1.jsonl" 2>&1; }
run_b() { timeout -k 10 300 python scripts/configs_bench.py --rounds 3 > "$OUT/ab_B$1.jsonl" 2>&1; }
run_a 1 || exit $?
run_b 1 || exit $?
run_b 2 || exit $?   # second pair in the other order
run_a 2 || exit $?
python - "$OUT" <<'PY'
import json, sys, glob, statistics
out = sys.argv[1]
res = {}
for tag in "AB":
    for f in sorted(glob.glob(f"{out}/ab_{tag}*.jsonl")):
        for l in open(f):
            if l.startswith('{"config'):
                d = json.loads(l)
                res.setdefault((d["config"], d.get("layout", "")), {}).setdefault(tag, []).append(d["GBps"])
for (c, lay), v in res.items():
    a, b = statistics.mean(v["A"]), statistics.mean(v["B"])
    print(json.dumps({"config": c, "layout": lay, "A_GBps": round(a, 1), "B_GBps": round(b, 1),
                      "B_over_A": round(b / a, 4), "A_runs": v["A"], "B_runs": v["B"]}))
PY
