"""Busy/idle reading of a rocprofv3 memory-copy + kernel trace of bench.py's end-to-end leg
(scripts/r06_e2e_trace.sh). The leg's copies are the many-copy kind (the pinned host pool's
direction shows as DEVICE_TO_DEVICE under this trace); per copy stream: the leg window (first copy
start to last copy end), the union of busy intervals, and the idle gaps sorted into bins, so a
reader can tell per-copy overhead (many short gaps) from pipeline drain (few long ones).

    python scripts/e2e_trace_summary.py gpurun_out/r06_e2e_trace_clay104 [...]  > summary.json
"""
import csv
import json
import sys
from pathlib import Path

BINS_US = (10, 100, 1000)


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def summarise(d):
    d = Path(d)
    copies = {}
    with open(d / "run_memory_copy_trace.csv") as f:
        for r in csv.DictReader(f):
            if r["Direction"] != "MEMORY_COPY_DEVICE_TO_DEVICE":
                continue
            copies.setdefault(int(r["Stream_Id"]), []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    kern = []
    with open(d / "run_kernel_trace.csv") as f:
        for r in csv.DictReader(f):
            kern.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    lo = min(s for v in copies.values() for s, _ in v)
    hi = max(e for v in copies.values() for _, e in v)
    out = {"trace": d.name, "window_ms": round((hi - lo) / 1e6, 3), "streams": []}
    for sid, v in sorted(copies.items(), key=lambda kv: -len(kv[1])):
        u = union(v)
        busy = sum(e - s for s, e in u)
        gaps = [u[i + 1][0] - u[i][1] for i in range(len(u) - 1)]
        bins = {}
        for g in gaps:
            key = next(("<%dus" % b for b in BINS_US if g < b * 1000), ">=%dus" % BINS_US[-1])
            c = bins.setdefault(key, [0, 0])
            c[0] += 1
            c[1] += g
        s0, s1 = u[0][0], u[-1][1]
        out["streams"].append({
            "stream": sid, "copies": len(v), "span_ms": round((s1 - s0) / 1e6, 3),
            "busy_frac": round(busy / max(1, s1 - s0), 4),
            "avg_copy_us": round(sum(e - s for s, e in v) / len(v) / 1e3, 2),
            "gaps": {k: {"count": c, "total_ms": round(t / 1e6, 3)} for k, (c, t) in sorted(bins.items())}})
    ku = union([(s, e) for s, e, _ in kern if e > lo and s < hi])
    out["kernel_busy_frac_in_window"] = round(sum(min(e, hi) - max(s, lo) for s, e in ku) / max(1, hi - lo), 4)
    return out


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(json.dumps(summarise(p)))
