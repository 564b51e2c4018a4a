"""Launch-shape sweep of k_gf_check (isParityCorrect batch, apply_check.hip) on the published
RS(17,3) 200,000-B shape: ring depth x XCD runs x stagger, average launch time by HIP events
over a resident pool of 4,096 stripes, bytes verified (every verdict 1).  One JSON line per shape.

  python scripts/check_sweep.py [--pool 4096] [--reps 20] > gpurun_out/check_sweep.jsonl
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pool", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--encode", action="store_true", help="also time encodeParity on the same pool per shape")
    a = ap.parse_args()
    import torch
    import rpamd
    ecx = rpamd.load(shape_knobs=True)
    L, P = 200000, a.pool
    pool = torch.empty((P, 20, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 5)
    rs = ecx.ReedSolomon.create(17, 3)
    rs.encodeParityBatch(pool, 20 * L, L, P, 0, L)
    verdict = torch.zeros(P, dtype=torch.uint8, device="cuda")
    shapes = []
    for depth in (4, 8, 20):
        for xm, run in ((0, 8), (1, 4), (1, 8), (1, 16), (1, 32)):
            for stagger in (0, 2, 4, 8):
                shapes.append((depth, xm, run, stagger))
    for depth, xm, run, stagger in shapes:
        ecx.tune("depth", depth)
        ecx.tune("xcd_misaligned", xm)
        ecx.tune("xcd_run", run)
        ecx.tune("stagger", stagger)
        rs.isParityCorrectBatch(pool, 20 * L, L, P, 0, L, verdict)
        torch.cuda.synchronize()
        ok = bool((verdict == 1).all())
        kern = ecx.last_kernel()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
        for e0, e1 in ev:
            e0.record()
            rs.isParityCorrectBatch(pool, 20 * L, L, P, 0, L, verdict)
            e1.record()
        torch.cuda.synchronize()
        ms = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
        med = ms[len(ms) // 2]
        line = {"depth": depth, "xcd_runs": xm, "xcd_run": run, "stagger": stagger, "kernel": kern, "verified": ok,
                "median_ms": round(med, 4), "min_ms": round(ms[0], 4),
                "frac": round(P * 20 * L / (med * 1e-3) / 8e12, 4)}
        if a.encode:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
            for e0, e1 in ev:
                e0.record()
                rs.encodeParityBatch(pool, 20 * L, L, P, 0, L)
                e1.record()
            torch.cuda.synchronize()
            ems = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
            line["encode_median_ms"] = round(ems[len(ems) // 2], 4)
        print(json.dumps(line), flush=True)
    for k, v in (("depth", 0), ("xcd_misaligned", 1), ("xcd_run", 8), ("stagger", 0)):
        ecx.tune(k, v)


if __name__ == "__main__":
    main()
