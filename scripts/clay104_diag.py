"""Which part of the Clay(10,4) plane-group repair kernel (k_clay_repair_grp) stops it short
of its access pattern's ceiling: DIAGNOSTIC builds (ecx_tune "rtc_diag", clay_rtc.hpp
RtcShape::diag; outputs are not the repair) each remove one part -- 1 the row-yc partner
loads, 2 the LDS exchange and barrier, 4 the lane-row exchange, 8 all output stores but
one, 16 the bit-plane transposes -- and are timed against the real kernel in interleaved
rounds on BASELINE config 4 (2,048 resident stripes, 1 MiB node blocks, repair of node 3).
Median launch time -> algorithmic GB/s of the REAL repair's bytes, fraction of 8 TB/s.

    python scripts/clay104_diag.py [--rounds 3 --reps 10]
"""
import argparse
import json
import os
import statistics
import sys
from pathlib import Path

os.environ["ECX_DIAGNOSTIC"] = "1"  # diagnostic builds are refused otherwise
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402

VARIANTS = [0, 1, 2, 4, 8, 16, 1 | 2, 1 | 2 | 4, 1 | 2 | 4 | 8, 31]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pool", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default=None, help="comma-separated rtc_diag values")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE")
    args = ap.parse_args()
    import torch
    ecx = rpamd.load()
    for kv in args.tune:
        k_, _, v_ = kv.partition("=")
        ecx.tune(k_, int(v_))
    variants = [int(v) for v in args.variants.split(",")] if args.variants else VARIANTS
    k, m, v, b, a = 10, 4, 2, 4096, 256
    n, P = k + m, args.pool
    pool = torch.empty((P, n * a, b), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 11)
    step = ecx.ClayCodeErasureDecodingStep([3], k, m, virtualUnits=v)
    info = step.map().info()
    unit = (info["n_in"] + info["n_out"]) * b
    out = torch.empty((P, a, b), dtype=torch.uint8, device="cuda")
    times = {d: [] for d in variants}
    ref = None
    try:
        for _ in range(args.rounds):
            for d in variants:
                ecx.tune("rtc_diag", d)
                step.performCodingBatch(pool, n * a * b, b, out, a * b, b, P, b)
                torch.cuda.synchronize()
                if ecx.last_kernel() != "k_clay_repair_grp":
                    raise SystemExit("ran %s" % ecx.last_kernel())
                if d == 0:
                    if ref is None:
                        ref = out.clone()
                    elif not torch.equal(out, ref):
                        raise SystemExit("the real kernel's output changed between rounds")
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(args.reps)]
                for e0, e1 in evs:
                    e0.record()
                    step.performCodingBatch(pool, n * a * b, b, out, a * b, b, P, b)
                    e1.record()
                torch.cuda.synchronize()
                times[d].extend(e0.elapsed_time(e1) for e0, e1 in evs)
    finally:
        ecx.tune("rtc_diag", 0)
    for d in variants:
        ms = statistics.median(times[d])
        gbs = P * unit / (ms * 1e-3) / 1e9
        print(json.dumps({"rtc_diag": d, "tune": args.tune, "launch_ms": round(ms, 4), "GBps": round(gbs, 1),
                          "frac": round(gbs / 8000.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
