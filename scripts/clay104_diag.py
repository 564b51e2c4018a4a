"""Which part of the Clay(10,4) plane-group repair kernel (k_clay_repair_grp) stops it short
of its access pattern's ceiling: DIAGNOSTIC builds (ecx_tune "rtc_diag", clay_rtc.hpp
RtcShape::diag; outputs are not the repair) each remove one part -- 1 the row-yc partner
loads, 2 the LDS exchange and barrier, 4 the lane-row exchange, 8 all output stores but
one, 16 the bit-plane transposes -- and are timed against the real kernel in interleaved
rounds on BASELINE config 4 (2,048 resident stripes, 1 MiB node blocks, repair of node 3).
Median launch time -> algorithmic GB/s of the REAL repair's bytes, fraction of 8 TB/s.

    python scripts/clay104_diag.py [--rounds 3 --reps 10] [--shapes | --lean | --final | --nt | --json LIST]
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
# --shapes: real (non-diagnostic) code shapes of the same kernel, as tune dicts
SHAPES = [{}, {"rtc_units": 2}, {"rtc_units": 2, "rtc_waves": 2}, {"rtc_waves": 2},
          {"rtc_units": 2, "rtc_xcd": 3}, {"rtc_units": 2, "rtc_waves": 2, "rtc_xcd": 3}]
LEAN = [{}, {"rtc_sched": 1, "rtc_waves": 4, "rtc_lookahead": 0}, {"rtc_sched": 1, "rtc_waves": 4},
        {"rtc_sched": 1, "rtc_waves": 4, "rtc_lookahead": 2}, {"rtc_sched": 1, "rtc_waves": 4, "rtc_lookahead": 3},
        {"rtc_sched": 1, "rtc_waves": 4, "rtc_xcd": 3}, {"rtc_sched": 1, "rtc_waves": 4, "rtc_xcd": 1},
        {"rtc_sched": 2, "rtc_lookahead": 0}, {"rtc_sched": 2, "rtc_waves": 4, "rtc_lookahead": 0},
        {"rtc_sched": 2}, {"rtc_sched": 2, "rtc_lookahead": 8}]
FINAL = [{}, {"rtc_sched": 2, "rtc_lookahead": 8}, {"rtc_sched": 2, "rtc_lookahead": 0},
         {"rtc_sched": 1, "rtc_waves": 4, "rtc_lookahead": 0}, {"rtc_sched": 1, "rtc_waves": 4, "rtc_lookahead": 0, "rtc_xcd": 3}]
# --nt: non-temporal load policies (rtc_nt bits: 1 rows read once, 2 row-yc own, 4 row-yc partners; default 5)
NT = [{"rtc_nt": 0}, {"rtc_nt": 1}, {"rtc_nt": 3}, {"rtc_nt": 7}, {}, {"rtc_nt": 2}, {"rtc_nt": 1, "rtc_xcd": 3}]
# --json '[{...}, ...]': any list of bit-exact shapes
DEFAULTS = {"rtc_units": 1, "rtc_waves": 3, "rtc_xcd": 2, "rtc_lookahead": 1, "rtc_diag": 0, "rtc_sched": 2, "rtc_nt": 5}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pool", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default=None, help="comma-separated rtc_diag values")
    ap.add_argument("--shapes", action="store_true", help="time the SHAPES code shapes instead (all bit-exact)")
    ap.add_argument("--lean", action="store_true", help="time the LEAN schedule shapes instead (all bit-exact)")
    ap.add_argument("--final", action="store_true", help="time the FINAL candidates instead (all bit-exact)")
    ap.add_argument("--nt", action="store_true", help="time the NT load policies instead (all bit-exact)")
    ap.add_argument("--json", default=None, help="a JSON list of tune dicts to time (all bit-exact)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE")
    args = ap.parse_args()
    import torch
    ecx = rpamd.load(shape_knobs=True)
    for kv in args.tune:
        k_, _, v_ = kv.partition("=")
        ecx.tune(k_, int(v_))
    if args.json:
        variants = [dict(sh) for sh in json.loads(args.json)]
    elif args.shapes or args.lean or args.final or args.nt:
        variants = [dict(sh) for sh in (SHAPES if args.shapes else LEAN if args.lean else FINAL if args.final else NT)]
    else:
        variants = [{"rtc_diag": int(v)} for v in (args.variants.split(",") if args.variants else VARIANTS)]
    k, m, v, b, a = 10, 4, 2, 4096, 256
    n, P = k + m, args.pool
    pool = torch.empty((P, n * a, b), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 11)
    step = ecx.ClayCodeErasureDecodingStep([3], k, m, virtualUnits=v)
    info = step.map().info()
    unit = (info["n_in"] + info["n_out"]) * b
    out = torch.empty((P, a, b), dtype=torch.uint8, device="cuda")
    times = {i: [] for i in range(len(variants))}
    ref = None
    try:
        for _ in range(args.rounds):
            for i, d in enumerate(variants):
                for k_, v_ in DEFAULTS.items():
                    ecx.tune(k_, d.get(k_, v_))
                step.performCodingBatch(pool, n * a * b, b, out, a * b, b, P, b)
                torch.cuda.synchronize()
                if ecx.last_kernel() != "k_clay_repair_grp":
                    raise SystemExit("ran %s" % ecx.last_kernel())
                if not d.get("rtc_diag"):  # every real shape must give the same repair
                    if ref is None:
                        ref = out.clone()
                    elif not torch.equal(out, ref):
                        raise SystemExit("shape %s: output differs" % d)
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(args.reps)]
                for e0, e1 in evs:
                    e0.record()
                    step.performCodingBatch(pool, n * a * b, b, out, a * b, b, P, b)
                    e1.record()
                torch.cuda.synchronize()
                times[i].extend(e0.elapsed_time(e1) for e0, e1 in evs)
    finally:
        for k_, v_ in DEFAULTS.items():
            ecx.tune(k_, v_)
    for i, d in enumerate(variants):
        ms = statistics.median(times[i])
        gbs = P * unit / (ms * 1e-3) / 1e9
        print(json.dumps({"variant": d, "tune": args.tune, "launch_ms": round(ms, 4), "GBps": round(gbs, 1),
                          "frac": round(gbs / 8000.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
