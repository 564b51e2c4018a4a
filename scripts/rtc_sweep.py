"""Sweep the generated per-helper-plane Clay kernel's code shape (ecx_tune
"rtc_lookahead" x "rtc_waves" x "rtc_xcd", and the plane-group kernel "rtc_group" 1 x
"rtc_waves" x "rtc_xcd") on BASELINE config 4 (shortened Clay(10,4), 1 MiB node
blocks = 256 x 4 KiB sub-chunks, repair of node 3) in one process: one resident pool,
every shape verified against the composed-map kernel, interleaved rounds, median
per-launch time -> algorithmic GB/s and fraction of the 8 TB/s HBM peak.

    python scripts/rtc_sweep.py [--pool 2048 --reps 10 --rounds 2]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pool", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--erased", type=int, default=3)
    ap.add_argument("--grp", default=None, help="plane-group shapes as la:waves:persist[:xcd],... (default XCD order 2)")
    ap.add_argument("--group-only", action="store_true", help="composed, the default per-plane shape and the "
                    "plane-group kernel shapes only")
    args = ap.parse_args()
    import torch
    ecx = rpamd.load(shape_knobs=True)
    k, m, v, b, a = 10, 4, 2, 4096, 256
    n, P = k + m, args.pool
    pool = torch.empty((P, n * a, b), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 11)
    step = ecx.ClayCodeErasureDecodingStep([args.erased], k, m, virtualUnits=v)
    info = step.map().info()
    unit = (info["n_in"] + info["n_out"]) * b
    ref = torch.empty((P, a, b), dtype=torch.uint8, device="cuda")
    ecx.tune("clay_rtc", 0)
    step.performCodingBatch(pool, n * a * b, b, ref, a * b, b, P, b)
    torch.cuda.synchronize()
    shapes = [("composed", None, None, 0)]
    if args.group_only:
        shapes += [("rtc", 1, 3, 1)]
    else:
        shapes += [("rtc", la, w, x) for x in (0, 1) for w in (2, 3) for la in (0, 1, 2)]
    if args.grp:
        for t in args.grp.split(","):
            f = [int(v) for v in t.split(":")]
            shapes.append(("grp", f[0], f[1], f[3] if len(f) > 3 else 2, f[2]))
    elif args.group_only:
        shapes += [("grp", la, w, 1) for la in (0, 1, 2, 3) for w in (2, 3)]
    else:
        shapes += [("grp", la, w, x) for x in (0, 1) for w in (2, 3) for la in (0, 1, 2, 3)]
    out = torch.empty_like(ref)
    times = {s: [] for s in shapes}
    for _ in range(args.rounds):
        for s in shapes:
            if s[0] == "composed":
                ecx.tune("clay_rtc", 0)
            else:
                ecx.tune("clay_rtc", 2)
                ecx.tune("rtc_group", 1 if s[0] == "grp" else 0)
                ecx.tune("rtc_lookahead", s[1] if s[1] is not None else 1)
                ecx.tune("rtc_waves", s[2])
                ecx.tune("rtc_xcd", s[3])
                ecx.tune("rtc_persist", s[4] if len(s) > 4 else 0)
            out.fill_(0)
            step.performCodingBatch(pool, n * a * b, b, out, a * b, b, P, b)
            torch.cuda.synchronize()
            if not (s[1] or 0) & 16 and not torch.equal(out, ref):  # bit 4: movement-only diagnostic build
                raise SystemExit("shape %s differs from the composed kernel" % (s,))
            if s[0] != "composed":
                want = "k_clay_repair_grp" if s[0] == "grp" else "k_clay_repair"
                if ecx.last_kernel() != want:
                    raise SystemExit("shape %s ran %s" % (s, ecx.last_kernel()))
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
            for e0, e1 in evs:
                e0.record()
                step.performCodingBatch(pool, n * a * b, b, out, a * b, b, P, b)
                e1.record()
            torch.cuda.synchronize()
            times[s].extend(e0.elapsed_time(e1) for e0, e1 in evs)
    for s in shapes:
        ms = statistics.median(times[s])
        gbs = P * unit / (ms * 1e-3) / 1e9
        print(json.dumps({"kernel": s[0], "rtc_lookahead": s[1], "rtc_waves": s[2], "rtc_xcd": s[3],
                          "rtc_persist": s[4] if len(s) > 4 else 0,
                          "launch_ms": round(ms, 4),
                          "GBps": round(gbs, 1), "frac": round(gbs / 8000.0, 4)}), flush=True)
    ecx.tune("clay_rtc", 1)
    ecx.tune("rtc_lookahead", 1)
    ecx.tune("rtc_waves", 3)
    ecx.tune("rtc_xcd", 2)
    ecx.tune("rtc_group", 1)
    ecx.tune("rtc_persist", 0)


if __name__ == "__main__":
    main()
