"""Headline sweep over the erased node ("also sweep
e=0..5"): Clay(4,2), B = 32 KiB, single-node repair of node e over one resident pool
of valid stripes, every e verified against the erased originals, then timed in
interleaved rounds (median).  Algorithmic bytes per repair: 20 helper + 8 repaired
sub-chunks (917,504 B) for every e.

    python scripts/erased_sweep.py [--pool 16384 --rounds 5 --reps 5]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import rpamd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pool", type=int, default=1 << 14)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    ecx = rpamd.load()
    P = args.pool
    wl = bench.Clay42(ecx, torch, torch.device("cuda", 0), P, 0, 0x5EED)
    steps = {e: ecx.ClayCodeErasureDecodingStep([e], bench.K, bench.M) for e in range(bench.N_NODES)}
    unit = 28 * bench.B

    def launch(e):
        steps[e].performCodingBatch(wl.pool, bench.STRIPE_BYTES, bench.B, wl.out, bench.ALPHA * bench.B, bench.B,
                                    P, bench.B)

    ok = {}
    for e in steps:
        launch(e)
        torch.cuda.synchronize()
        ok[e] = bool(torch.equal(wl.out, wl.pool.view(P, bench.ALPHA, bench.N_NODES, bench.B)[:, :, e, :]))
    times = {e: [] for e in steps}
    for _ in range(args.rounds):
        for e in steps:
            launch(e)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                launch(e)
            e1.record()
            torch.cuda.synchronize()
            times[e].append(e0.elapsed_time(e1) / args.reps * 1e-3)
    for e in steps:
        sec = statistics.median(times[e])
        inf = steps[e].map().info()
        print(json.dumps({"config": "Clay(4,2) single repair, 32 KiB", "erased": e, "stripes": P, "map": inf,
                          "ms_per_launch": round(sec * 1e3, 3), "GiBps": round(unit * P / sec / 2**30, 1),
                          "GBps": round(unit * P / sec / 1e9, 1), "frac_of_peak": round(unit * P / sec / 8e12, 4),
                          "verified": ok[e]}), flush=True)
    if not all(ok.values()):
        raise SystemExit("a repair differs from the erased originals")


if __name__ == "__main__":
    main()
