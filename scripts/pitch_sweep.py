"""RS(12,4) 2-erasure decode in place over a sweep of shard pitches (powers of two
from 256 KiB to 8 MiB, plus pads), each with the one-chunk kernel and with
k_gf_apply_skew (ecx_tune "skew_chunks" 4): which layouts collide in HBM, and
whether rotating the chunk order avoids it.  One resident buffer, viewed with each
pitch; interleaved rounds, median algorithmic GB/s (12 read + 2 written shards).

    python scripts/pitch_sweep.py [--rounds 3 --reps 3]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402

TOTAL = 24 << 30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pads", default="0,4096,8192,65536")
    args = ap.parse_args()
    import torch
    ecx = rpamd.load(shape_knobs=True)
    buf = torch.empty(TOTAL, dtype=torch.uint8, device="cuda")
    ecx.fill_random(buf, buf.numel(), 7)
    rs = ecx.ReedSolomon.create(12, 4)
    dmap = rs.decode_map([False, False] + [True] * 14)
    cases = []
    for lg in range(18, 24):
        L = 1 << lg
        for pad in [int(x) for x in args.pads.split(",")]:
            p = L + pad
            S = min(4096, TOTAL // (16 * p))
            cases.append((L, pad, S, lambda p=p, S=S, L=L: dmap.apply_batch(buf, 16 * p, p, buf, 16 * p, p, S, L)))
    res = {}
    for _ in range(args.rounds):
        for L, pad, S, fn in cases:
            for k in (0, 4):
                ecx.tune("skew_chunks", k)
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((L, pad, k), []).append(14 * L * S / (e0.elapsed_time(e1) / args.reps * 1e-3) / 1e9)
    ecx.tune("skew_chunks", 1)
    for (L, pad, k), v in res.items():
        med = statistics.median(v)
        print(json.dumps({"shard_KiB": L >> 10, "pad": pad, "skew_chunks": k, "GBps_median": round(med, 1),
                          "frac": round(med / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
