"""Load-ring depth of the one-workgroup-per-tile kernel on single-tile maps,
interleaved rounds in one process (median algorithmic GB/s): the headline Clay(4,2)
repair (20 entries), LRC encode (12), RS(12,4) 2-erasure decode (12) on two shard
pitches, LRC repair (3).  Depth 0 = the library's per-map rule.

    python scripts/depth_bench.py [--rounds 5 --reps 5 --depths 0,8,12,20]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--depths", default="0,8,12,20")
    args = ap.parse_args()
    import torch
    ecx = rpamd.load(shape_knobs=True)
    depths = [int(d) for d in args.depths.split(",")]
    cases = []
    B, P = 32768, 1 << 14
    pool = torch.empty((P, 48, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 1)
    out = torch.empty((P, 8, B), dtype=torch.uint8, device="cuda")
    rep = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
    cases.append(("Clay(4,2) repair e=1, 32 KiB (20 entries)", 28 * B * P,
                  lambda: rep.performCodingBatch(pool, 48 * B, B, out, 8 * B, B, P, B), (pool, out, rep)))
    B3, S3 = 65536, 1 << 14
    lpool = torch.empty((S3, 16, B3), dtype=torch.uint8, device="cuda")
    ecx.fill_random(lpool, lpool.numel(), 2)
    encm = np.zeros((4, 16), np.uint8)
    for g in range(4):
        encm[g, 4 * g:4 * g + 3] = 1
    emap = ecx.GfMap.from_matrix(encm, in_slot=list(range(16)), out_slot=[3, 7, 11, 15])
    cases.append(("LRC encode, 64 KiB (12 entries)", 16 * B3 * S3,
                  lambda: emap.apply_batch(lpool, 16 * B3, B3, lpool, 16 * B3, B3, S3, B3), (lpool, emap)))
    rmap = ecx.GfMap.from_matrix(np.array([[1, 1, 1]], np.uint8), in_slot=[0, 1, 3], out_slot=[0])
    lout = torch.empty((S3, 1, B3), dtype=torch.uint8, device="cuda")
    cases.append(("LRC repair, 64 KiB (3 entries)", 4 * B3 * S3,
                  lambda: rmap.apply_batch(lpool, 16 * B3, B3, lout, B3, B3, S3, B3), (lout, rmap)))
    rs = ecx.ReedSolomon.create(12, 4)
    dmap = rs.decode_map([False, False] + [True] * 14)
    for L, pad, S in ((4 << 20, 4096, 256), (1 << 20, 0, 1024)):
        p = L + pad
        rpool = torch.empty((S, 16, p), dtype=torch.uint8, device="cuda")
        ecx.fill_random(rpool, rpool.numel(), 4)
        cases.append((f"RS(12,4) decode, {L >> 20} MiB shards, pitch +{pad} (12 entries)", 14 * L * S,
                      lambda rpool=rpool, p=p, S=S, L=L: dmap.apply_batch(rpool, 16 * p, p, rpool, 16 * p, p, S, L),
                      rpool))
    res = {(c[0], d): [] for c in cases for d in depths}
    for _ in range(args.rounds):
        for name, nbytes, fn, _keep in cases:
            for d in depths:
                ecx.tune("depth", d)
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[(name, d)].append(nbytes / (e0.elapsed_time(e1) / args.reps * 1e-3) / 1e9)
    ecx.tune("depth", 0)
    for (name, d), v in res.items():
        med = statistics.median(v)
        print(json.dumps({"case": name, "depth": d, "GBps_median": round(med, 1), "frac": round(med / 8000, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
