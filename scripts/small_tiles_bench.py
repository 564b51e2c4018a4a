"""Small single-tile maps (RS(12,4) 2-erasure decode = 2 rows, LRC encode = 4 rows,
LRC repair = 1 row) on the 8-row kernel vs the small-tile variants (ecx_tune
"small_tiles": 2 / 4 accumulator rows, ring depth 4 / 8 / 12).  Interleaved rounds
in one process, median algorithmic GB/s (BASELINE.md section 3 bytes per unit).

    python scripts/small_tiles_bench.py [--rounds 5 --reps 5]
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

SHAPES = [("rows8 auto", 0, 0), ("small d4", 1, 4), ("small d8", 1, 8), ("small d12", 1, 12), ("rows8 d8", 0, 8)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    ecx = rpamd.load(shape_knobs=True)
    cases = []
    rs = ecx.ReedSolomon.create(12, 4)
    dmap = rs.decode_map([False, False] + [True] * 14)
    L, S = 4 << 20, 256
    for pad in (4096, 0):
        p = L + pad
        pool = torch.empty((S, 16, p), dtype=torch.uint8, device="cuda")
        ecx.fill_random(pool, pool.numel(), 1)
        cases.append((f"RS(12,4) decode {{0,1}} in place, pitch 4 MiB + {pad}", 14 * L * S,
                      lambda pool=pool, p=p: dmap.apply_batch(pool, 16 * p, p, pool, 16 * p, p, S, L), pool))
    B, S3 = 65536, 1 << 14
    lpool = torch.empty((S3, 16, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(lpool, lpool.numel(), 2)
    encm = np.zeros((4, 16), np.uint8)
    for g in range(4):
        encm[g, 4 * g:4 * g + 3] = 1
    emap = ecx.GfMap.from_matrix(encm, in_slot=list(range(16)), out_slot=[3, 7, 11, 15])
    cases.append(("LRC encode, 64 KiB", 16 * B * S3,
                  lambda: emap.apply_batch(lpool, 16 * B, B, lpool, 16 * B, B, S3, B), (lpool, emap)))
    rmap = ecx.GfMap.from_matrix(np.array([[1, 1, 1]], np.uint8), in_slot=[0, 1, 3], out_slot=[0])
    lout = torch.empty((S3, 1, B), dtype=torch.uint8, device="cuda")
    cases.append(("LRC repair of block 2, 64 KiB", 4 * B * S3,
                  lambda: rmap.apply_batch(lpool, 16 * B, B, lout, B, B, S3, B), (lout, rmap)))
    res = {(c[0], s[0]): [] for c in cases for s in SHAPES}
    for _ in range(args.rounds):
        for name, nbytes, fn, _keep in cases:
            for label, st, depth in SHAPES:
                ecx.tune("small_tiles", st)
                ecx.tune("depth", depth)
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[(name, label)].append(nbytes / (e0.elapsed_time(e1) / args.reps * 1e-3) / 1e9)
    ecx.tune("small_tiles", 2)
    ecx.tune("depth", 0)
    for (name, label), v in res.items():
        med = statistics.median(v)
        print(json.dumps({"case": name, "shape": label, "GBps_median": round(med, 1), "frac": round(med / 8000, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
