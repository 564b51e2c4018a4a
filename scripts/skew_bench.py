"""Single-tile maps on the one-chunk kernel vs k_gf_apply_skew (ecx_tune
"skew_chunks" 2 / 4): RS(12,4) 2-erasure decode in place at 4 MiB shard pitches with
and without a 4 KiB pad and at 1 MiB, LRC encode / repair, and the Clay(4,2) repair.
Interleaved rounds in one process, median algorithmic GB/s.

    python scripts/skew_bench.py [--rounds 5 --reps 5]
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

SKEWS = (0, 2, 4)


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
    for L, pad, S in ((4 << 20, 0, 256), (4 << 20, 4096, 256), (1 << 20, 0, 1024), (1 << 20, 4096, 1024)):
        p = L + pad
        pool = torch.empty((S, 16, p), dtype=torch.uint8, device="cuda")
        ecx.fill_random(pool, pool.numel(), 1)
        cases.append((f"RS(12,4) decode {{0,1}} in place, {L >> 20} MiB shards, pitch +{pad}", 14 * L * S,
                      lambda pool=pool, p=p, S=S, L=L: dmap.apply_batch(pool, 16 * p, p, pool, 16 * p, p, S, L), pool))
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
    CB, P = 32768, 1 << 14
    cpool = torch.empty((P, 48, CB), dtype=torch.uint8, device="cuda")
    ecx.fill_random(cpool, cpool.numel(), 3)
    cout = torch.empty((P, 8, CB), dtype=torch.uint8, device="cuda")
    rep = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
    cases.append(("Clay(4,2) repair e=1, 32 KiB", 28 * CB * P,
                  lambda: rep.performCodingBatch(cpool, 48 * CB, CB, cout, 8 * CB, CB, P, CB), (cpool, cout, rep)))
    res = {(c[0], k): [] for c in cases for k in SKEWS}
    for _ in range(args.rounds):
        for name, nbytes, fn, _keep in cases:
            for k in SKEWS:
                ecx.tune("skew_chunks", k)
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[(name, k)].append(nbytes / (e0.elapsed_time(e1) / args.reps * 1e-3) / 1e9)
    ecx.tune("skew_chunks", 1)
    for (name, k), v in res.items():
        med = statistics.median(v)
        print(json.dumps({"case": name, "skew_chunks": k, "GBps_median": round(med, 1), "frac": round(med / 8000, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
