"""Is a map's kernel bound by its arithmetic or by its memory traffic?

Runs each map next to a copy of itself with every non-zero coefficient set to 1.
The copy has the same tiles, entries, loads and stores, but every multiply-add
becomes one v_bitop3 instead of 3 v_perm + 2 v_bitop3 (kernels.hip apply_entry).
Same speed => memory-bound; much faster => VALU-bound.  Interleaved rounds,
median algorithmic GB/s (BASELINE.md section 3 bytes per unit).

    python scripts/ones_bench.py [--rounds 3 --reps 5]
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    ecx = rpamd.load()

    cases = []
    # shortened Clay(10,4) repair, 4 KiB sub-chunks
    k, m, v, B, S = 10, 4, 2, 4096, 2048
    n, a = 14, 256
    pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 3)
    o = torch.empty((S, a, B), dtype=torch.uint8, device="cuda")
    step = ecx.ClayCodeErasureDecodingStep([3], k, m, virtualUnits=v)
    cases.append(("clay104 repair", step.map(), pool, n * a * B, o, a * B, S, B))
    # Clay(4,2) encode and repair, 32 KiB
    B2, P = 32768, 1 << 13
    pool2 = torch.empty((P, 48, B2), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool2, pool2.numel(), 1)
    par = torch.empty((P, 16, B2), dtype=torch.uint8, device="cuda")
    cases.append(("clay42 encode", ecx.ClayCodeErasureDecodingStep([4, 5], 4, 2).map(), pool2, 48 * B2, par,
                  16 * B2, P, B2))
    cases.append(("clay42 repair", ecx.ClayCodeErasureDecodingStep([1], 4, 2).map(), pool2, 48 * B2, par,
                  16 * B2, P, B2))
    cases.append(("clay42 2-erasure repair {0,3}", ecx.ClayCodeErasureDecodingStep([0, 3], 4, 2).map(), pool2,
                  48 * B2, par, 16 * B2, P, B2))

    runs = []
    for name, gmap, inp, iss, out, oss, ns, nb in cases:
        M, ins, outs = gmap.matrix()
        ones = ecx.GfMap.from_matrix((M != 0).astype(np.uint8), in_slot=list(ins), out_slot=list(outs))
        info = gmap.info()
        nbytes = (info["n_in"] + info["n_out"]) * nb * ns
        for label, g in (("real", gmap), ("ones", ones)):
            runs.append((name, label, nbytes, lambda g=g, inp=inp, iss=iss, out=out, oss=oss, ns=ns, nb=nb:
                         g.apply_batch(inp, iss, nb, out, oss, nb, ns, nb), ones))
    res = {(r[0], r[1]): [] for r in runs}
    for _ in range(args.rounds):
        for name, label, nbytes, fn, _keep in runs:
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[(name, label)].append(nbytes / (e0.elapsed_time(e1) / args.reps * 1e-3) / 1e9)
    for (name, label), v in res.items():
        med = statistics.median(v)
        print(json.dumps({"case": name, "coefficients": label, "GBps_median": round(med, 1),
                          "frac": round(med / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
