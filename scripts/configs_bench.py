"""Secondary measurements: every BASELINE.json config on one MI355X, device
resident, as achieved algorithmic GB/s of the dominant kernel against the
8 TB/s HBM peak (BASELINE.md section 3 bytes per unit).  One JSON line per
config and launch shape; recorded in DESIGN.md (the bench.py headline is config 2).

All configs are set up first (about 100 GB of HBM), then timed in interleaved
rounds (each round: every config, `--reps` launches after one warm-up launch);
the reported time is the median round, so clock and thermal drift hit every
config alike.

    python scripts/configs_bench.py [--rounds 3] [--reps 5] [--sweep]
"""
import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402

PEAK = 8000.0
SWEEP = [(0, 1), (4, 1), (8, 1), (0, 0)]  # (load-ring depth, nontemporal); first = default (0 = per map)


def cases(ecx, torch):
    out = []
    # ---- config 2e: Clay(4,2) encode (stripe generation), 32 KiB sub-chunks
    B, P = 32768, 1 << 13
    pool = torch.empty((P, 48, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 1)
    par = torch.empty((P, 16, B), dtype=torch.uint8, device="cuda")
    enc = ecx.ClayCodeErasureDecodingStep([4, 5], 4, 2)
    out.append(("Clay(4,2) encode, 32 KiB (16x32 map)", 32 * B + 16 * B, P,
                lambda: enc.performCodingBatch(pool, 48 * B, B, par, 16 * B, B, P, B), {}, (pool, par, enc)))
    # ---- config 2 (the headline): Clay(4,2) single repair of node 1, 32 KiB
    rep = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
    rout = torch.empty((P, 8, B), dtype=torch.uint8, device="cuda")
    out.append(("Clay(4,2) single repair e=1, 32 KiB (headline map)", 28 * B, P,
                lambda: rep.performCodingBatch(pool, 48 * B, B, rout, 8 * B, B, P, B), {}, (rout, rep)))
    # ---- config 3: LRC 12+4 XOR groups, 64 KiB blocks: encode, and repair of block 2
    B3, S3 = 65536, 1 << 14
    lpool = torch.empty((S3, 16, B3), dtype=torch.uint8, device="cuda")
    ecx.fill_random(lpool, lpool.numel(), 2)
    encm = np.zeros((4, 16), np.uint8)
    for g in range(4):
        encm[g, 4 * g:4 * g + 3] = 1
    emap = ecx.GfMap.from_matrix(encm, in_slot=list(range(16)), out_slot=[3, 7, 11, 15])
    out.append(("LRC encode, 64 KiB blocks", 16 * B3, S3,
                lambda: emap.apply_batch(lpool, 16 * B3, B3, lpool, 16 * B3, B3, S3, B3), {}, (lpool, emap)))
    rmap = ecx.GfMap.from_matrix(np.array([[1, 1, 1]], np.uint8), in_slot=[0, 1, 3], out_slot=[0])
    lout = torch.empty((S3, 1, B3), dtype=torch.uint8, device="cuda")
    out.append(("LRC repair of block 2, 64 KiB", 4 * B3, S3,
                lambda: rmap.apply_batch(lpool, 16 * B3, B3, lout, B3, B3, S3, B3), {}, (lout, rmap)))
    # ---- config 4: shortened Clay(10,4), 1 MiB node block = 256 x 4 KiB, single repair
    k, m, v, B4, S4 = 10, 4, 2, 4096, 2048
    n, a = 14, 256
    cpool = torch.empty((S4, n * a, B4), dtype=torch.uint8, device="cuda")
    ecx.fill_random(cpool, cpool.numel(), 3)
    cout = torch.empty((S4, a, B4), dtype=torch.uint8, device="cuda")
    step = ecx.ClayCodeErasureDecodingStep([3], k, m, virtualUnits=v)
    inf = step.map().info()
    out.append(("Clay(10,4) shortened, 1 MiB blocks, single repair (e=3)", (inf["n_in"] + inf["n_out"]) * B4, S4,
                lambda: step.performCodingBatch(cpool, n * a * B4, B4, cout, a * B4, B4, S4, B4), {"map": inf},
                (cpool, cout, step)))
    # ---- config 5: RS(12,4), 4 MiB shards, erasures {0,1}, decoded in place.  A power-of-two
    # shard pitch puts the 12 streams of one byte position on the same HBM banks; a 4 KiB pad
    # per shard spreads them (profiles/r01_rs124.jsonl).
    L, S5 = 4 << 20, 256
    rs = ecx.ReedSolomon.create(12, 4)
    dmap = rs.decode_map([False, False] + [True] * 14)
    for pad, label in ((0, "in place, pitch 4 MiB"), (4096, "in place, pitch 4 MiB + 4 KiB")):
        Lp = L + pad
        rpool = torch.empty((S5, 16, Lp), dtype=torch.uint8, device="cuda")
        ecx.fill_random(rpool, rpool.numel(), 4)
        out.append(("RS(12,4) 2-erasure decode, 4 MiB", 14 * L, S5,
                    lambda rpool=rpool, Lp=Lp: dmap.apply_batch(rpool, 16 * Lp, Lp, rpool, 16 * Lp, Lp, S5, L),
                    {"layout": label}, (rpool, dmap, rs)))
    # ---- f4: multi-erasure Clay (doDecodeMulti), Clay(4,2) repair of nodes {0, 3}, 32 KiB
    mrep = ecx.ClayCodeErasureDecodingStep([0, 3], 4, 2)
    minf = mrep.map().info()
    mout = torch.empty((P, 16, B), dtype=torch.uint8, device="cuda")
    out.append(("Clay(4,2) 2-erasure repair {0,3} (doDecodeMulti), 32 KiB", (minf["n_in"] + minf["n_out"]) * B, P,
                lambda: mrep.performCodingBatch(pool, 48 * B, B, mout, 16 * B, B, P, B), {"map": minf}, (mout, mrep)))
    # ---- f2: one helper's decodeMissingSingle contribution along a repair chain, XOR-accumulated
    # into the 2 missing shards' partial sums: RS(12,4), 4 MiB shards; reads the helper's shard and
    # the 2 partials, writes the 2 partials (5 x 4 MiB per stripe).
    Sp = 128
    hin = torch.empty((Sp, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(hin, hin.numel(), 5)
    acc = torch.zeros((Sp, 2, L), dtype=torch.uint8, device="cuda")
    present = [False, False] + [True] * 14
    out.append(("RS(12,4) chain partial sum (decodeMissingSingle batch, accumulate), 4 MiB", 5 * L, Sp,
                lambda: rs.decodePartialBatch(present, 5, hin, L, acc, 2 * L, L, Sp, L, False), {}, (hin, acc)))
    return out


def knob_variants(args, ecx, torch, cs):
    """A/B/... of ecx_tune knob sets, interleaved: every round runs every variant over
    every case.  Each variant sets only the knobs it names, so name every knob that
    another variant changes (e.g. 'xcd_group=0;xcd_group=3,xcd_run=8')."""
    variants = [dict(kv.split("=") for kv in v.split(",") if kv) for v in args.knobs.split(";")]
    times = {(vi, i): [] for vi in range(len(variants)) for i in range(len(cs))}
    for _ in range(args.rounds):
        for vi, v in enumerate(variants):
            for k, val in v.items():
                ecx.tune(k, int(val))
            for i, (_name, _ub, _u, fn, _x, _keep) in enumerate(cs):
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[(vi, i)].append(e0.elapsed_time(e1) / args.reps * 1e-3)
    for vi, v in enumerate(variants):
        for i, (name, unit_bytes, units, _fn, extra, _keep) in enumerate(cs):
            sec = statistics.median(times[(vi, i)])
            gbs = unit_bytes * units / sec / 1e9
            d = {"config": name, "knobs": v, "ms_per_launch": round(sec * 1e3, 3), "GBps": round(gbs, 1),
                 "frac_of_peak": round(gbs / PEAK, 4), "rounds": args.rounds, "reps": args.reps}
            d.update(extra)
            print(json.dumps(d), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sweep", action="store_true", help="also the non-default launch shapes of SWEEP")
    ap.add_argument("--depths", default=None, help="comma list of ring depths to sweep (nt 1), e.g. 0,8,12,20")
    ap.add_argument("--knobs", default=None, help="variants of ecx_tune knobs, interleaved inside every round: "
                    "'k=v,k=v;k=v' (';' separates variants, '' = defaults)")
    ap.add_argument("--only", default=None, help="substring filter on the config names")
    args = ap.parse_args()
    import torch
    ecx = rpamd.load(shape_knobs=True)
    lib = ecx.lib()
    lib.ecx_tune.argtypes = [ctypes.c_char_p, ctypes.c_int]
    cs = cases(ecx, torch)
    if args.only:
        cs = [c for c in cs if any(o in c[0] for o in args.only.split("|"))]
    if args.knobs is not None:
        return knob_variants(args, ecx, torch, cs)
    shapes = SWEEP if args.sweep else SWEEP[:1]
    if args.depths:
        shapes = [(int(d), 1) for d in args.depths.split(",")]
    for depth, nt in shapes:
        lib.ecx_tune(b"depth", depth)
        lib.ecx_tune(b"nontemporal", nt)
        times = {i: [] for i in range(len(cs))}
        for _ in range(args.rounds):
            for i, (_name, _ub, _u, fn, _x, _keep) in enumerate(cs):
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[i].append(e0.elapsed_time(e1) / args.reps * 1e-3)
        for i, (name, unit_bytes, units, _fn, extra, _keep) in enumerate(cs):
            sec = statistics.median(times[i])
            gbs = unit_bytes * units / sec / 1e9
            d = {"config": name, "units": units, "bytes_per_unit": unit_bytes, "ms_per_launch": round(sec * 1e3, 3),
                 "GBps": round(gbs, 1), "GiBps": round(unit_bytes * units / sec / 2**30, 1),
                 "frac_of_peak": round(gbs / PEAK, 4), "rounds": args.rounds, "reps": args.reps}
            d.update(extra)
            d.update(depth=depth, nontemporal=nt)
            print(json.dumps(d), flush=True)
    lib.ecx_tune(b"depth", 0)
    lib.ecx_tune(b"nontemporal", 1)


if __name__ == "__main__":
    main()
