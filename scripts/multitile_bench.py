"""Multi-tile maps (inputs re-read across the tiles of a (stripe, chunk) unit):
launch-shape A/B, interleaved rounds in one process, median GB/s (algorithmic
bytes).  Modes:
    waves   -- k_gf_apply_lds: one workgroup per group of tiles, input union staged via LDS
    tiles   -- k_gf_apply: one workgroup per tile, identity block order (default)
    tiles_sgpr    -- as tiles, every split-table dword from SGPRs (lds_tables 0)
    tiles_lds_all -- as tiles, low table dwords from LDS for single-tile maps too (lds_tables 2)
    tiles_sc      -- as tiles, output stores `nt sc0 sc1` (store_scope 1)
    tiles_cm      -- as tiles, chunk-major block order (chunk_major 1)
    tiles_w64     -- as tiles, one-wave workgroups over 1 KiB chunks (block_threads 64)
    grp     -- k_gf_apply_grp: tile groups in one workgroup, each wave loading its own entries
    tiles_d2      -- as tiles_sgpr, load ring of 2 (63 VGPRs, 8 waves per SIMD)
    tiles_d4      -- as tiles, load ring of 4 (6 waves per SIMD)
    wide    -- k_gf_apply_wide: pairs of 8-row tiles sharing inputs in one workgroup (wide_tiles 2 = forced)
    tiles2  -- k_gf_apply with xcd_group 2 (whole units per XCD)

    python scripts/multitile_bench.py                          # all configs x all modes
    python scripts/multitile_bench.py --only clay104 --mode tiles --reps 2 --rounds 1   # one shape (PMC runs)
"""
import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402


def cases(ecx, torch, only):
    out = []
    if only in (None, "clay104"):
        k, m, v, B, S = 10, 4, 2, 4096, 2048
        n, a = 14, 256
        pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
        ecx.fill_random(pool, pool.numel(), 3)
        o = torch.empty((S, a, B), dtype=torch.uint8, device="cuda")
        step = ecx.ClayCodeErasureDecodingStep([3], k, m, virtualUnits=v)
        inf = step.map().info()
        out.append(("clay104 repair e=3, 4 KiB sub-chunks", (inf["n_in"] + inf["n_out"]) * B * S,
                    lambda pool=pool, o=o, step=step, n=n, a=a, B=B, S=S:
                    step.performCodingBatch(pool, n * a * B, B, o, a * B, B, S, B), (pool, o, step)))
    if only in (None, "clay42enc"):
        B, P = 32768, 1 << 13
        pool = torch.empty((P, 48, B), dtype=torch.uint8, device="cuda")
        ecx.fill_random(pool, pool.numel(), 1)
        par = torch.empty((P, 16, B), dtype=torch.uint8, device="cuda")
        enc = ecx.ClayCodeErasureDecodingStep([4, 5], 4, 2)
        out.append(("clay42 encode, 32 KiB", 48 * B * P,
                    lambda pool=pool, par=par, enc=enc, B=B, P=P:
                    enc.performCodingBatch(pool, 48 * B, B, par, 16 * B, B, P, B), (pool, par, enc)))
    if only in (None, "clay42multi"):
        B, P = 32768, 1 << 13
        pool = torch.empty((P, 48, B), dtype=torch.uint8, device="cuda")
        ecx.fill_random(pool, pool.numel(), 5)
        o = torch.empty((P, 16, B), dtype=torch.uint8, device="cuda")
        mrep = ecx.ClayCodeErasureDecodingStep([0, 3], 4, 2)
        inf = mrep.map().info()
        out.append(("clay42 2-erasure repair {0,3}, 32 KiB", (inf["n_in"] + inf["n_out"]) * B * P,
                    lambda pool=pool, o=o, mrep=mrep, B=B, P=P:
                    mrep.performCodingBatch(pool, 48 * B, B, o, 16 * B, B, P, B), (pool, o, mrep)))
    if only in (None, "clay42rep"):
        B, P = 32768, 1 << 13
        pool = torch.empty((P, 48, B), dtype=torch.uint8, device="cuda")
        ecx.fill_random(pool, pool.numel(), 4)
        o = torch.empty((P, 8, B), dtype=torch.uint8, device="cuda")
        rep = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
        out.append(("clay42 repair e=1, 32 KiB (single tile)", 28 * B * P,
                    lambda pool=pool, o=o, rep=rep, B=B, P=P:
                    rep.performCodingBatch(pool, 48 * B, B, o, 8 * B, B, P, B), (pool, o, rep)))
    return out


MODES = {"waves": {"wave_groups": 1, "xcd_group": 0, "lds_tables": 1, "store_scope": 0, "chunk_major": 0, "block_threads": 256, "depth": 0, "wide_tiles": 0},
         "tiles": {"wave_groups": 0, "xcd_group": 0, "lds_tables": 1, "store_scope": 0, "chunk_major": 0, "block_threads": 256, "depth": 0, "wide_tiles": 0},
         "tiles_sgpr": {"wave_groups": 0, "xcd_group": 0, "lds_tables": 0, "store_scope": 0, "chunk_major": 0, "block_threads": 256, "depth": 0, "wide_tiles": 0},
         "tiles_lds_all": {"wave_groups": 0, "xcd_group": 0, "lds_tables": 2, "store_scope": 0, "chunk_major": 0, "block_threads": 256, "depth": 0, "wide_tiles": 0},
         "tiles_sc": {"wave_groups": 0, "xcd_group": 0, "lds_tables": 1, "store_scope": 1, "chunk_major": 0, "block_threads": 256, "depth": 0, "wide_tiles": 0},
         "tiles_cm": {"wave_groups": 0, "xcd_group": 0, "lds_tables": 1, "store_scope": 0, "chunk_major": 1, "block_threads": 256, "depth": 0, "wide_tiles": 0},
         "tiles_w64": {"wave_groups": 0, "xcd_group": 0, "lds_tables": 1, "store_scope": 0, "chunk_major": 0,
                       "block_threads": 64, "depth": 0, "wide_tiles": 0},
         "grp": {"wave_groups": 2, "xcd_group": 0, "lds_tables": 1, "store_scope": 0, "chunk_major": 0,
                 "block_threads": 256, "depth": 0, "wide_tiles": 0},
         "tiles_d2": {"wave_groups": 0, "xcd_group": 0, "lds_tables": 0, "store_scope": 0, "chunk_major": 0,
                      "block_threads": 256, "depth": 2, "wide_tiles": 0},
         "tiles_d4": {"wave_groups": 0, "xcd_group": 0, "lds_tables": 1, "store_scope": 0, "chunk_major": 0,
                      "block_threads": 256, "depth": 4, "wide_tiles": 0},
         "wide": {"wave_groups": 0, "xcd_group": 0, "lds_tables": 1, "store_scope": 0, "chunk_major": 0,
                  "block_threads": 256, "depth": 0, "wide_tiles": 2},
         "tiles2": {"wave_groups": 0, "xcd_group": 2, "lds_tables": 1, "store_scope": 0, "chunk_major": 0, "block_threads": 256, "depth": 0, "wide_tiles": 0}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--mode", default=None, help="comma-separated subset of MODES")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import torch
    ecx = rpamd.load(shape_knobs=True)
    lib = ecx.lib()
    lib.ecx_tune.argtypes = [ctypes.c_char_p, ctypes.c_int]
    modes = args.mode.split(",") if args.mode else list(MODES)
    cs = cases(ecx, torch, args.only)
    res = {(c[0], x): [] for c in cs for x in modes}
    for _ in range(args.rounds):
        for name, nbytes, fn, _keep in cs:
            for x in modes:
                for key, val in MODES[x].items():
                    lib.ecx_tune(key.encode(), val)
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[(name, x)].append(nbytes / (e0.elapsed_time(e1) / args.reps * 1e-3) / 1e9)
    for key, val in MODES["tiles"].items():
        lib.ecx_tune(key.encode(), val)
    for (name, x), v in res.items():
        med = statistics.median(v)
        print(json.dumps({"case": name, "mode": x, "GBps_median": round(med, 1),
                          "frac": round(med / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
