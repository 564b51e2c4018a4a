"""The many-stream RS maps on the real kernels, per shard pitch, under launch-shape and
unit-order knobs (include/ecx_tune.h): RS(12,4) 2-erasure decodeMissing in place (12
shards read, 2 written) and RS(17,3) encodeParity in place (17 read, 3 written).
Interleaved rounds, median algorithmic GB/s as a fraction of 8 TB/s; every setting's
output is compared with the default's (bit-exact, or the script stops).  Each setting runs
on its own fresh map; with no knobs set (the default: ecx_tune "layout_select" 1) its first
calls are the per-layout shape selection, run with a sync after each until it has chosen.

    python scripts/layout_sweep.py [--set orders] [--rounds 3 --reps 3] [--cases rs124,rs173]

The unit orders are the ones scripts/addr_probe.hip prices on the bare access pattern:
stagger G (G stripes interleaved at G chunk offsets) and runs of R units per XCD.
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402

TOTAL = 16 << 30
RS124 = [(4 << 20, 0), (4 << 20, 4096), (1 << 20, 0), (1 << 20, 4096), (3 << 20, 0), (8 << 20, 0), (4 << 20, 65536),
         (1 << 19, 0)]
RS173 = [(200000, 0), (262144, 0)]
CLAY42 = [(32768, 0), (65536, 0), (262144, 0), (1 << 20, 0), (4 << 20, 0), (16384, 0)]
DEFAULTS = {"depth": 0, "block_threads": 0, "small_tiles": 2, "skew_chunks": 1, "xcd_group": 0, "xcd_run": 8,
            "xcd_misaligned": 1, "stagger": 0, "chunk_major": 0, "layout_select": 1}
SETS = {
    "orders": [{}, {"stagger": 2}, {"stagger": 4}, {"stagger": 8}, {"stagger": 16},
               {"xcd_group": 3, "xcd_run": 32}, {"stagger": 8, "xcd_group": 3, "xcd_run": 32},
               {"stagger": 4, "xcd_group": 3, "xcd_run": 32}],
    "shapes": [{}, {"skew_chunks": 0, "block_threads": 256}, {"skew_chunks": 0, "block_threads": 64},
               {"skew_chunks": 4}, {"skew_chunks": 0, "block_threads": 256, "stagger": 8},
               {"skew_chunks": 0, "block_threads": 64, "stagger": 8}, {"skew_chunks": 4, "stagger": 8},
               {"skew_chunks": 0, "block_threads": 256, "stagger": 4}, {"skew_chunks": 0, "block_threads": 64, "stagger": 4},
               {"skew_chunks": 0, "block_threads": 256, "depth": 16}, {"skew_chunks": 0, "block_threads": 256, "depth": 16, "stagger": 8}],
    "default": [{}],
    # the per-layout selection (default) against the static rules alone
    "select": [{}, {"layout_select": 0}],
    # unit orders without the XCD runs that misaligned layouts get by default (RS(17,3) at 200,000 B)
    # ring depth / accumulator rows under the stagger, one-wave and 4 KiB workgroups (4 MiB pitch)
    "depth": [{}, {"layout_select": 0},
              {"block_threads": 64, "stagger": 2, "depth": 4}, {"block_threads": 64, "stagger": 2},
              {"block_threads": 64, "stagger": 4, "depth": 4},
              {"block_threads": 256, "skew_chunks": 0, "small_tiles": 1, "depth": 12, "stagger": 2},
              {"block_threads": 256, "skew_chunks": 0, "small_tiles": 1, "depth": 8, "stagger": 2},
              {"block_threads": 256, "skew_chunks": 0, "small_tiles": 1, "depth": 12},
              {"block_threads": 256, "skew_chunks": 0, "depth": 12, "stagger": 2},
              {"block_threads": 256, "skew_chunks": 0, "depth": 16, "stagger": 2},
              {"skew_chunks": 4, "stagger": 2}, {"skew_chunks": 2, "stagger": 2}, {"skew_chunks": 2}],
    # bytes in flight per workgroup: shallower rings (depth 16 costs 20 % on RS(17,3))
    "inflight": [{}, {"layout_select": 0}, {"depth": 4, "layout_select": 0}, {"depth": 2, "layout_select": 0},
                 {"depth": 4, "block_threads": 64}, {"depth": 4, "skew_chunks": 0, "block_threads": 256},
                 {"depth": 2, "skew_chunks": 0, "block_threads": 256}, {"depth": 12, "layout_select": 0}],
    # the skewed-chunk kernel on colliding and non-colliding pitches: what the rotation repairs
    "skewcheck": [{}, {"skew_chunks": 4, "block_threads": 256}, {"skew_chunks": 2, "block_threads": 256},
                  {"skew_chunks": 0, "block_threads": 256}, {"skew_chunks": 0, "block_threads": 64},
                  {"skew_chunks": 4, "block_threads": 64}, {"skew_chunks": 2, "block_threads": 64},
                  {"skew_chunks": 4, "block_threads": 64, "depth": 4}, {"skew_chunks": 4, "block_threads": 64, "stagger": 2}],
    # the 8-row Clay(4,2) repair map across sub-chunk sizes
    "clay": [{}, {"block_threads": 64}, {"skew_chunks": 2}, {"stagger": 2}, {"stagger": 8},
             {"block_threads": 64, "stagger": 2}, {"block_threads": 64, "stagger": 8}, {"chunk_major": 1},
             {"xcd_group": 3, "xcd_run": 32}],
    "misaligned": [{}, {"layout_select": 0}, {"xcd_misaligned": 0, "layout_select": 0},
                   {"stagger": 8, "xcd_misaligned": 0}, {"stagger": 4, "xcd_misaligned": 0},
                   {"stagger": 16, "xcd_misaligned": 0}, {"stagger": 8, "xcd_misaligned": 0, "block_threads": 64},
                   {"xcd_group": 3, "xcd_run": 32, "layout_select": 0}, {"xcd_group": 3, "xcd_run": 128, "layout_select": 0}],
}


def run_case(ecx, torch, buf, kind, L, pad, knobs, rounds, reps):
    p = L + pad
    if kind == "rs124":
        n, S = 16, min(4096, TOTAL // (16 * p))
        mat, ins, outs = ecx.ReedSolomon.create(12, 4).decode_map([False, False] + [True] * 14).matrix()
        out_view = lambda: buf[:S * n * p].view(S, n, p)[:, :2, :L]  # noqa: E731
        moved = (12 + 2) * L * S
    elif kind == "clay42":  # Clay(4,2) repair of node 1 (8 x 20), B-byte sub-chunks: [S][48][B] -> [S][8][B]
        n, S = 48, min(1 << 15, (TOTAL * 6 // 7) // (48 * p))
        mat, ins, outs = ecx.ClayCodeErasureDecodingStep([1], 4, 2).map().matrix()
        obase = S * n * p
        gm0 = ecx.GfMap.from_matrix(mat, in_slot=[int(i) for i in ins], out_slot=[int(o) for o in outs])
        out_view = lambda: buf[obase:obase + S * 8 * p].view(S, 8, p)[:, :, :L]  # noqa: E731
        moved = 28 * L * S
        del gm0
    else:
        n, S = 20, min(8192, TOTAL // (20 * p))
        mat, ins, outs = ecx.ReedSolomon.create(17, 3).encode_map().matrix()
        out_view = lambda: buf[:S * n * p].view(S, n, p)[:, 17:, :L]  # noqa: E731
        moved = 20 * L * S
    # a fresh map per setting, so each one's per-layout launch-shape selection starts anew
    maps = [ecx.GfMap.from_matrix(mat, in_slot=[int(i) for i in ins], out_slot=[int(o) for o in outs])
            for _ in knobs]
    res, kern, ref, picks = {}, {}, None, {}
    for _ in range(rounds):
        for i, kn in enumerate(knobs):
            gm = maps[i]
            if kind == "clay42":
                ob = buf[S * n * p:]
                launch = lambda: gm.apply_batch(buf, n * p, p, ob, 8 * p, p, S, L)  # noqa: E731
            else:
                launch = lambda: gm.apply_batch(buf, n * p, p, buf, n * p, p, S, L)  # noqa: E731
            for k, v in kn.items():
                ecx.tune(k, v)
            try:
                for _ in range(64):  # the layout selection's timed first calls (if it runs)
                    launch()
                    torch.cuda.synchronize()
                    if gm.layout_choice(p) != -1 or kn.get("layout_select", 1) == 0 or len(kn) > 0:
                        break
                kern[i] = ecx.last_kernel()
                picks[i] = gm.layout_choice(p)
                o = out_view()
                if ref is None:
                    ref = o.clone()
                elif not bool(torch.equal(o, ref)):
                    raise SystemExit("output differs under %s (%s pitch %d)" % (kn, kind, p))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    launch()
                e1.record()
                torch.cuda.synchronize()
            finally:
                for k in kn:
                    ecx.tune(k, DEFAULTS[k])
            res.setdefault(i, []).append(moved / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9)
    for i, kn in enumerate(knobs):
        med = statistics.median(res[i])
        print(json.dumps({"case": kind, "shard": L, "pad": pad, "stripes": S, "knobs": kn, "GBps": round(med, 1),
                          "frac": round(med / 8000, 4), "kernel": kern[i], "layout_choice": picks[i]}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="orders", choices=sorted(SETS))
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cases", default="rs124,rs173")
    ap.add_argument("--pitches", default=None, help="comma-separated shard+pad byte pairs as L:pad (default: all)")
    args = ap.parse_args()
    import torch
    ecx = rpamd.load(shape_knobs=True)
    buf = torch.empty(TOTAL, dtype=torch.uint8, device="cuda")
    ecx.fill_random(buf, buf.numel(), 7)
    for kind in args.cases.split(","):
        cases = {"rs124": RS124, "rs173": RS173, "clay42": CLAY42}[kind]
        if args.pitches:
            cases = [tuple(int(x) for x in c.split(":")) for c in args.pitches.split(",")]
        for L, pad in cases:
            run_case(ecx, torch, buf, kind, L, pad, SETS[args.set], args.rounds, args.reps)


if __name__ == "__main__":
    main()
