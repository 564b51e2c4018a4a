"""RS(17,3) encodeParity over HBM-resident stripes of 200,000-byte shards (the shape of
the reference's published benchmark, ReedSolomonBenchmark.java:25-33) under launch-shape
knobs (include/ecx_tune.h): interleaved rounds, median algorithmic GB/s (17 read + 3
written shards per stripe) as a fraction of the 8 TB/s HBM peak, with the kernel each
setting ran.  Every setting's parity is compared with the default's.

    python scripts/rs173_knobs.py [--rounds 3 --reps 5]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402

K, M, SHARD = 17, 3, 200 * 1000
KNOBS = [{}, {"depth": 4}, {"depth": 12}, {"depth": 16}, {"depth": 20}, {"block_threads": 64}, {"small_tiles": 1},
         {"small_tiles": 1, "depth": 12}, {"skew_chunks": 2}, {"skew_chunks": 4}, {"nontemporal": 0}]
KNOBS_XCD = [{}, {"block_threads": 64}, {"xcd_group": 3, "xcd_run": 8}, {"xcd_group": 3, "xcd_run": 49},
             {"xcd_group": 3, "xcd_run": 196}, {"block_threads": 64, "xcd_group": 3, "xcd_run": 8},
             {"block_threads": 64, "xcd_group": 3, "xcd_run": 196}, {"chunk_major": 1}, {"xcd_misaligned": 0},
             {"block_threads": 256}]
KNOBS_SHAPES = [{}, {"block_threads": 64}, {"block_threads": 256}]
KNOBS_T256 = [{}, {"block_threads": 256}, {"block_threads": 256, "depth": 4}, {"block_threads": 256, "depth": 12},
              {"block_threads": 256, "depth": 16}, {"block_threads": 256, "depth": 20},
              {"block_threads": 256, "xcd_misaligned": 0}, {"block_threads": 256, "small_tiles": 1},
              {"block_threads": 256, "small_tiles": 1, "depth": 12}]
DEFAULTS = {"depth": 0, "block_threads": 0, "small_tiles": 2, "skew_chunks": 1, "nontemporal": 1, "xcd_group": 0,
            "xcd_run": 8, "chunk_major": 0, "xcd_misaligned": 1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--pad", type=int, default=0, help="bytes between shards")
    ap.add_argument("--shard", type=int, default=SHARD, help="shard bytes (the published benchmark: 200,000)")
    ap.add_argument("--k", type=int, default=17, help="data shards (RS(k, m) encode; default 17)")
    ap.add_argument("--m", type=int, default=3, help="parity shards (default 3)")
    ap.add_argument("--gib", type=float, default=None, help="size the stripe count to this many GiB of stripes")
    ap.add_argument("--set", default="knobs", choices=["knobs", "xcd", "default", "shapes", "t256"])
    args = ap.parse_args()
    knobs = {"knobs": KNOBS, "xcd": KNOBS_XCD, "default": [{}], "shapes": KNOBS_SHAPES, "t256": KNOBS_T256}[args.set]
    import torch
    ecx = rpamd.load(shape_knobs=True)
    K, M = args.k, args.m
    shard = args.shard
    p = shard + args.pad
    S = args.stripes if args.gib is None else max(1, int(args.gib * 2**30 / ((K + M) * p)))
    pool = torch.empty(S * (K + M) * p, dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 17)
    rs = ecx.ReedSolomon.create(K, M)
    res, kern, ref = {}, {}, None
    for _ in range(args.rounds):
        for i, kn in enumerate(knobs):
            for k, v in kn.items():
                ecx.tune(k, v)
            try:
                rs.encodeParityBatch(pool, (K + M) * p, p, S, 0, shard)
                torch.cuda.synchronize()
                kern[i] = ecx.last_kernel()
                par = pool.view(S, K + M, p)[:, K:, :shard]
                if ref is None:
                    ref = par.clone()
                elif not bool(torch.equal(par, ref)):
                    raise SystemExit("parity differs under %s" % kn)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    rs.encodeParityBatch(pool, (K + M) * p, p, S, 0, shard)
                e1.record()
                torch.cuda.synchronize()
            finally:
                for k in kn:
                    ecx.tune(k, DEFAULTS[k])
            res.setdefault(i, []).append((K + M) * shard * S / (e0.elapsed_time(e1) / args.reps * 1e-3) / 1e9)
    for i, kn in enumerate(knobs):
        med = statistics.median(res[i])
        print(json.dumps({"k": K, "m": M, "knobs": kn, "shard": shard, "pad": args.pad, "stripes": S, "GBps": round(med, 1), "frac": round(med / 8000, 4),
                          "kernel": kern[i]}), flush=True)


if __name__ == "__main__":
    main()
