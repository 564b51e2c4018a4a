"""Resident workgroups per CU for the single-tile composed maps (ecx_tune "occ_lds": dummy
LDS per k_gf_apply workgroup caps them at floor(160 KiB / occ_lds)): RS(k, m) encodes and
RS(12,4) decodes over several shard sizes and pitches, in place, default launch against
capped ones, interleaved rounds, median launch, algorithmic GB/s as a fraction of 8 TB/s.
Every capped run's outputs equal the default's.

    python scripts/occ_bench.py [--rounds 3 --reps 4] [--sets "occ_lds=0;occ_lds=40960"]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402

# (name, k, m, erased data shards (None = encode), shard bytes, pitch)
CASES = [("RS(17,3) encode", 17, 3, None, 200000, 200000), ("RS(17,3) encode", 17, 3, None, 262144, 262144),
         ("RS(10,4) encode", 10, 4, None, 1 << 20, 1 << 20), ("RS(12,4) encode", 12, 4, None, 4 << 20, (4 << 20) + 4096),
         ("RS(8,3) encode", 8, 3, None, 262144, 262144),
         ("RS(12,4) decode {0,1}", 12, 4, [0, 1], 4 << 20, (4 << 20) + 4096),
         ("RS(12,4) decode {0,1}", 12, 4, [0, 1], 4 << 20, 4 << 20),
         ("RS(12,4) decode {0,1}", 12, 4, [0, 1], 1 << 20, (1 << 20) + 4096),
         ("RS(12,4) decode {0,1}", 12, 4, [0, 1], 1 << 20, 1 << 20),
         ("RS(12,4) decode {3}", 12, 4, [3], 4 << 20, (4 << 20) + 4096)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--gib", type=float, default=16.0)
    ap.add_argument("--sets", default="occ_lds=0;occ_lds=40960;occ_lds=32768;block_threads=64,occ_lds=10240")
    args = ap.parse_args()
    sets = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in s.split(",") if kv) for s in args.sets.split(";")]
    import torch
    ecx = rpamd.load(shape_knobs=True)
    for name, k, m, erased, L, pitch in CASES:
        n = k + m
        rs = ecx.ReedSolomon.create(k, m)
        gmap = rs.encode_map() if erased is None else rs.decode_map([i not in erased for i in range(n)])
        _, _, outs = gmap.matrix()
        S = max(1, int(args.gib * 2**30 / (n * pitch)))
        pool = torch.empty((S, n, pitch), dtype=torch.uint8, device="cuda")
        ecx.fill_random(pool, pool.numel(), 5)
        algo = (gmap.info()["n_in"] + len(outs)) * L * S
        ref, times, kern = None, [[] for _ in sets], [None] * len(sets)
        for _ in range(args.rounds):
            for i, kn in enumerate(sets):
                for kk, vv in kn.items():
                    ecx.tune(kk, vv)
                try:
                    gmap.apply_batch(pool, n * pitch, pitch, pool, n * pitch, pitch, S, L)
                    torch.cuda.synchronize()
                    kern[i] = ecx.last_kernel()
                    got = pool[:, list(outs), :L]
                    if ref is None:
                        ref = got.clone()
                    elif not torch.equal(got, ref):
                        raise SystemExit("%s %s: outputs differ" % (name, kn))
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.reps):
                        gmap.apply_batch(pool, n * pitch, pitch, pool, n * pitch, pitch, S, L)
                    e1.record()
                    torch.cuda.synchronize()
                    times[i].append(e0.elapsed_time(e1) / args.reps)
                finally:
                    for kk in kn:
                        ecx.tune(kk, 0)
        for i, kn in enumerate(sets):
            ms = statistics.median(times[i])
            gbs = algo / (ms * 1e-3) / 1e9
            print(json.dumps({"case": name, "shard": L, "pitch": pitch, "set": kn, "stripes": S, "launch_ms": round(ms, 4),
                              "GBps": round(gbs, 1), "frac": round(gbs / 8000, 4), "kernel": kern[i]}), flush=True)
        del pool
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
