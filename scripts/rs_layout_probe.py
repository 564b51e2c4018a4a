"""Where an in-place RS encode loses against its read/write-mix model: RS(17,3) encodeParity
(200,000-B shards, the published shape) and RS(12,4) 2-erasure decode (4 MiB + 4 KiB pitch)
run as the same GF map under different layouts and store policies, interleaved rounds,
median launch, algorithmic GB/s as a fraction of 8 TB/s:

  inplace     parity / repaired shards written back into the stripe (the API's layout)
  separate    the same reads, outputs to a separate [S][m][L] buffer
  compact     data shards only in [S][k][L], outputs to a separate buffer
  inplace+sc  in place, output stores `nt sc0 sc1` (ecx_tune store_scope 1)

Every layout's outputs are compared with the in-place run's.

    python scripts/rs_layout_probe.py [--rounds 4 --reps 5] [--case rs173|rs124|both]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402


def run_case(ecx, torch, name, k, m, L, pitch, present, rounds, reps, gib):
    n = k + m
    rs = ecx.ReedSolomon.create(k, m)
    if present is None:  # encode: data slots 0..k-1 -> parity slots k..n-1
        mat, ins, outs = rs.encode_map().matrix()
    else:
        mat, ins, outs = rs.decode_map(present).matrix()
    S = max(1, int(gib * 2**30 / (n * pitch)))
    pool = torch.empty((S, n, pitch), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 3)
    sep = torch.empty((S, len(outs), L), dtype=torch.uint8, device="cuda")
    compact = torch.empty((S, len(ins), L), dtype=torch.uint8, device="cuda")
    compact.copy_(pool[:, list(ins), :L])
    m_inplace = ecx.GfMap.from_matrix(mat, in_slot=list(ins), out_slot=list(outs))
    m_sep = ecx.GfMap.from_matrix(mat, in_slot=list(ins), out_slot=list(range(len(outs))))
    m_compact = ecx.GfMap.from_matrix(mat, in_slot=list(range(len(ins))), out_slot=list(range(len(outs))))
    algo = (len(ins) + len(outs)) * L * S

    def inplace():
        m_inplace.apply_batch(pool, n * pitch, pitch, pool, n * pitch, pitch, S, L)

    def separate():
        m_sep.apply_batch(pool, n * pitch, pitch, sep, len(outs) * L, L, S, L)

    def compact_run():
        m_compact.apply_batch(compact, len(ins) * L, L, sep, len(outs) * L, L, S, L)

    variants = [("inplace", inplace, {}), ("separate", separate, {}), ("compact", compact_run, {}),
                ("inplace+sc", inplace, {"store_scope": 1}), ("separate+sc", separate, {"store_scope": 1})]
    inplace()
    torch.cuda.synchronize()
    ref = pool[:, list(outs), :L].clone()
    times = {v[0]: [] for v in variants}
    kern = {}
    for _ in range(rounds):
        for vname, fn, knobs in variants:
            for kk, vv in knobs.items():
                ecx.tune(kk, vv)
            try:
                fn()
                torch.cuda.synchronize()
                kern[vname] = ecx.last_kernel()
                got = pool[:, list(outs), :L] if vname.startswith("inplace") else sep
                if not torch.equal(got, ref):
                    raise SystemExit("%s %s: outputs differ" % (name, vname))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[vname].append(e0.elapsed_time(e1) / reps)
            finally:
                for kk in knobs:
                    ecx.tune(kk, 0)
    for vname, _, _ in variants:
        ms = statistics.median(times[vname])
        gbs = algo / (ms * 1e-3) / 1e9
        print(json.dumps({"case": name, "layout": vname, "stripes": S, "pitch": pitch, "launch_ms": round(ms, 4),
                          "GBps": round(gbs, 1), "frac": round(gbs / 8000, 4), "kernel": kern[vname]}), flush=True)
    del pool, sep, compact
    torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--gib", type=float, default=16.0)
    ap.add_argument("--case", default="both", choices=["rs173", "rs124", "both"])
    args = ap.parse_args()
    import torch
    ecx = rpamd.load(shape_knobs=True)
    if args.case in ("rs173", "both"):
        for pitch in (200000, 262144):
            run_case(ecx, torch, "RS(17,3) encode", 17, 3, min(pitch, 200000) if pitch == 200000 else pitch, pitch,
                     None, args.rounds, args.reps, args.gib)
    if args.case in ("rs124", "both"):
        L = 4 << 20
        run_case(ecx, torch, "RS(12,4) decode {0,1}", 12, 4, L, L + 4096, [False, False] + [True] * 14, args.rounds,
                 args.reps, args.gib * 2)


if __name__ == "__main__":
    main()
