"""(Round 3 tool, kept for the provenance of profiles/r03_shape_trial_check.jsonl: the
skew_trial knob it drives was replaced in round 4 by the per-layout selection, ecx_tune
"layout_select", so it no longer runs; scripts/layout_sweep.py --set select is its successor.)

skew_trial (include/ecx_tune.h) against the kernels it chooses between: RS(12,4)
2-erasure decode in place at several shard pitches, each timed with the one-chunk
launch in 256-thread and in one-wave workgroups (skew_chunks 0, block_threads 256 / 64),
the skewed launch (skew_chunks 4), the static rules (skew_trial 0, the default) and the
trial (skew_trial 1: measured on the first batch of a fresh map at that pitch).
Interleaved rounds, median algorithmic GB/s (12 read + 2 written shards) as a fraction of
8 TB/s; a good rule matches the fastest of the first three at every pitch.

    python scripts/skew_trial_check.py [--rounds 3 --reps 3]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402

TOTAL = 24 << 30
CASES = [(1 << 20, 0), (1 << 20, 4096), (4 << 20, 0), (4 << 20, 4096), (4 << 20, 65536), (8 << 20, 0),
         (1 << 19, 0), (3 << 20, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    ecx = rpamd.load(shape_knobs=True)
    buf = torch.empty(TOTAL, dtype=torch.uint8, device="cuda")
    ecx.fill_random(buf, buf.numel(), 7)
    present = [False, False] + [True] * 14
    mat, ins, outs = ecx.ReedSolomon.create(12, 4).decode_map(present).matrix()
    res, picks = {}, {}
    variants = (("one_chunk_256", {"skew_chunks": 0, "block_threads": 256}), ("skewed", {"skew_chunks": 4}),
                ("one_chunk_64", {"skew_chunks": 0, "block_threads": 64}), ("static_rule", {}),
                ("trial", {"skew_trial": 1}))
    for rnd in range(args.rounds):
        for L, pad in CASES:
            p = L + pad
            S = min(4096, TOTAL // (16 * p))
            for name, knobs in variants:
                dmap = ecx.GfMap.from_matrix(mat, in_slot=[int(i) for i in ins],  # fresh: nothing measured
                                             out_slot=[int(o) for o in outs])
                for k, v in knobs.items():
                    ecx.tune(k, v)
                try:
                    dmap.apply_batch(buf, 16 * p, p, buf, 16 * p, p, S, L)  # the trial runs here
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.reps):
                        dmap.apply_batch(buf, 16 * p, p, buf, 16 * p, p, S, L)
                    e1.record()
                    torch.cuda.synchronize()
                    kern = ecx.last_kernel()
                finally:
                    ecx.tune("skew_chunks", 1)
                    ecx.tune("skew_trial", 0)
                    ecx.tune("block_threads", 0)
                res.setdefault((L, pad, name), []).append(14 * L * S / (e0.elapsed_time(e1) / args.reps * 1e-3) / 1e9)
                if name == "trial":
                    picks.setdefault((L, pad), []).append((dmap.skew_choice(p), kern))
    for L, pad in CASES:
        row = {"shard_KiB": L >> 10, "pad": pad}
        for name, _ in variants:
            row[name] = round(statistics.median(res[(L, pad, name)]) / 8000, 4)
        row["trial_picks"] = [c for c, _ in picks[(L, pad)]]
        row["trial_kernel"] = picks[(L, pad)][-1][1]
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
