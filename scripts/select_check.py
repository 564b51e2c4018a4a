"""How well the per-layout launch-shape selection (ecx_tune "layout_select") predicts the
steady state, RS(12,4) 2-erasure decode in place: for each shard pitch, several fresh maps
run the selection (a sync after each call, as layout_sweep.py does) and report their choice
and per-candidate median times; then every candidate, forced through the tune knobs, is
timed both ways -- single launches from an idle GPU (what a selection probe sees) and
back-to-back batches (what a caller's stream sees) -- in interleaved rounds.

    python scripts/select_check.py [--pitches 262144:0,4194304:0] [--maps 4] [--rounds 5]
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
# launch_apply_core's pick codes (kernels.hip kLayoutCand) as tune knobs
FORCED = {-1: {"layout_select": 0}, 0: {"skew_chunks": 0, "block_threads": 256}, 1: {"skew_chunks": 4},
          2: {"skew_chunks": 0, "block_threads": 64}, 18: {"skew_chunks": 0, "block_threads": 64, "stagger": 2},
          66: {"skew_chunks": 0, "block_threads": 64, "stagger": 8},
          32: {"skew_chunks": 0, "block_threads": 256, "stagger": 4}}
DEFAULTS = {"layout_select": 1, "skew_chunks": 1, "block_threads": 0, "stagger": 0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pitches", default="262144:0,4194304:0,1048576:4096")
    ap.add_argument("--maps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import torch
    ecx = rpamd.load(shape_knobs=True)
    buf = torch.empty(TOTAL, dtype=torch.uint8, device="cuda")
    ecx.fill_random(buf, buf.numel(), 7)
    mat, ins, outs = ecx.ReedSolomon.create(12, 4).decode_map([False, False] + [True] * 14).matrix()
    for spec in args.pitches.split(","):
        L, pad = (int(x) for x in spec.split(":"))
        p, n = L + pad, 16
        S = min(4096, TOTAL // (n * p))
        moved = 14 * L * S

        def launch(gm):
            gm.apply_batch(buf, n * p, p, buf, n * p, p, S, L)

        for i in range(args.maps):
            gm = ecx.GfMap.from_matrix(mat, in_slot=[int(x) for x in ins], out_slot=[int(o) for o in outs])
            for _ in range(64):
                launch(gm)
                torch.cuda.synchronize()
                if gm.layout_choice(p) != -1:
                    break
            choice, ms = gm.layout_choice(p, with_times=True)
            print(json.dumps({"pitch": p, "shard": L, "map": i, "choice": choice,
                              "frac_by_cand": [round(moved / (t * 1e-3) / 8e12, 4) for t in ms if t > 0]}), flush=True)
        gm = ecx.GfMap.from_matrix(mat, in_slot=[int(x) for x in ins], out_slot=[int(o) for o in outs])
        single, batch = {}, {}
        for _ in range(args.rounds):
            for code, kn in FORCED.items():
                for k, v in kn.items():
                    ecx.tune(k, v)
                try:
                    launch(gm)
                    torch.cuda.synchronize()
                    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                    e[0].record()
                    launch(gm)
                    e[1].record()
                    torch.cuda.synchronize()
                    e[2].record()
                    for _ in range(3):
                        launch(gm)
                    e[3].record()
                    torch.cuda.synchronize()
                finally:
                    for k in kn:
                        ecx.tune(k, DEFAULTS[k])
                single.setdefault(code, []).append(moved / (e[0].elapsed_time(e[1]) * 1e-3) / 8e12)
                batch.setdefault(code, []).append(moved / (e[2].elapsed_time(e[3]) / 3 * 1e-3) / 8e12)
        for code in FORCED:
            print(json.dumps({"pitch": p, "shard": L, "code": code, "knobs": FORCED[code],
                              "single_frac": round(statistics.median(single[code]), 4),
                              "batch_frac": round(statistics.median(batch[code]), 4)}), flush=True)


if __name__ == "__main__":
    main()
