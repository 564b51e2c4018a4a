"""Clay(10,4) single-node repair (shortened Clay(12,4), node 3 erased) with large sub-chunks at
several sub-chunk pitches: the batch API takes the sub-chunk stride apart from the sub-chunk size
(ecx_clay_perform_coding_batch in_sub_stride / buf_size), so a caller can pad 1 MiB sub-chunks off
the power-of-two strides whose address bits the HBM interleave does not spread.
Interleaved rounds in one process, one pool per pitch holding the same bytes, the repaired outputs
compared across pitches (bit-exact, or the script stops); fraction of 8 TB/s over the algorithmic
bytes (832 helper + 256 repaired sub-chunks per stripe).

    python scripts/clay_pitch_probe.py [--sub 1048576] [--pads 0,4096,8192,65536] [--stripes 6]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sub", type=int, default=1 << 20)
    ap.add_argument("--pads", default="0,4096,8192,12288,65536")
    ap.add_argument("--stripes", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--erased", type=int, default=3)
    args = ap.parse_args()
    import torch
    ecx = rpamd.load()
    k, m, v, a, B, S, e = 10, 4, 2, 256, args.sub, args.stripes, args.erased
    n = k + m
    step = ecx.ClayCodeErasureDecodingStep([e], k, m, virtualUnits=v)
    info = step.map().info()
    moved = (info["n_in"] + info["n_out"]) * B * S
    pads = [int(x) for x in args.pads.split(",")]
    src = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(src, src.numel(), 31)  # non-codeword stripes: the map is what is compared
    pools, outs = [], []
    for pad in pads:
        p = B + pad
        pool = torch.empty((S, n * a, p), dtype=torch.uint8, device="cuda")
        pool[:, :, :B].copy_(src)
        pools.append(pool)
        outs.append(torch.empty((S, a, B), dtype=torch.uint8, device="cuda"))
    del src
    res, ref = {}, None
    for _ in range(args.rounds):
        for i, pad in enumerate(pads):
            p = B + pad
            launch = lambda: step.performCodingBatch(pools[i], n * a * p, p, outs[i], a * B, B, S, B)  # noqa: E731
            launch()
            torch.cuda.synchronize()
            if ref is None:
                ref = outs[i].clone()
            elif not bool(torch.equal(outs[i], ref)):
                raise SystemExit("pad %d: repaired bytes differ" % pad)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                launch()
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(pad, []).append(moved / (e0.elapsed_time(e1) / args.reps * 1e-3) / 1e9)
    for pad in pads:
        med = statistics.median(res[pad])
        print(json.dumps({"case": "clay104", "sub_bytes": B, "sub_pitch": B + pad, "pad": pad, "stripes": S,
                          "GBps": round(med, 1), "frac": round(med / 8000, 4),
                          "all": [round(x / 8000, 4) for x in res[pad]], "kernel": ecx.last_kernel()}), flush=True)


if __name__ == "__main__":
    main()
