"""Would copying whole spans (the used sub-chunks plus the erased node's one-slot holes between them)
beat one strided copy per run on the host pipe?  Shortened Clay(10,4), node 3: its 832 helper
sub-chunks lie in planes 192-255, 65 runs per stripe with one-slot holes; the same map over the
896-slot span (zero columns for the holes) moves 7.7 % more bytes in ONE strided copy per chunk.
Both from one pinned host buffer, interleaved, outputs compared; prints GiB/s of algorithmic bytes.

    python scripts/clay_span_probe.py [--stripes 200] [--rounds 4]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--erased", type=int, default=3)
    args = ap.parse_args()
    ecx = rpamd.load()
    k, m, v, a, B, S = 10, 4, 2, 256, 4096, args.stripes
    n = k + m
    step = ecx.ClayCodeErasureDecodingStep([args.erased], k, m, virtualUnits=v)
    M, ins, outs = step.map().matrix()
    lo, hi = int(ins.min()), int(ins.max())
    span = np.arange(lo, hi + 1, dtype=np.int32)
    Ms = np.zeros((M.shape[0], len(span)), np.uint8)
    Ms[:, ins - lo] = M
    smap = ecx.GfMap.from_matrix(Ms, span, outs)
    hb = ecx.HostBuffer(S * n * a * B)
    pool = hb.array
    rng = np.random.default_rng(5)
    for s in range(S):
        pool[s * n * a * B:(s + 1) * n * a * B] = rng.integers(0, 256, n * a * B, dtype=np.uint8)
    o1, o2 = ecx.HostBuffer(S * a * B), ecx.HostBuffer(S * a * B)
    moved = (len(ins) + a) * B * S
    res = {"runs": [], "span": []}
    for r in range(args.rounds + 1):
        for name in ("runs", "span") if r % 2 == 0 else ("span", "runs"):
            t0 = time.perf_counter()
            if name == "runs":
                step.performCodingBatchHost(pool, n * a * B, B, o1.array, a * B, B, S, B)
            else:
                smap.apply_batch_host(pool, n * a * B, B, o2.array, a * B, B, S, B)
            dt = time.perf_counter() - t0
            if r:
                res[name].append(moved / dt / 2**30)
        if r == 0 and not np.array_equal(o1.array, o2.array):
            raise SystemExit("span map output differs")
    print(json.dumps({"case": "clay104 node %d" % args.erased, "stripes": S, "used_slots": len(ins),
                      "span_slots": len(span), "GiBps_runs": [round(x, 2) for x in res["runs"]],
                      "GiBps_span": [round(x, 2) for x in res["span"]]}))


if __name__ == "__main__":
    main()
