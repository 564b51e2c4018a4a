"""Does the stride between a stripe's sub-chunks (exact powers of two vs padded)
change the achieved bandwidth?  Interleaved rounds in one process.  Same bytes,
same map; only the layout's strides differ."""
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402


def main():
    import torch
    ecx = rpamd.load()
    res = {}
    cases = []
    # Clay(4,2) e=1 repair, B = 32 KiB: sub-chunk stride B + pad, stripe stride 48 * sub stride (+ pad2)
    B, P = 32768, 1 << 13
    step = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
    for pad, spad in ((0, 0), (256, 0), (4096, 0), (0, 4096), (256, 256 * 48 + 512)):
        sub = B + pad
        st = 48 * sub + spad
        buf = torch.empty((P * st + 4096,), dtype=torch.uint8, device="cuda")
        ecx.fill_random(buf, buf.numel(), 1)
        out = torch.empty((P, 8, B), dtype=torch.uint8, device="cuda")
        cases.append((f"clay42 sub_stride=B+{pad} stripe_pad={spad}", P * 28 * B,
                      (lambda step=step, buf=buf, out=out, st=st, sub=sub:
                       step.performCodingBatch(buf, st, sub, out, 8 * B, B, P, B)), buf, out))
    # RS(12,4) 2-erasure decode, L = 4 MiB: shard stride L + pad
    L, S = 4 << 20, 128
    rs = ecx.ReedSolomon.create(12, 4)
    dmap = rs.decode_map([False, False] + [True] * 14)
    for pad in (0, 256, 4096, 65536 + 256):
        sh = L + pad
        buf = torch.empty((S * 16 * sh,), dtype=torch.uint8, device="cuda")
        ecx.fill_random(buf, buf.numel(), 2)
        cases.append((f"rs124 shard_stride=L+{pad}", S * 14 * L,
                      (lambda buf=buf, sh=sh: dmap.apply_batch(buf, 16 * sh, sh, buf, 16 * sh, sh, S, L)), buf, None))
    for name, *_ in cases:
        res[name] = []
    for _ in range(3):
        for name, nbytes, fn, *_ in cases:
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(nbytes / (e0.elapsed_time(e1) / 10 * 1e-3) / 1e9)
    for name, *_ in cases:
        print(json.dumps({"case": name, "GBps_median": round(statistics.median(res[name]), 1),
                          "frac": round(statistics.median(res[name]) / 8000, 4)}))


if __name__ == "__main__":
    main()
