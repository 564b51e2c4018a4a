"""RS(12,4) 2-erasure decode (BASELINE config 5) launch/layout A/B, interleaved
rounds in one process, median algorithmic GB/s (12 shards read + 2 written per
stripe).  Variants: in place vs separate output, shard pitch L vs L + 4 KiB,
shard length 4 MiB / 1 MiB / 256 KiB (same total bytes), ring depth 4 vs 8, and
block order stripe-major vs chunk-major (ecx_tune "chunk_major")."""
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402


def main():
    import torch
    ecx = rpamd.load(shape_knobs=True)
    rs = ecx.ReedSolomon.create(12, 4)
    dmap = rs.decode_map([False, False] + [True] * 14)
    total = 16 << 30  # bytes of stripes resident per variant (6 variants: ~100 GB of HBM)
    cases = []
    keep = []
    for L, pad, inplace in [(4 << 20, 0, True), (4 << 20, 0, False), (4 << 20, 4096, True), (1 << 20, 0, True),
                            (256 << 10, 0, True), (1 << 20, 4096, True)]:
        pitch = L + pad
        S = total // (16 * pitch)
        buf = torch.empty((S * 16 * pitch,), dtype=torch.uint8, device="cuda")
        ecx.fill_random(buf, buf.numel(), 2)
        out = buf if inplace else torch.empty((S * 2 * L,), dtype=torch.uint8, device="cuda")
        keep.append((buf, out))
        ost, osl = (16 * pitch, pitch) if inplace else (2 * L, L)
        name = f"L={L >> 10}KiB pitch=L+{pad} {'in-place' if inplace else 'separate out'}"
        cases.append((name, S * 14 * L, lambda buf=buf, out=out, S=S, pitch=pitch, L=L, ost=ost, osl=osl:
                      dmap.apply_batch(buf, 16 * pitch, pitch, out, ost, osl, S, L)))
    shapes = [(d, cm) for d in (0, 4, 8) for cm in (0, 1)]
    res = {(c[0], s): [] for c in cases for s in shapes}
    for _ in range(3):
        for name, nbytes, fn in cases:
            for d, cm in shapes:
                ecx.tune("depth", d)
                ecx.tune("chunk_major", cm)
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[(name, (d, cm))].append(nbytes / (e0.elapsed_time(e1) / 5 * 1e-3) / 1e9)
    ecx.tune("depth", 0)
    ecx.tune("chunk_major", 0)
    for (name, (d, cm)), v in res.items():
        med = statistics.median(v)
        print(json.dumps({"case": "RS(12,4) decode {0,1}, " + name, "depth": d or "auto", "chunk_major": cm,
                          "GBps_median": round(med, 1), "frac": round(med / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
