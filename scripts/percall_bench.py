"""Per-call latency of the host-buffer entry points -- the shape in which the
reference's nodes call the codec, one message at a time (ClayCodeNode.kt:125-274,
SampleEncoder.java:83, LRCErasureCodeExample.kt:45): staging H2D, one kernel,
D2H, synchronize.  One JSON line per case: microseconds per call (median of
timed calls) and GiB/s of the call's algorithmic bytes."""
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT)]
import rpamd  # noqa: E402


def timeit(fn, reps=50):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def main():
    import numpy as np
    ecx = rpamd.load(shape_knobs=True)
    rng = np.random.default_rng(0)
    cases = []
    for L in (4096, 32768, 1 << 20):
        sh = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(4)] + [np.zeros(L, np.uint8) for _ in range(2)]
        rs = ecx.ReedSolomon.create(4, 2)
        cases.append((f"RS(4,2) encodeParity, {L} B shards", 6 * L, lambda sh=sh, rs=rs, L=L: rs.encodeParity(sh, 0, L)))
        present = [True, False, True, True, True, True]
        cases.append((f"RS(4,2) decodeMissing (1 data shard), {L} B shards", 5 * L,
                      lambda sh=sh, rs=rs, L=L: rs.decodeMissing(sh, present, 0, L)))
    for B in (4096, 32768):
        inputs = [None if i % 6 == 1 else rng.integers(0, 256, B, dtype=np.uint8) for i in range(48)]
        outs = [np.zeros(B, np.uint8) for _ in range(8)]
        step = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
        cases.append((f"Clay(4,2) performCoding repair e=1, B={B}", 28 * B,
                      lambda inputs=inputs, outs=outs, step=step, B=B: step.performCoding(inputs, outs, B)))
    for zc in (0, 1):
        ecx.tune("host_zero_copy", zc)
        for name, nbytes, gpu in cases:
            tg = timeit(gpu)
            print(json.dumps({"case": name, "host_zero_copy": zc, "us_per_call": round(tg * 1e6, 1),
                              "GiBps": round(nbytes / tg / 2**30, 3)}), flush=True)
    ecx.tune("host_zero_copy", 1)


if __name__ == "__main__":
    main()
