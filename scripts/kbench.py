"""In-process A/B of k_gf_apply launch shapes (load-ring depth, non-temporal policy) on the headline
workload (Clay(4,2) repair, B = 32 KiB, resident pool), interleaved rounds
(cdna_hip_programming.md 5.4 rule 24), plus two ceilings for this access
pattern: an XOR-only map with the identical 20-read / 8-write layout, and a
plain device-to-device copy.  Prints one JSON object per variant."""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import rpamd  # noqa: E402

K, M, B, ALPHA = 4, 2, 32768, 8
ALGO = 20 * B + 8 * B


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pool", type=int, default=1 << 14)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="0:1,4:1,8:1")
    args = ap.parse_args()
    import torch
    ecx = rpamd.load(shape_knobs=True)
    lib = ecx.lib()
    import ctypes
    lib.ecx_tune.argtypes = [ctypes.c_char_p, ctypes.c_int]
    lib.ecx_tune.restype = ctypes.c_int
    lib.ecx_probe_bandwidth.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                        ctypes.c_void_p]
    lib.ecx_probe_bandwidth.restype = ctypes.c_int
    P = args.pool
    pool = torch.empty((P, 48, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 1)
    out = torch.empty((P, ALPHA, B), dtype=torch.uint8, device="cuda")
    step = ecx.ClayCodeErasureDecodingStep([1], K, M)
    mat, ins, outs = step.map().matrix()
    xor_map = ecx.GfMap.from_matrix((mat != 0).astype("uint8"), in_slot=ins, out_slot=outs)
    copy_src = pool.view(-1)[: P * ALPHA * B]

    def clay():
        step.performCodingBatch(pool, 48 * B, B, out, ALPHA * B, B, P, B)

    def xor_only():
        xor_map.apply_batch(pool, 48 * B, B, out, ALPHA * B, B, P, B)

    def copy():
        out.view(-1).copy_(copy_src)

    PROBE = (P * 48 * B) // 2 // 16384 * 16384
    src, dst = pool.view(-1)[:PROBE], pool.view(-1)[PROBE:2 * PROBE]
    cs = torch.cuda.current_stream().cuda_stream

    def probe(kind, nt):
        return lambda: lib.ecx_probe_bandwidth(kind, src.data_ptr(), dst.data_ptr(), PROBE, nt, cs)

    variants = []
    for v in args.variants.split(","):
        extra = {}
        if "@" in v:  # depth:nt[:threads[:scope]]@key=value;key=value (any ecx_tune key)
            v, kv = v.split("@", 1)
            extra = {k: int(x) for k, x in (p.split("=") for p in kv.split(";"))}
        f = list(map(int, v.split(":")))
        depth, nt = f[0], f[1]
        threads = f[2] if len(f) > 2 else 256
        scope = f[3] if len(f) > 3 else 0
        tag = "".join(f" {k}={x}" for k, x in extra.items())
        variants.append((f"clay depth={depth} nt={nt} threads={threads} store_scope={scope}{tag}", clay, depth, nt,
                         P * ALGO, threads, scope, extra))
    variants.append(("xor-only depth=0 nt=1", xor_only, 0, 1, P * ALGO, 256, 0, {}))
    variants.append(("probe read nt=0", probe(0, 0), 4, 0, PROBE, 256, 0, {}))
    variants.append(("probe read nt=1", probe(0, 1), 4, 0, PROBE, 256, 0, {}))
    variants.append(("probe copy nt=0", probe(1, 0), 4, 0, 2 * PROBE, 256, 0, {}))
    variants.append(("probe copy nt=1", probe(1, 1), 4, 0, 2 * PROBE, 256, 0, {}))
    variants.append(("d2d copy (torch)", copy, 4, 0, 2 * P * ALPHA * B, 256, 0, {}))

    res = {name: [] for name, *_ in variants}
    for r in range(args.rounds):
        for name, fn, depth, nt, nbytes, threads, scope, extra in variants:
            lib.ecx_tune(b"block_threads", threads)
            lib.ecx_tune(b"store_scope", scope)
            for k, x in extra.items():
                lib.ecx_tune(k.encode(), x)
            lib.ecx_tune(b"depth", depth)
            lib.ecx_tune(b"nontemporal", nt)
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.launches):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.launches
            res[name].append(nbytes / (ms * 1e-3) / 1e9)
            for k in extra:  # back to the library default
                lib.ecx_tune(k.encode(), {"xcd_group": 0, "chunk_major": 0}.get(k, 0))
    lib.ecx_tune(b"depth", 0)
    lib.ecx_tune(b"nontemporal", 1)
    lib.ecx_tune(b"block_threads", 0)
    lib.ecx_tune(b"store_scope", 0)
    for name, *_ in variants:
        v = res[name]
        print(json.dumps({"variant": name, "GBps_median": round(statistics.median(v), 1),
                          "GBps_max": round(max(v), 1), "frac_of_8TBps": round(statistics.median(v) / 8000, 4)}))



if __name__ == "__main__":
    main()
