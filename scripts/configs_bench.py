"""Secondary measurements: every BASELINE.json config on one MI355X, device
resident, as achieved algorithmic GB/s of the dominant kernel against the
8 TB/s HBM peak (BASELINE.md section 3 bytes per unit).  One JSON line per
config; recorded in DESIGN.md (the bench.py headline is config 2)."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rpamd  # noqa: E402

PEAK = 8000.0


def timed(fn, reps=10):
    import torch
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


SWEEP = [(0, 1), (4, 1), (8, 1), (0, 0)]  # (load-ring depth, nontemporal); first = default (0 = per map)


def sweep(lib, name, unit_bytes, units, fn, reps=10, extra=None):
    """Time fn under each launch shape of SWEEP (results are bit-identical)."""
    for depth, nt in SWEEP:
        lib.ecx_tune(b"depth", depth)
        lib.ecx_tune(b"nontemporal", nt)
        t = timed(fn, reps)
        report(name, unit_bytes, units, t, dict(extra or {}, depth=depth, nontemporal=nt))
    lib.ecx_tune(b"depth", 0)
    lib.ecx_tune(b"nontemporal", 1)


def report(name, unit_bytes, units, sec, extra=None):
    gbs = unit_bytes * units / sec / 1e9
    d = {"config": name, "units": units, "bytes_per_unit": unit_bytes, "ms_per_launch": round(sec * 1e3, 3),
         "GBps": round(gbs, 1), "GiBps": round(unit_bytes * units / sec / 2**30, 1), "frac_of_peak": round(gbs / PEAK, 4)}
    if extra:
        d.update(extra)
    print(json.dumps(d), flush=True)


def main():
    import ctypes
    import torch
    ecx = rpamd.load()
    lib = ecx.lib()
    lib.ecx_tune.argtypes = [ctypes.c_char_p, ctypes.c_int]
    # ---- config 2 encode (stripe generation): Clay(4,2), 32 KiB
    B, P = 32768, 1 << 13
    pool = torch.empty((P, 48, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 1)
    par = torch.empty((P, 16, B), dtype=torch.uint8, device="cuda")
    enc = ecx.ClayCodeErasureDecodingStep([4, 5], 4, 2)
    sweep(lib, "Clay(4,2) encode, 32 KiB (16x32 map)", 32 * B + 16 * B, P,
          lambda: enc.performCodingBatch(pool, 48 * B, B, par, 16 * B, B, P, B))
    del pool, par
    # ---- config 3: LRC 12+4 XOR groups, 64 KiB blocks: encode and repair of block 2
    B, S = 65536, 1 << 14
    pool = torch.empty((S, 16, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 2)
    import numpy as np
    encm = np.zeros((4, 16), np.uint8)
    for g in range(4):
        encm[g, 4 * g:4 * g + 3] = 1
    emap = ecx.GfMap.from_matrix(encm, in_slot=list(range(16)), out_slot=[3, 7, 11, 15])
    sweep(lib, "LRC encode, 64 KiB blocks", 16 * B, S, lambda: emap.apply_batch(pool, 16 * B, B, pool, 16 * B, B, S, B))
    rmap = ecx.GfMap.from_matrix(np.array([[1, 1, 1]], np.uint8), in_slot=[0, 1, 3], out_slot=[0])
    out = torch.empty((S, 1, B), dtype=torch.uint8, device="cuda")
    sweep(lib, "LRC repair of block 2, 64 KiB", 4 * B, S, lambda: rmap.apply_batch(pool, 16 * B, B, out, B, B, S, B))
    del pool, out
    # ---- config 4: shortened Clay(10,4), 1 MiB node block = 256 x 4 KiB, single repair
    k, m, v, B, S = 10, 4, 2, 4096, 2048
    n, a = 14, 256
    pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 3)
    out = torch.empty((S, a, B), dtype=torch.uint8, device="cuda")
    step = ecx.ClayCodeErasureDecodingStep([3], k, m, virtualUnits=v)
    inf = step.map().info()
    sweep(lib, "Clay(10,4) shortened, 1 MiB blocks, single repair (e=3)", (inf["n_in"] + inf["n_out"]) * B, S,
          lambda: step.performCodingBatch(pool, n * a * B, B, out, a * B, B, S, B), reps=5, extra={"map": inf})
    del pool, out
    # ---- config 5: RS(12,4), 4 MiB shards, erasures {0,1}, in place
    L, S = 4 << 20, 256
    rs = ecx.ReedSolomon.create(12, 4)
    pool = torch.empty((S, 16, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 4)
    dmap = rs.decode_map([False, False] + [True] * 14)
    sweep(lib, "RS(12,4) 2-erasure decode, 4 MiB", 14 * L, S,
          lambda: dmap.apply_batch(pool, 16 * L, L, pool, 16 * L, L, S, L), reps=5)


if __name__ == "__main__":
    main()
