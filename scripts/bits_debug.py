"""Debug: which kernel runs for each map under ecx_tune bitslice / depth, and whether
its bytes match the numpy table product."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "oracle")]
import numpy as np
import torch
import rpamd
from conftest import gf_apply_numpy
ecx = rpamd.load()
rng = np.random.default_rng(1)
maps = {
    "clay104": ecx.ClayCodeErasureDecodingStep([3], 10, 4, virtualUnits=2).map().matrix(),
    "clay42": ecx.ClayCodeErasureDecodingStep([1], 4, 2).map().matrix(),
    "dense40x24": (rng.integers(0, 256, (40, 24)).astype(np.uint8), np.arange(24), np.arange(40)),
}
for name, (m, ins, outs) in maps.items():
    gm = ecx.GfMap.from_matrix(m, in_slot=[int(i) for i in ins], out_slot=[int(o) for o in outs])
    ni, no = int(max(ins)) + 1, int(max(outs)) + 1
    S, L = 2, 4096 * 2
    inp = torch.empty((S, ni, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(inp, inp.numel(), 5)
    host = inp.cpu().numpy()
    ref = [gf_apply_numpy(m, [host[s, j] for j in ins]) for s in range(S)]
    for bs, depth in ((0, 0), (2, 2), (2, 4), (1, 0)):
        ecx.tune("bitslice", bs)
        ecx.tune("depth", depth)
        out = torch.full((S, no, L), 0x5A, dtype=torch.uint8, device="cuda")
        gm.apply_batch(inp, ni * L, L, out, no * L, L, S, L)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        bad = sum(int((got[s, slot] != ref[s][o]).sum()) for s in range(S) for o, slot in enumerate(outs))
        print(name, "bitslice", bs, "depth", depth, "->", ecx.last_kernel(), "mismatched bytes", bad, flush=True)
ecx.tune("bitslice", 1)
ecx.tune("depth", 0)

# the launch-shape test's layout: Clay(10,4) shortened, B = 4096, S = 5 stripes of n*alpha sub-chunks
step = ecx.ClayCodeErasureDecodingStep([3], 10, 4, virtualUnits=2)
m, ins, outs = step.map().matrix()
n, a, B, S = 14, step.subPacketSize, 4096, 5
pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
ecx.fill_random(pool, pool.numel(), 31)
host = pool.cpu().numpy()
ref = [gf_apply_numpy(m, [host[s, j] for j in ins]) for s in range(S)]
for wg, lt, sc, cm, bt, wd, bs in ((1, 1, 0, 0, 256, 0, 1), (0, 0, 0, 0, 256, 0, 1), (0, 1, 0, 0, 256, 0, 0),
                                   (0, 1, 0, 0, 256, 0, 1), (0, 1, 1, 0, 256, 0, 1), (0, 1, 0, 1, 64, 0, 2)):
    for k, v in (("wave_groups", wg), ("lds_tables", lt), ("store_scope", sc), ("chunk_major", cm),
                 ("block_threads", bt), ("wide_tiles", wd), ("bitslice", bs)):
        ecx.tune(k, v)
    o = torch.full((S, a, B), 7, dtype=torch.uint8, device="cuda")
    step.performCodingBatch(pool, n * a * B, B, o, a * B, B, S, B)
    torch.cuda.synchronize()
    got = o.cpu().numpy()
    bad = [(s, r) for s in range(S) for r in range(a) if (got[s, outs[r]] != ref[s][r]).any()]
    print("variant", (wg, lt, sc, cm, bt, wd, bs), ecx.last_kernel(), "bad rows", len(bad), bad[:6], flush=True)
