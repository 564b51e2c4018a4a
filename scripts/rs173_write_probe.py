"""Where RS(17,3) encodeParity loses against the read-only check (round-4 verdict item 6).

On the published shape (200,000-B shards back to back, 4,096 resident stripes) it times, by HIP
events, median of --reps launches each:
  encode_in_place      the bench's rs173 launch (parity written into slots 17-19 of each stripe)
  encode_out_dense     the same map, parity written to a separate dense [S][3][200,000] buffer
  encode_out_aligned   ... to a separate buffer whose parity rows are 128-B aligned (pitch 200,064)
  encode_reads_only    the same kernel with every stripe's parity written to ONE 600 KB scratch
                       area (out stride 0: the writes stay in L2, HBM sees the 17 reads only)
  check_read_only      isParityCorrect (k_gf_check): the 20 slots read, nothing written
  encode_nt0 / nt2     in place with plain / always-non-temporal loads and stores
Each line: median ms, the fraction of 8 TB/s on the bytes that case moves to or from HBM, and
the same on the encode's own 20 x 200,000 B per stripe.  One JSON line per case."""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pool", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    import rpamd
    ecx = rpamd.load(shape_knobs=True)
    L, P = 200000, a.pool
    pool = torch.empty((P, 20, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 11)
    rs = ecx.ReedSolomon.create(17, 3)
    rs.encodeParityBatch(pool, 20 * L, L, P, 0, L)
    emap = rs.encode_map()
    # the encode's parity rows as a map over the 17 data slots only, outputs at rows 0..2
    mat, ins, outs = emap.matrix()
    pmap = ecx.GfMap.from_matrix(mat, in_slot=list(ins), out_slot=[0, 1, 2])
    dense = torch.empty((P, 3, L), dtype=torch.uint8, device="cuda")
    pitch = 200064
    aligned = torch.empty((P, 3, pitch), dtype=torch.uint8, device="cuda")
    scratch = torch.empty((3, L), dtype=torch.uint8, device="cuda")
    verdict = torch.empty(P, dtype=torch.uint8, device="cuda")
    enc_bytes = P * 20 * L

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
        for e0, e1 in ev:
            e0.record()
            fn()
            e1.record()
        torch.cuda.synchronize()
        ms = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
        return ms[len(ms) // 2], ecx.last_launch_shape()

    cases = [
        ("encode_in_place", lambda: rs.encodeParityBatch(pool, 20 * L, L, P, 0, L), enc_bytes, None),
        ("encode_out_dense", lambda: pmap.apply_batch(pool, 20 * L, L, dense, 3 * L, L, P, L), enc_bytes, None),
        ("encode_out_aligned", lambda: pmap.apply_batch(pool, 20 * L, L, aligned, 3 * pitch, pitch, P, L), enc_bytes,
         None),
        ("encode_reads_only", lambda: pmap.apply_batch(pool, 20 * L, L, scratch, 0, L, P, L), P * 17 * L, None),
        ("check_read_only", lambda: rs.isParityCorrectBatch(pool, 20 * L, L, P, 0, L, verdict), enc_bytes, None),
        ("encode_nt0", lambda: rs.encodeParityBatch(pool, 20 * L, L, P, 0, L), enc_bytes, ("nontemporal", 0)),
        ("encode_nt2", lambda: rs.encodeParityBatch(pool, 20 * L, L, P, 0, L), enc_bytes, ("nontemporal", 2)),
        ("encode_in_place_again", lambda: rs.encodeParityBatch(pool, 20 * L, L, P, 0, L), enc_bytes, None),
    ]
    enc = lambda: rs.encodeParityBatch(pool, 20 * L, L, P, 0, L)  # noqa: E731
    for knobs in ([("depth", 4)], [("depth", 8)], [("small_tiles", 1), ("depth", 4)], [("small_tiles", 1), ("depth", 8)],
                  [("small_tiles", 1), ("depth", 12)], [("small_tiles", 1), ("depth", 4), ("stagger", 4)],
                  [("depth", 4), ("xcd_misaligned", 0)], [("small_tiles", 1), ("depth", 4), ("xcd_misaligned", 0)]):
        cases.append(("encode_" + "_".join("%s%d" % kv for kv in knobs), enc, enc_bytes,
                      [("layout_select", 0)] + knobs))
    defaults = {"nontemporal": 1, "layout_select": 1, "depth": 0, "small_tiles": 2, "stagger": 0, "xcd_misaligned": 1}
    for name, fn, hbm, knob in cases:
        knobs = [knob] if isinstance(knob, tuple) else (knob or [])
        for k, v in knobs:
            ecx.tune(k, v)
        try:
            ms, shape = timed(fn)
        finally:
            for k, _ in knobs:
                ecx.tune(k, defaults[k])
        print(json.dumps({"case": name, "median_ms": round(ms, 4), "hbm_bytes": hbm,
                          "frac_of_moved": round(hbm / (ms * 1e-3) / 8e12, 4),
                          "frac_on_encode_bytes": round(enc_bytes / (ms * 1e-3) / 8e12, 4), "shape": shape}),
              flush=True)
    rs.isParityCorrectBatch(pool, 20 * L, L, P, 0, L, verdict)
    torch.cuda.synchronize()
    assert bool((verdict == 1).all()), "the pool's parity changed"
    ref = dense[:, :, :].clone()
    assert torch.equal(ref, pool[:, 17:20, :]) and torch.equal(aligned[:, :, :L], pool[:, 17:20, :])


if __name__ == "__main__":
    main()
