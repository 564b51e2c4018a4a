"""The reference's two RS measurements, side by side on this host and its MI355X.

1. BASELINE config 1: RS(4,2) encode + single-erasure decode of LP-block.jpg through the
   SampleEncoder / SampleDecoder file format (SampleEncoder.java:54-83,
   SampleDecoder.java:34-98): the oracle (the reference's JVM path restated in C,
   oracle/) against the product's per-call entry points (repair-pipelining_amd:
   sample_encode / sample_decode over ecx_rs_encode_parity / ecx_rs_decode_missing).
   Both files round-trip bit-exactly, and every shard equals the oracle's.

2. The reference's only published number: RS(17,3) encodeParity on 200,000-byte shards
   with InputOutputByteTableCodingLoop, 525.7 MB/s on a Backblaze storage pod
   (rs/README.md:53).  Same methodology (ReedSolomonBenchmark.java:25-33,104-124): MB/s =
   17 x 200,000 data bytes per call / 10^6 / seconds, buffer sets cycled so the data
   spans at least twice the L3 (here twice THIS host's L3, not the pod's 10 MiB),
   two warm-up measurements, then the average of ten 2-second measurements, one thread.
   Rows: the oracle on 1 thread and on the lease's threads; ecx_rs_encode_parity per call
   (host byte[]s in, parity back to host, as EcxCodingLoop would run inside ReedSolomon);
   and the device-resident batch (ecx_rs_encode_parity_batch over stripes in HBM).

One JSON line per row (stdout).  Needs a GPU for the product rows.
"""
import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle")]
import bench  # noqa: E402
import oracle as O  # noqa: E402
import rpamd  # noqa: E402

PUBLISHED_MBPS = 525.7  # rs/README.md:53, InputOutputByteTableCodingLoop encodeParity
K17, M17, SHARD = 17, 3, 200 * 1000


def emit(d):
    print(json.dumps(d), flush=True)


def measure(fn, seconds, data_bytes):
    """ReedSolomonBenchmark.doOneEncodeMeasurement: call until `seconds` have elapsed."""
    n, t0 = 0, time.perf_counter()
    while True:
        fn(n)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return n * data_bytes / 1e6 / el


def config1(ecx, reps):
    f = np.frombuffer((ROOT / "tests" / "golden" / "LP-block.jpg").read_bytes(), np.uint8)
    ref = O.sample_encode(f)
    got = ecx.sample_encode(f)
    assert all((a == b).all() for a, b in zip(ref, got)), "encoded shards differ from the oracle"
    lost = [s if i != 1 else None for i, s in enumerate(ref)]  # one data shard erased
    dec_ref, _ = O.sample_decode(lost)
    dec_got, _ = ecx.sample_decode(lost)
    assert (dec_ref == f).all() and (np.asarray(dec_got) == f).all(), "decoded file differs"
    for name, enc, dec in (("oracle (reference JVM path restated, 1 thread)", O.sample_encode, O.sample_decode),
                           ("product per-call (MI355X, host buffers)", ecx.sample_encode, ecx.sample_decode)):
        for op, fn in (("encode", lambda: enc(f)), ("decode 1 data shard", lambda: dec(lost))):
            fn()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            t = float(np.median(ts))
            emit({"config": "1: RS(4,2) SampleEncoder/SampleDecoder, LP-block.jpg (%d B)" % f.size, "op": op,
                  "path": name, "us_per_file": round(t * 1e6, 1), "MBps_file_bytes": round(f.size / t / 1e6, 1),
                  "bit_exact_vs_oracle": True})


def rs173(ecx, seconds, measurements):
    import torch
    info = bench.host_cpu_info()
    l3 = info["l3_bytes_machine"] or (32 << 20)
    data_bytes = K17 * SHARD
    sets = 2 * l3 // data_bytes + 1  # NUMBER_OF_BUFFER_SETS, for this host's L3
    rng = np.random.default_rng(0)
    arena = np.empty((sets, K17 + M17, SHARD), np.uint8)
    base = rng.integers(0, 256, (8, K17 + M17, SHARD), dtype=np.uint8)
    for s in range(sets):
        arena[s] = base[s % 8]
    common = {"config": "RS(17,3) encodeParity, 200,000-B shards (ReedSolomonBenchmark)",
              "unit": "MB/s (data bytes, 10^6)", "published_MBps": PUBLISHED_MBPS,
              "buffer_sets": int(sets), "data_span_bytes": int(sets * data_bytes)}

    # oracle: orc_bench_run(encodeParity) on 1 thread and on the lease's threads
    addrs = (np.arange(sets, dtype=np.int64)[:, None] * arena[0].nbytes + arena.ctypes.data +
             np.arange(K17 + M17, dtype=np.int64)[None, :] * SHARD)
    threads = max(1, min(info["cgroup_quota_cpus"] or info["omp_num_threads"] or info["affinity_cpus"],
                         info["affinity_cpus"], 256))
    for th in (1, threads):
        rates = []
        for i in range(measurements + 2):
            n, el = O.bench_run(O.BENCH_RS_ENCODE, K17, M17, [], SHARD, addrs[:sets // th * th], th, seconds)
            if i >= 2:
                rates.append(n * data_bytes / 1e6 / el)
        emit(dict(common, path="oracle (InputOutputByteTableCodingLoop restated), %d thread%s" % (
            th, "" if th == 1 else "s"), MBps=round(float(np.mean(rates)), 1), threads=th,
            vs_published=round(float(np.mean(rates)) / PUBLISHED_MBPS, 2), cpu=info["model"]))

    # product per call: ecx_rs_encode_parity on host byte[]s, one thread
    lib = ecx.lib()
    rs = ecx.ReedSolomon.create(K17, M17)
    ptrs = []
    for s in range(sets):
        p = (ctypes.c_void_p * (K17 + M17))()
        p[:] = [arena[s, i].ctypes.data for i in range(K17 + M17)]
        ptrs.append(p)

    def call(n):
        st = lib.ecx_rs_encode_parity(rs._h, ptrs[n % sets], K17 + M17, SHARD, 0, SHARD)
        assert st == 0, st
    rates = [measure(call, seconds, data_bytes) for _ in range(measurements + 2)][2:]
    ref = [arena[3, i].copy() for i in range(K17)] + [np.zeros(SHARD, np.uint8) for _ in range(M17)]
    O.ReedSolomon(K17, M17).encode_parity(ref, 0, SHARD)
    exact = all((arena[3, K17 + p] == ref[K17 + p]).all() for p in range(M17))
    emit(dict(common, path="product per call: ecx_rs_encode_parity, host buffers (EcxCodingLoop shape), 1 thread",
              MBps=round(float(np.mean(rates)), 1), vs_published=round(float(np.mean(rates)) / PUBLISHED_MBPS, 1),
              bit_exact_vs_oracle=bool(exact)))

    # product device batch: stripes resident in HBM
    S = 4096
    pitch = (K17 + M17) * SHARD
    pool = torch.empty(S * pitch, dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 17)
    rs.encodeParityBatch(pool, pitch, SHARD, S, 0, SHARD)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(10):
        e0.record()
        rs.encodeParityBatch(pool, pitch, SHARD, S, 0, SHARD)
        e1.record()
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) * 1e-3)
    t = float(np.median(best))
    kern = ecx.last_kernel()
    host = pool[:pitch].cpu().numpy().reshape(K17 + M17, SHARD)
    ref = [host[i].copy() for i in range(K17)] + [np.zeros(SHARD, np.uint8) for _ in range(M17)]
    O.ReedSolomon(K17, M17).encode_parity(ref, 0, SHARD)
    exact = all((host[K17 + p] == ref[K17 + p]).all() for p in range(M17))
    mbps = S * data_bytes / 1e6 / t
    emit(dict(common, path="product device batch: ecx_rs_encode_parity_batch, %d stripes resident in HBM" % S,
              MBps=round(mbps, 1), vs_published=round(mbps / PUBLISHED_MBPS, 1), kernel=kern,
              hbm_frac=round(S * pitch / t / 8e12, 4), bit_exact_vs_oracle=bool(exact)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=2.0, help="per measurement (reference: 2 s)")
    ap.add_argument("--measurements", type=int, default=10, help="averaged (reference: 10)")
    ap.add_argument("--reps", type=int, default=50, help="config 1: timed calls per row (median)")
    args = ap.parse_args()
    ecx = rpamd.load()
    config1(ecx, args.reps)
    rs173(ecx, args.seconds, args.measurements)


if __name__ == "__main__":
    main()
