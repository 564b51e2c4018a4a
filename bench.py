"""Headline benchmark: device-resident Clay(4,2) single-node repair, 32 KiB
sub-chunks (BASELINE.json configs[1]), on N GPUs (one process per GPU).

One "step" = batch repair of 2^20 synthetic stripes per GPU (the config's
"1M synthetic stripes"), executed as passes over a resident pool of valid
stripes in HBM (random data + GPU Clay encode).  Stripes are independent, so
the work is partitioned across ranks with no data-path collective (weak
scaling); the only collectives are the timing barrier and the max-over-ranks.

Metric: algorithmic bytes per stripe = 20 helper
sub-chunks read + 8 repaired sub-chunks written = 917,504 B; GiB/s = bytes
* stripes / time / 2^30, whole job.  ``roofline`` prices the dominant kernel
(k_gf_apply<false,true,1,8,false>) against the MI355X HBM peak from per-launch HIP events;
``cpu_baseline`` times the oracle (the C restatement of the reference's JVM
path, stage by stage) on this host for a bounded sample: one thread, then one
thread per host core (oracle/orc_bench.c).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for _p in (ROOT, ROOT / "oracle"):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

K, M, B = 4, 2, 32768
N_NODES = K + M
ALPHA = 8
STRIPE_BYTES = N_NODES * ALPHA * B          # 1.5 MiB per stripe in the pool
READ_BYTES = 20 * B                          # helper sub-chunks read by one repair
WRITE_BYTES = ALPHA * B                      # repaired sub-chunks written
ALGO_BYTES = READ_BYTES + WRITE_BYTES        # 917,504 B per stripe
HBM_PEAK_GBS = 8000.0                        # MI355X HBM3E spec (MI355X_MICROARCH.md)
KERNEL = "k_gf_apply<false,true,1,8,false>"  # dominant kernel (SAFE=false, NT loads, NT stores, depth 8, SGPR tables)
METRIC = "GiB/s repair-decode (device-resident), Clay(4,2) 32 KiB blocks, 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--stripes-per-step", type=int, default=1 << 20)
    ap.add_argument("--pool", type=int, default=1 << 15, help="resident stripes per GPU (48 GiB at 2^15)")
    ap.add_argument("--erased", type=int, default=1, help="erased node (README: '1 LP 1 pipeline')")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample; 0 = skip")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-probes", action="store_true", help="skip the in-run memory ceiling probes")
    return ap.parse_args()


def _cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def cpu_baseline(seconds: float, erased: int, sample=None):
    """Oracle (C restatement of the reference JVM path: InputOutputByteTableCodingLoop
    + the ClayCodeErasureDecodingStep.doDecodeSingle stage sequence), timed by
    oracle/orc_bench.c on one host thread and then on one thread per host core
    (independent stripes per thread).  ``value`` is the
    all-cores figure; the 1-thread figure rides along.  `sample` = (stripe, GPU repair
    output) of one pool stripe: the oracle repairs it too, and ``oracle_check`` says
    whether the bytes agree (the sampled byte-compare of SURVEY.md 8(d))."""
    import numpy as np
    import oracle as O

    oracle_check = None
    if sample is not None:
        stripe, got = sample
        inputs = [None if (i % N_NODES) == erased else stripe[i].copy() for i in range(N_NODES * ALPHA)]
        ref = [np.zeros(B, np.uint8) for _ in range(ALPHA)]
        O.Clay(K, M, [erased]).perform_coding(inputs, ref, B)
        oracle_check = all(bool((got[z] == ref[z]).all()) for z in range(ALPHA))

    threads = int(os.environ.get("OMP_NUM_THREADS") or len(os.sched_getaffinity(0)))
    threads = max(1, min(threads, len(os.sched_getaffinity(0)), 64))
    per_thread = 2
    rng = np.random.default_rng(0)

    def stripe():
        data = [rng.integers(0, 256, B, dtype=np.uint8) if (i % N_NODES) < K else None
                for i in range(N_NODES * ALPHA)]
        par = O.clay_encode(K, M, data, B)
        full = [data[i] if (i % N_NODES) < K else par[(i // N_NODES) * M + (i % N_NODES) - K]
                for i in range(N_NODES * ALPHA)]
        return [None if (i % N_NODES) == erased else full[i] for i in range(N_NODES * ALPHA)]

    stripes = [stripe() for _ in range(per_thread * threads)]
    n1, el1 = O.bench_clay_repair(K, M, erased, B, stripes[:per_thread], 1, seconds / 2)
    nn, eln = O.bench_clay_repair(K, M, erased, B, stripes, threads, seconds)
    one = n1 * ALGO_BYTES / el1 / 2**30
    return {
        "value": round(nn * ALGO_BYTES / eln / 2**30, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "single_thread_value": round(one, 3),
        "oracle_check": oracle_check,
        "sample": f"Clay(4,2) single repairs (e={erased}, B=32 KiB), stage-by-stage C restatement of the "
                  f"reference JVM path (oracle/): {nn} repairs on {threads} threads x {per_thread} host-resident "
                  f"valid stripes each in {eln:.1f} s; single thread {n1} repairs in {el1:.1f} s; {_cpu_model()}",
    }


def pmc_traffic(pool: int):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (if it matches)."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        if d.get("pool_stripes") == pool and d.get("kernel") == KERNEL:
            return d["hbm_bytes_per_launch"]
    except Exception:
        return None
    return None


def memory_probes(ecx, torch, pool, reps: int = 5):
    """In-run memory ceilings on this GPU: NT read stream, NT copy
    kernel, hipMemcpyDtoD (torch copy_), each the best of `reps` over 8 GiB regions of
    the (already verified and timed) pool.  The mix model prices this workload's
    20-read : 8-write bytes from the read and copy probes."""
    flat = pool.view(-1)
    n = min(8 << 30, flat.numel() // 2) // 16384 * 16384
    src, dst = flat[:n], flat[n:2 * n]

    def best(fn, nbytes):
        out = 0.0
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            out = max(out, nbytes / (e0.elapsed_time(e1) * 1e-3) / 1e9)
        return out

    rd = best(lambda: ecx.probe_bandwidth(0, src, dst, n, True), n)
    cp = best(lambda: ecx.probe_bandwidth(1, src, dst, n, True), 2 * n)
    dd = best(lambda: dst.copy_(src), 2 * n)
    w = 1.0 / (2.0 / cp - 1.0 / rd)  # write-equivalent rate implied by the copy probe
    mix = (20 + 8) / (20 / rd + 8 / w)
    return {"read_probe_GBps": round(rd, 1), "copy_probe_GBps": round(cp, 1), "dtod_copy_GBps": round(dd, 1),
            "mix_model_GBps": round(mix, 1)}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import rpamd
    ecx = rpamd.load()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # ECX_BENCH_BACKEND=gloo rehearses the multi-process path on a box with fewer
    # GPUs than ranks (ranks share devices round-robin); the default is RCCL.
    backend = os.environ.get("ECX_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    ecx.set_device(local)

    P = args.pool
    passes = max(1, args.stripes_per_step // P)
    stripes_per_step = passes * P

    # ---- resident pool of valid Clay(4,2) stripes: random data + GPU encode
    pool = torch.empty((P, N_NODES * ALPHA, B), dtype=torch.uint8, device=dev)
    out = torch.empty((P, ALPHA, B), dtype=torch.uint8, device=dev)
    par = torch.empty((P, M * ALPHA, B), dtype=torch.uint8, device=dev)
    ecx.fill_random(pool, pool.numel(), 0x5EED + rank)
    enc = ecx.ClayCodeErasureDecodingStep(list(range(K, N_NODES)), K, M)
    enc.performCodingBatch(pool, STRIPE_BYTES, B, par, M * ALPHA * B, B, P, B)
    pool.view(P, ALPHA, N_NODES, B)[:, :, K:, :] = par.view(P, ALPHA, M, B)
    del par
    step_obj = ecx.ClayCodeErasureDecodingStep([args.erased], K, M)

    def repair():
        step_obj.performCodingBatch(pool, STRIPE_BYTES, B, out, ALPHA * B, B, P, B)

    repair()
    torch.cuda.synchronize()
    verified = None
    if not args.no_verify:
        verified = bool(torch.equal(out, pool.view(P, ALPHA, N_NODES, B)[:, :, args.erased, :]))
        if not verified:
            raise SystemExit("repair output differs from the erased node's original sub-chunks")

    for _ in range(args.warmup):
        for _ in range(passes):
            repair()
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps * passes)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    i = 0
    for _ in range(args.steps):
        for _ in range(passes):
            evs[i][0].record(stream)
            repair()
            evs[i][1].record(stream)
            i += 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    launch_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    per_launch_bytes = P * ALGO_BYTES
    achieved = per_launch_bytes / (launch_ms * 1e-3) / 1e9
    total_stripes = stripes_per_step * args.steps * world
    value = total_stripes * ALGO_BYTES / el / 2**30
    traffic = pmc_traffic(P)

    sample = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:  # one repaired stripe for the oracle check
        sample = (pool[P // 2].cpu().numpy(), out[P // 2].cpu().numpy())
    probes = memory_probes(ecx, torch, pool) if not args.no_probes else None

    cpu = None
    if sample is not None:
        cpu = cpu_baseline(args.cpu_seconds, args.erased, sample)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (device splitmix64 data, GPU Clay(4,2) encode -> valid stripes)",
            "config": {
                "workload": "Clay(4,2) single-node repair (erased node %d), CLAY_BLOCK_SIZE=32768, "
                            "%d stripes per GPU per step over a resident pool of %d" % (args.erased,
                                                                                         stripes_per_step, P),
                "global_batch": stripes_per_step * world,
                "parallelism": "stripe-partitioned dp%d (no data-path collective)" % world,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": KERNEL,
                "avg_launch_ms": round(launch_ms, 4),
                "algorithmic_bytes_per_launch": per_launch_bytes,
                "measured_ceilings": probes,
                "frac_of_mix_model": round(achieved / probes["mix_model_GBps"], 4) if probes else None,
            },
            "repaired_output_GiBps": round(total_stripes * WRITE_BYTES / el / 2**30, 3),
            "cpu_baseline": cpu,
            "verified": verified,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
