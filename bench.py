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
(the k_gf_apply instance the library reports it launched, ecx_last_kernel) against
the MI355X HBM peak from per-launch HIP events;
``cpu_baseline`` times the oracle (the C restatement of the reference's JVM
path, stage by stage) on this host for a bounded sample: one thread, then one
thread per CPU of the lease, over a working set of >= 2x the host L3 (oracle/orc_bench.c).

``--gpus N`` runs N ranks, one process per GPU: under torch.distributed.run (the
driver's launch) each process is one rank; without a launcher, bench.py starts
torch.distributed.run itself as a child process.

``--workload`` runs the other multi-GPU BASELINE configs with the same
contract (same launch, timing and JSON line; the default is the headline):
  clay104  config 4: shortened Clay(10,4), 1 MiB node blocks (256 x 4 KiB sub-chunks),
           single repair of node 3, 2,048 resident stripes per GPU
  rs124    config 5: RS(12,4), 4 MiB shards, 2-erasure decode {0,1} in place,
           512 resident stripes per GPU (shard pitch 4 MiB + 4 KiB, --pitch-pad)
  lrc      config 3: LRC (12 data, 4 XOR local parities), 64 KiB blocks, repair of
           data block 2 from its local group, 2^15 resident stripes per GPU
  clay42x2 SURVEY 8(f) f4: Clay(4,2), 32 KiB, two-node repair of nodes {0, 3}
           (doDecodeMulti) over the headline's pool of 2^15 stripes
  lrcenc   config 3's other half: LRC encode (4 XOR local parities of 3 blocks each, written in
           place, LRCErasureCodeExample.kt:30-60), 64 KiB blocks, 2^15 resident stripes per GPU
  rs173    the reference's only published benchmark (rs/README.md:53): RS(17,3)
           encodeParity in place on 200,000-B shards, 4,096 resident stripes per GPU;
           value in its own convention, MB/s of input data (10^6 B,
           ReedSolomonBenchmark.java:116-121), with vs_baseline = value / 525.7 MB/s
  rs173check the same benchmark's other half (ReedSolomonBenchmark.java:73-87,126-149): RS(17,3)
           isParityCorrect over the encoded pool, read-only, one verdict byte per stripe; MB/s of
           data bytes checked (no published figure)
Every workload's N=1 line carries a cpu_baseline (rank 0, after the timed region): the
oracle's restatement of the reference path for that workload on this host's cores.
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
METRIC = "GiB/s repair-decode (device-resident), Clay(4,2) 32 KiB blocks, 1/2/4/8 GPU"

# workload -> (metric, default resident pool per GPU, default stripes per step per GPU)
WORKLOADS = {
    "clay42": (METRIC, 1 << 15, 1 << 20),
    "clay104": ("GiB/s repair-decode (device-resident), Clay(10,4) 1 MiB blocks, 1/2/4/8 GPU", 2048, 1 << 15),
    "rs124": ("GiB/s 2-erasure decode (device-resident), RS(12,4) 4 MiB blocks, 1/2/4/8 GPU", 512, 4096),
    "lrc": ("GiB/s local-group repair (device-resident), LRC(12,4) 64 KiB blocks, 1/2/4/8 GPU", 1 << 15, 1 << 18),
    "clay42x2": ("GiB/s two-node repair-decode (device-resident), Clay(4,2) 32 KiB blocks, 1/2/4/8 GPU", 1 << 15,
                 1 << 18),
    "lrcenc": ("GiB/s local-parity encode (device-resident), LRC(12,4) 64 KiB blocks, 1/2/4/8 GPU", 1 << 15, 1 << 18),
    "rs173": ("MB/s RS(17,3) encodeParity (device-resident), 200,000-B shards, input data bytes / 10^6 "
              "(ReedSolomonBenchmark convention), 1/2/4/8 GPU", 4096, 1 << 15),
    "rs173check": ("MB/s RS(17,3) isParityCorrect (device-resident), 200,000-B shards, data bytes checked / 10^6 "
                   "(ReedSolomonBenchmark convention), 1/2/4/8 GPU", 4096, 1 << 15),
}
# ecx_tune keys the product library always accepts (include/ecx_tune.h); --tune of any other key
# opts this process in to the shape knobs (ECX_SHAPE_KNOBS=1)
DEPLOYMENT_KEYS = {"layout_select", "plan_cache", "roctx", "host_chunk_kib", "host_buffers", "host_gather_kib",
                   "host_zero_copy", "host_contexts", "host_exec_kib"}
# the one published reference number for a workload: vs_baseline = value / it
PUBLISHED = {"rs173": 525.7}  # MB/s, RS(17,3) encodeParity, InputOutputByteTableCodingLoop (rs/README.md:53)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)  # 8 x 32 headline launches: >= 1 s timed
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="clay42", choices=list(WORKLOADS))
    ap.add_argument("--stripes-per-step", type=int, default=None, help="default: per workload (2^20 for clay42)")
    ap.add_argument("--pool", type=int, default=None, help="resident stripes per GPU (clay42: 2^15 = 48 GiB)")
    ap.add_argument("--erased", type=int, default=None, help="erased node (clay42: 1, README '1 LP 1 pipeline')")
    ap.add_argument("--sub-bytes", type=int, default=None,
                    help="clay104: bytes per sub-chunk (CLAY_BLOCK_SIZE). Default 4096: 1 MiB node blocks of 256 "
                         "sub-chunks; 1048576 is config 4's other reading, 1 MiB sub-chunks (256 MiB node blocks)")
    ap.add_argument("--layout", default="natural", choices=["natural", "blocked"],
                    help="rs173 / rs124: natural = the shards back to back ([stripe][shard][pitch]); blocked = "
                         "the engine's layout contract (ecx_rs_blocked_layout: 64 KiB blocks block-major, tails "
                         "apart; DESIGN.md section 4.6)")
    ap.add_argument("--pitch", default=None,
                    help="rs173 / rs124 natural layout: the shard pitch in bytes, or 'recommended' "
                         "(ecx_rs_recommended_pitch); default: the shard size (rs124: plus --pitch-pad)")
    ap.add_argument("--pitch-pad", type=int, default=0,
                    help="rs124: bytes of padding per 4 MiB shard (default 0: the natural contiguous [S][16][4 MiB] layout)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="CPU baseline on: > 0 (the bounded protocol's all-thread sample length); 0 = skip")
    ap.add_argument("--cpu-protocol", default="reference", choices=["bounded", "reference"],
                    help="reference (default): BASELINE.md section 4 / ReedSolomonBenchmark.java:104-124, 2 warm-ups + "
                         "the mean of 10 x 2 s measurements per thread count (~50 s on rank 0 after the timed region); "
                         "bounded: one sample of cpu-seconds/2 on one thread and one of cpu-seconds on all")
    ap.add_argument("--e2e-seconds", type=float, default=2.0,
                    help="end-to-end leg (pinned host -> H2D -> kernel -> D2H) after the timed region, on every "
                         "rank at once: > 0 = its length in seconds; 0 = skip")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-probes", action="store_true", help="skip the in-run memory ceiling probes")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="launch-shape knob (include/ecx_tune.h), for A/B runs; repeatable")
    ap.add_argument("--meta", default=None, help="write the launch metadata (kernel, pool, bytes per launch, "
                                                 "kernel-source hash) as JSON here (scripts/pmc.sh)")
    args = ap.parse_args()
    _metric, pool, per_step = WORKLOADS[args.workload]
    if args.sub_bytes is not None and args.workload != "clay104":
        ap.error("--sub-bytes applies to --workload clay104 only")
    if (args.layout != "natural" or args.pitch is not None) and args.workload not in ("rs173", "rs124"):
        ap.error("--layout / --pitch apply to --workload rs173 and rs124 only")
    if args.layout == "blocked" and (args.pitch is not None or args.pitch_pad):
        ap.error("--layout blocked has no shard pitch")
    if args.workload == "clay104" and args.sub_bytes and args.sub_bytes != Clay104.b:
        # the same 2^15 x 1,088 x 4 KiB of algorithmic bytes per step, over a pool of 16 stripes
        # (56 GiB at 1 MiB sub-chunks) instead of 2,048
        scale = args.sub_bytes / Clay104.b
        pool = max(1, min(16, int(2 * pool / scale)))
        per_step = max(pool, int(per_step / scale))
    args.pool = args.pool or pool
    args.stripes_per_step = args.stripes_per_step or per_step
    if args.erased is None:
        args.erased = {"clay42": 1, "clay104": 3}.get(args.workload, 0)
    return args


def _cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def _size_bytes(text: str) -> int:
    t = text.strip().upper()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}.get(t[-1:], 1)
    return int(t.rstrip("KMG")) * mult


def host_cpu_info() -> dict:
    """What the CPU baseline may use on this host: CPUs present, the affinity mask, the
    cgroup CPU quota (the lease's share; os.cpu_count() shows the whole machine), and
    the L3 capacity of the whole machine and of the CPUs in the affinity mask (sum over
    distinct L3 instances, /sys/devices/system/cpu/*/cache/index3)."""
    aff = sorted(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(period))))
    except (OSError, ValueError):
        pass
    l3_all, l3_aff, seen = 0, 0, set()
    for cpu in range(os.cpu_count() or 1):
        d = "/sys/devices/system/cpu/cpu%d/cache/index3" % cpu
        try:
            shared = open(d + "/shared_cpu_list").read().strip()
            size = _size_bytes(open(d + "/size").read())
        except (OSError, ValueError):
            continue
        if shared in seen:
            continue
        seen.add(shared)
        l3_all += size
        members = set()
        for part in shared.split(","):
            lo, _, hi = part.partition("-")
            members.update(range(int(lo), int(hi or lo) + 1))
        if members & set(aff):
            l3_aff += size
    omp = os.environ.get("OMP_NUM_THREADS")
    return {"model": _cpu_model(), "cpus_present": os.cpu_count(), "affinity_cpus": len(aff),
            "cgroup_quota_cpus": quota, "omp_num_threads": int(omp) if omp and omp.isdigit() else None,
            "l3_bytes_machine": l3_all or None, "l3_bytes_affinity": l3_aff or None}


CPU_ARENA_BYTES = 8 << 30  # host bytes of unit copies the CPU baseline may allocate (see cpu_baseline)
# BASELINE.md section 4's measurement protocol (ReedSolomonBenchmark.java:104-124)
REF_WARMUPS, REF_MEASUREMENTS, REF_SECONDS = 2, 10, 2.0


def cpu_baseline(wl, seconds: float, sample=None, max_units=None, units=None, protocol="bounded"):
    """The oracle (C restatement of the reference JVM path, stage by stage) on this host for
    workload `wl`, timed by oracle/orc_bench.c: one host thread, then one thread per CPU
    the lease allows (the cgroup quota, else OMP_NUM_THREADS, else the affinity mask;
    independent units and codec objects per thread).  Following
    ReedSolomonBenchmark.java:25-33, the units cycled through span at least twice the
    machine's L3, so the operations stream from DRAM as the reference's benchmark does.
    GiB/s counts the workload's own algorithmic bytes per unit (wl.unit_bytes), as the
    GPU line does.  ``value`` is the all-threads figure; the 1-thread figure rides along.
    `sample` = (unit, GPU output) of one pool unit: the oracle computes it too, and
    ``oracle_check`` says whether the bytes agree (the sampled byte-compare of 8(d)).
    `units` = a few units of the GPU run's own pool as host arrays (BASELINE.md section 4:
    "the same synthetic stripes as the GPU run"), tiled through the arena; without them the
    workload's cpu_spec() makes its own.  protocol "bounded" (the bench default, so the line
    finishes in minutes): one sample of seconds/2 on one thread and one of `seconds` on all;
    "reference" (ReedSolomonBenchmark.java:104-124): on each thread
    count 2 warm-up measurements, then the mean of 10 measurements of 2 s each."""
    import numpy as np
    import oracle as O

    spec = wl.cpu_spec()
    oracle_check = None
    if sample is not None:
        oracle_check = bool(wl.oracle_check(*sample))

    info = host_cpu_info()
    threads = info["cgroup_quota_cpus"] or info["omp_num_threads"] or info["affinity_cpus"]
    threads = max(1, min(threads, info["affinity_cpus"], 256))
    # Working set: the bytes an operation touches (the workload's algorithmic bytes per CPU
    # unit), summed over every unit cycled through, >= 2x the machine's L3 (32 MiB assumed if unknown).
    unit_bytes = spec.get("unit_bytes", wl.unit_bytes)
    l3 = info["l3_bytes_machine"] or (32 << 20)
    n_units = max(2 * threads, -(-2 * l3 // unit_bytes))
    if max_units:  # tests: a bounded arena
        threads = min(threads, max_units)
        n_units = max_units
    per_thread = -(-n_units // threads)
    n_units = per_thread * threads
    # 8 distinct units (spec["make"]: valid stripes, or random bytes where the oracle's work
    # does not depend on the data), tiled through one host arena of n_units units: every
    # unit has its own memory (the cache sees the whole working set).
    distinct = list(units) if units else spec["make"](np.random.default_rng(0))
    data_kind = "GPU-pool" if units else spec["data_kind"]
    # Units far larger than the L3 (Clay(10,4) at 1 MiB sub-chunks: 3.5 GiB) are not copied
    # per unit: when n_units copies would exceed CPU_ARENA_BYTES, the units the oracle only
    # reads (read_only_units) alias the distinct ones, each still >> L3 (the DRAM-streaming
    # premise of ReedSolomonBenchmark.java:25-33 holds per unit).
    n_arena = n_units
    if n_units * distinct[0].nbytes > CPU_ARENA_BYTES and spec.get("read_only_units"):
        n_arena = max(1, min(len(distinct), CPU_ARENA_BYTES // distinct[0].nbytes))
    if n_arena < n_units:
        arena_units = [np.ascontiguousarray(d) for d in distinct[:n_arena]]
    else:
        arena = np.empty((n_units,) + distinct[0].shape, np.uint8)
        for u in range(n_units):
            arena[u] = distinct[u % len(distinct)]
        arena_units = list(arena)
    slot_bytes = distinct[0].shape[-1]
    zero = np.zeros(slot_bytes, np.uint8)  # a shared zero-filled node (shortened Clay's virtual nodes)
    rows = np.array([arena_units[u % n_arena].ctypes.data for u in range(n_units)], np.int64)[:, None]
    addrs = np.where(spec["present"][None, :] == 1, rows + spec["arena_slot"][None, :] * slot_bytes,
                     np.where(spec["present"][None, :] == 2, zero.ctypes.data, 0)).astype(np.int64)
    op, data, parity, erased = spec["op"], spec["data"], spec["parity"], spec["erased"]

    def rate(th, secs):
        n, el = O.bench_run(op, data, parity, erased, slot_bytes, addrs, th, secs)
        return n * unit_bytes / el / 2**30, n, el

    if protocol == "reference":
        runs = {}
        for th in (1, threads):
            for _ in range(REF_WARMUPS):
                rate(th, REF_SECONDS)
            runs[th] = [rate(th, REF_SECONDS) for _ in range(REF_MEASUREMENTS)]
        one = sum(r[0] for r in runs[1]) / REF_MEASUREMENTS
        allv = sum(r[0] for r in runs[threads]) / REF_MEASUREMENTS
        timing = (f"mean of {REF_MEASUREMENTS} measurements of {REF_SECONDS:g} s after {REF_WARMUPS} warm-ups on "
                  f"{threads} threads "
                  f"({min(r[0] for r in runs[threads]):.2f}-{max(r[0] for r in runs[threads]):.2f} GiB/s) and "
                  f"on one ({min(r[0] for r in runs[1]):.3f}-{max(r[0] for r in runs[1]):.3f})")
        measurements = {"threads": [round(r[0], 3) for r in runs[threads]], "one": [round(r[0], 4) for r in runs[1]]}
    else:
        one, n1, el1 = rate(1, seconds / 2)
        allv, nn, eln = rate(threads, seconds)
        timing = (f"{nn} operations on {threads} threads in {eln:.1f} s; single thread {n1} operations over all "
                  f"{n_units} units in {el1:.1f} s")
        measurements = None
    ws = n_units * unit_bytes
    alias = ("" if n_arena == n_units else
             "; the %d units alias %d distinct %.1f GiB host units (read-only, each >> L3)"
             % (n_units, n_arena, distinct[0].nbytes / 2**30))
    out = {
        "value": round(allv, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "single_thread_value": round(one, 3),
        "oracle_check": oracle_check,
        "working_set_bytes": ws,
        "protocol": protocol,
        "host": info,
        "sample": f"{spec['what']}, stage-by-stage C restatement of the reference JVM path (oracle/), "
                  f"lease quota {info['cgroup_quota_cpus']} of {info['cpus_present']} CPUs (affinity "
                  f"{info['affinity_cpus']}), {per_thread} host-resident {data_kind} units per thread, "
                  f"{ws / 2**20:.0f} MiB of algorithmic bytes touched (>= 2x the {l3 / 2**20:.0f} MiB L3){alias}: {timing}; "
                  f"{info['model']}",
    }
    if measurements:
        out["measurements_GiBps"] = measurements
    return out


# Sources that define what the device executes for a given map, per kernel family: the
# shared planner / plan compiler / launch selection, plus either the composed-map kernels
# or the generated (hiprtc) Clay repair kernels.  Their hash is stored with every PMC
# profile (profiles/pmc_traffic.json, one per workload); a profile taken on other code
# for its kernel family is stale.
COMMON_SOURCES = ["engine.hpp", "engine.cpp", "codes.cpp", "codes.hpp"]
COMPOSED_SOURCES = ["kernels.hip", "apply.hpp", "apply_launch.inc", "apply_t256.hip", "apply_t64.hip",
                    "apply_skew.hip", "apply_bits.hip", "apply_lut.hip", "bits.hpp", "apply_check.hip"]
RTC_SOURCES = ["clay_rtc.hpp", "clay_rtc.cpp"]
# k_map_planes: its generator, the shared prelude (clay_rtc.cpp) and launch_apply's choice (kernels.hip)
PLANES_SOURCES = RTC_SOURCES + ["map_rtc.hpp", "map_rtc.cpp", "kernels.hip"]


def kernel_source_hash(kernel: str = "") -> str:
    """Hash of the sources behind `kernel`: the generated Clay kernels (k_clay_repair*),
    the generated map kernel (k_map_planes) or the composed-map family (anything else)."""
    import hashlib
    if kernel.startswith("k_clay_repair"):
        names = COMMON_SOURCES + RTC_SOURCES
    elif kernel.startswith("k_map_planes"):
        names = COMMON_SOURCES + PLANES_SOURCES
    else:
        names = COMMON_SOURCES + COMPOSED_SOURCES
    h = hashlib.sha256()
    for name in names:
        h.update(name.encode() + b"\0" + (ROOT / "repair-pipelining_amd" / "csrc" / name).read_bytes())
    return h.hexdigest()[:16]


def profile_key(args) -> str:
    """The PMC profile a run's line reads (profiles/pmc_traffic.json): the workload, plus the
    layout or sub-chunk size when the run is not the workload's default one (scripts/pmc.sh
    profiles those variants under the same names, e.g. rs173_blocked, clay104_sub1048576)."""
    key = args.workload
    if getattr(args, "layout", "natural") == "blocked":
        key += "_blocked"
    if getattr(args, "pitch", None) is not None:
        key += "_pitch%s" % args.pitch
    if getattr(args, "pitch_pad", 0):
        key += "_pad%d" % args.pitch_pad
    if args.workload == "clay104" and getattr(args, "sub_bytes", None) and args.sub_bytes != Clay104.b:
        key += "_sub%d" % args.sub_bytes
    return key


def pmc_traffic(workload: str, pool: int, kernel: str, shape: str = None):
    """HBM bytes per launch from the committed rocprofv3 PMC summary
    (scripts/pmc.sh + scripts/pmc_summary.py), used only if it was taken on this
    workload, pool size and FULL launch shape (kernel instance plus the unit order its name
    does not encode, ecx_last_launch_shape) AND on the current kernel sources.  A workload's
    entry keeps one profile per shape profiled (by_shape: every candidate of the per-layout
    selection, scripts/pmc.sh --candidates).  Returns (bytes or None, why-not)."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None, "no PMC profile"
    try:
        d = json.loads(f.read_text())
        w = d.get("workloads", {}).get(workload)
        if w is None:
            return None, "no PMC profile for this workload"
        if shape is not None and shape in w.get("by_shape", {}):
            w = w["by_shape"][shape]
        elif shape is not None and w.get("launch_shape") not in (None, shape):
            return None, "no PMC profile for this launch shape (%s)" % shape
        if w.get("kernel_source_hash") != kernel_source_hash(kernel):
            return None, "stale: PMC profile taken on other kernel sources"
        if w.get("pool_stripes") != pool or w.get("kernel") != kernel:
            return None, "stale: PMC profile taken on another pool size or kernel instance"
        return w["hbm_bytes_per_launch"], None
    except Exception as e:  # noqa: BLE001 - a malformed profile is reported, not fatal
        return None, "unreadable PMC profile: %s" % e


# Pinned host input per rank for the end-to-end leg.  One rank alone gets E2E_HOST_BYTES; the
# ranks of one node share E2E_NODE_BYTES (they run the leg at once on one host), and all of them
# together take at most E2E_MEM_FRACTION of the host memory the lease has free (the smaller of
# MemAvailable and the cgroup's memory.max - memory.current), read before the leg starts.
E2E_HOST_BYTES = 3 << 30
E2E_NODE_BYTES = 6 << 30
E2E_MEM_FRACTION = 0.25
E2E_COPY_CHUNK = 256 << 20  # device <-> host copies of the leg's fill and check, per step


def host_memory_free() -> dict:
    """Host memory this process may still take: /proc/meminfo MemAvailable and the cgroup
    (v2 memory.max - memory.current, or v1 memory.limit_in_bytes - usage_in_bytes) limit."""
    out = {"mem_available": None, "cgroup_limit": None, "cgroup_used": None}
    try:
        for ln in open("/proc/meminfo"):
            if ln.startswith("MemAvailable:"):
                out["mem_available"] = int(ln.split()[1]) * 1024
    except (OSError, ValueError, IndexError):
        pass
    for lim, cur in (("/sys/fs/cgroup/memory.max", "/sys/fs/cgroup/memory.current"),
                     ("/sys/fs/cgroup/memory/memory.limit_in_bytes", "/sys/fs/cgroup/memory/memory.usage_in_bytes")):
        try:
            text = open(lim).read().strip()
            used = int(open(cur).read().strip())
        except (OSError, ValueError):
            continue
        if text != "max" and int(text) < (1 << 60):  # v1 reports "no limit" as a huge number
            out["cgroup_limit"], out["cgroup_used"] = int(text), used
        break
    frees = [v for v in (out["mem_available"],
                         out["cgroup_limit"] - out["cgroup_used"] if out["cgroup_limit"] else None) if v is not None]
    out["free"] = max(0, min(frees)) if frees else None
    return out


def e2e_host_budget(world: int, free_bytes=None) -> int:
    """Pinned host input bytes one rank may use for the end-to-end leg: E2E_HOST_BYTES alone,
    an equal share of E2E_NODE_BYTES when `world` ranks run it at once, and never more than
    its share of E2E_MEM_FRACTION of the free host memory."""
    world = max(1, int(world))
    budget = min(E2E_HOST_BYTES, E2E_NODE_BYTES // world)
    if free_bytes is not None:
        budget = min(budget, int(free_bytes * E2E_MEM_FRACTION) // world)
    return max(0, budget)


def _copy_chunked(dst, src, chunk=None):
    """dst.copy_(src) for two flat uint8 tensors (one on the device, one a host view), at most
    `chunk` bytes per step, so no full-size host intermediate exists at any time."""
    chunk = chunk or E2E_COPY_CHUNK
    for a in range(0, src.numel(), chunk):
        dst[a:a + chunk].copy_(src[a:a + chunk])


def _peak_rss_bytes() -> int:
    import resource
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024  # Linux reports KiB


def e2e_rate(ecx, torch, wl, seconds: float, world: int = 1):
    """End-to-end rate of this workload's map on this rank's GPU with the data starting and
    ending in host memory, as the reference's path does (sub-chunks arrive and leave on
    sockets, ClayCoordinator.kt:372-395, ClayCodeNode.kt:330-347): pinned host stripes ->
    pipelined H2D -> the same kernel -> D2H (ecx_*_batch_host, host_pipe.cpp), repeated for
    >= `seconds`.  The host input holds the first stripes of the GPU run's own (valid) pool,
    copied into the pinned buffer straight from HBM in E2E_COPY_CHUNK steps (no pageable copy
    of the pool); the host outputs are compared with the device run's the same way.  The
    pinned input is bounded per rank by e2e_host_budget(world, free host memory).  GiBps
    counts the workload's algorithmic bytes per stripe (as `value`); h2d/d2h_GBps the bytes
    that crossed PCIe."""
    import numpy as np
    if not wl.host_ok:
        return None
    sb, ob = wl.host_stripe_bytes(), wl.host_out_bytes()
    mem = host_memory_free()
    budget = e2e_host_budget(world, mem["free"])
    n = min(wl.P, budget // sb)
    cap = {"budget_bytes_per_rank": budget, "world": world, "host_free_bytes": mem["free"],
           "mem_available": mem["mem_available"], "cgroup_limit": mem["cgroup_limit"]}
    if n == 0:  # one stripe alone is larger than this rank's share
        if world == 1 and (mem["free"] is None or sb + ob <= mem["free"] * E2E_MEM_FRACTION):
            n = 1  # a single rank may still take one (large) stripe within its memory fraction
        else:
            return {"skipped": "one %d-B stripe exceeds this rank's host budget" % sb, "host_cap": cap}
    hin = ecx.HostBuffer(n * sb)
    hout = ecx.HostBuffer(n * ob) if ob else None
    at = 0
    for region in wl.host_source(n):  # the first n stripes as they lie in HBM, in host order
        _copy_chunked(torch.from_numpy(hin.array[at:at + region.numel()]), region)
        at += region.numel()
    ha, ho = hin.array, (hout.array if hout else None)
    wl.host_call(ha, ho, n)  # warm-up: plans, pipe buffers
    ok = wl.host_expect(ha, ho if ho is not None else np.empty(0, np.uint8), n)
    calls, t0 = 0, time.perf_counter()
    while True:
        wl.host_call(ha, ho, n)
        calls += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    h2d, d2h = wl.pcie_bytes()
    units = calls * n
    out = {"GiBps": round(units * wl.unit_bytes / el / 2**30, 3),
           "h2d_GBps": round(units * h2d / el / 1e9, 2), "d2h_GBps": round(units * d2h / el / 1e9, 2),
           "stripes_per_call": n, "calls": calls, "seconds": round(el, 3), "verified": ok,
           "host_bytes": n * (sb + ob), "host_cap": cap, "peak_rss_bytes": _peak_rss_bytes(),
           "path": "pinned host -> H2D -> kernel -> D2H, pipelined (ecx host batch, host_pipe.cpp)"}
    plan = wl.host_plan(n)
    if plan is not None:
        out["plan"] = plan  # stripes per chunk, copies per chunk (3D, folded rows), column slices
    if wl.metric_unit != "GiB/s":
        out["value"] = round(units * (wl.metric_bytes or wl.unit_bytes) / el / wl.metric_scale, 1)
        out["unit"] = wl.metric_unit
    del hin, hout
    return out


def memory_probes(ecx, torch, region, reads: int, writes: int, reps: int = 5):
    """In-run memory ceilings on this GPU: NT read stream, NT copy
    kernel, hipMemcpyDtoD (torch copy_), each the best of `reps` over 8 GiB regions of
    the (already verified and timed) pool.  The mix model prices this workload's
    reads : writes streams from the read and copy probes."""
    flat = region.view(-1)
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
    mix = (reads + writes) / (reads / rd + writes / w)
    return {"read_probe_GBps": round(rd, 1), "copy_probe_GBps": round(cp, 1), "dtod_copy_GBps": round(dd, 1),
            "mix_model_GBps": round(mix, 1)}


class Workload:
    """A resident pool of valid stripes and one batch launch over all of it."""
    unit_bytes = ALGO_BYTES           # algorithmic bytes per stripe
    write_bytes = WRITE_BYTES         # of which written
    reads, writes = 20, 8             # equal-sized streams read / written per unit (mix model)
    description = ""
    # the line's `value` unit: GiB/s of algorithmic bytes, or (rs173) the published benchmark's
    # MB/s of input data bytes (metric_bytes per unit, per metric_scale bytes)
    metric_unit, metric_scale, metric_bytes = "GiB/s", float(2**30), None
    data_desc = "synthetic (device splitmix64 data, GPU encode -> valid stripes)"

    def launch(self):
        raise NotImplementedError

    def selected_map(self):
        """(GfMap, input slot pitch) when the launch's map takes its launch shape from the
        per-layout selection (ecx_tune "layout_select": the many-stream RS maps), else None."""
        return None

    def verify(self) -> bool:
        raise NotImplementedError

    def sample(self):
        """(one pool unit, the GPU's output for it) as host arrays, for oracle_check."""
        raise NotImplementedError

    def oracle_check(self, unit, got) -> bool:
        """The oracle's result for `unit` equals the GPU's `got`."""
        raise NotImplementedError

    def host_units(self, k: int):
        """k units of the resident pool (the GPU run's own data) as host arrays in the layout
        cpu_spec() describes."""
        raise NotImplementedError

    # ---- end-to-end (PCIe-inclusive) leg: the same map over pinned host stripes (ecx host batches)
    host_ok = True        # False: the workload has no host-memory form (the device check)

    def host_stripe_bytes(self) -> int:
        """Bytes of one stripe in the host input layout (the device pool's layout)."""
        return self.pool[0].numel()

    def host_out_bytes(self) -> int:
        """Bytes of one stripe's output in the host output buffer; 0 = written in place."""
        return self.out[0].numel()

    def host_call(self, hin, hout, n):
        raise NotImplementedError

    def host_plan(self, n):
        """How host_call's batch is chunked and copied (ecx_map_host_plan), or None."""
        return None

    def host_expect(self, hin, hout, n) -> bool:
        """The host outputs of the first n stripes equal the device run's (compared in
        E2E_COPY_CHUNK steps: no full-size host copy of the device side)."""
        import numpy as np
        if self.host_out_bytes() == 0:  # written in place: the whole host stripes equal the device pool's
            got, wants = hin[:n * self.host_stripe_bytes()], self.host_source(n)
        else:
            got, wants = hout[:n * self.host_out_bytes()], [self.out[:n].reshape(-1)]
        if got.size != sum(w.numel() for w in wants):
            return False
        at = 0
        for want in wants:
            for a in range(0, want.numel(), E2E_COPY_CHUNK):
                b = min(a + E2E_COPY_CHUNK, want.numel())
                if not np.array_equal(got[at + a:at + b], want[a:b].cpu().numpy()):
                    return False
            at += want.numel()
        return True

    def host_source(self, n):
        """The first n stripes of the resident pool as flat device regions, in the order the host
        input buffer holds them (the end-to-end leg copies and checks them region by region)."""
        return [self.pool[:n].reshape(-1)]

    def pcie_bytes(self):
        """(H2D, D2H) bytes per stripe: only the map's used input / output slots cross PCIe."""
        return self.reads * self.sub_bytes(), self.writes * self.sub_bytes()

    def sub_bytes(self) -> int:
        return self.write_bytes // max(1, self.writes)

    def cpu_spec(self) -> dict:
        """How cpu_baseline runs the oracle on this workload: op / data / parity / erased
        for orc_bench_run, make(rng) -> distinct host units [slots][bytes], and per oracle
        slot the arena slot it reads (arena_slot) and whether it is present (1), absent
        (0) or a shared zero node (2)."""
        raise NotImplementedError


class Clay42(Workload):
    """Config 2 (headline): Clay(4,2), B = 32 KiB, single-node repair."""

    def __init__(self, ecx, torch, dev, P, erased, seed):
        self.P, self.erased, self.torch = P, erased, torch
        self.pool = torch.empty((P, N_NODES * ALPHA, B), dtype=torch.uint8, device=dev)
        self.out = torch.empty((P, ALPHA, B), dtype=torch.uint8, device=dev)
        par = torch.empty((P, M * ALPHA, B), dtype=torch.uint8, device=dev)
        ecx.fill_random(self.pool, self.pool.numel(), seed)
        enc = ecx.ClayCodeErasureDecodingStep(list(range(K, N_NODES)), K, M)
        enc.performCodingBatch(self.pool, STRIPE_BYTES, B, par, M * ALPHA * B, B, P, B)
        self.pool.view(P, ALPHA, N_NODES, B)[:, :, K:, :] = par.view(P, ALPHA, M, B)
        del par
        self.step = ecx.ClayCodeErasureDecodingStep([erased], K, M)
        self.region = self.pool
        self.description = "Clay(4,2) single-node repair (erased node %d), CLAY_BLOCK_SIZE=32768" % erased

    def launch(self):
        self.step.performCodingBatch(self.pool, STRIPE_BYTES, B, self.out, ALPHA * B, B, self.P, B)

    def host_call(self, hin, hout, n):
        e = len(self.erased_list)
        self.step.performCodingBatchHost(hin, STRIPE_BYTES, B, hout, e * ALPHA * B, B, n, B)

    def host_plan(self, n):
        e = len(self.erased_list)
        return self.step.map().host_plan(STRIPE_BYTES, B, e * ALPHA * B, B, n, B)

    def verify(self):
        return bool(self.torch.equal(self.out, self.pool.view(self.P, ALPHA, N_NODES, B)[:, :, self.erased, :]))

    erased_list = property(lambda self: [self.erased])

    def host_units(self, k):
        return [self.pool[i].cpu().numpy() for i in range(min(k, self.P))]

    def sample(self):
        return self.pool[self.P // 2].cpu().numpy(), self.out[self.P // 2].cpu().numpy()

    def oracle_check(self, stripe, got):
        import numpy as np
        import oracle as O
        er = self.erased_list
        inputs = [None if (i % N_NODES) in er else stripe[i].copy() for i in range(N_NODES * ALPHA)]
        ref = [np.zeros(B, np.uint8) for _ in range(ALPHA * len(er))]
        O.Clay(K, M, er).perform_coding(inputs, ref, B)
        return all(bool((got[z] == ref[z]).all()) for z in range(len(ref)))

    def cpu_spec(self):
        import numpy as np
        import oracle as O
        er = self.erased_list

        def make(rng):  # valid stripes: random data + oracle encode
            out = []
            for _ in range(8):
                data = [rng.integers(0, 256, B, dtype=np.uint8) if (i % N_NODES) < K else None
                        for i in range(N_NODES * ALPHA)]
                par = O.clay_encode(K, M, data, B)
                out.append(np.stack([data[i] if (i % N_NODES) < K else par[(i // N_NODES) * M + (i % N_NODES) - K]
                                     for i in range(N_NODES * ALPHA)]))
            return out
        slots = np.arange(N_NODES * ALPHA)
        present = np.array([0 if (i % N_NODES) in er else 1 for i in slots], np.int64)
        return {"op": O.BENCH_CLAY, "data": K, "parity": M, "erased": er, "make": make, "arena_slot": slots,
                "present": present, "data_kind": "valid-stripe",
                "what": "Clay(4,2) repairs of nodes %s (B=32 KiB)" % er}


class Clay42x2(Clay42):
    """Clay(4,2), B = 32 KiB, repair of nodes {0, 3} (doDecodeMulti,
    ClayCodeErasureDecodingStep.java:311-421) over the same resident pool of valid stripes."""
    ERASED = [0, 3]

    def __init__(self, ecx, torch, dev, P, erased, seed):
        super().__init__(ecx, torch, dev, P, erased, seed)
        self.out = torch.empty((P, ALPHA * len(self.ERASED), B), dtype=torch.uint8, device=dev)
        self.step = ecx.ClayCodeErasureDecodingStep(self.ERASED, K, M)
        info = self.step.map().info()
        self.unit_bytes = (info["n_in"] + info["n_out"]) * B  # 32 helper + 16 repaired sub-chunks
        self.write_bytes = info["n_out"] * B
        self.reads, self.writes = info["n_in"], info["n_out"]
        self.description = "Clay(4,2) two-node repair (erased nodes 0 and 3, doDecodeMulti), CLAY_BLOCK_SIZE=32768"

    def launch(self):
        e = len(self.ERASED)
        self.step.performCodingBatch(self.pool, STRIPE_BYTES, B, self.out, e * ALPHA * B, B, self.P, B)

    def verify(self):
        e = len(self.ERASED)
        want = self.pool.view(self.P, ALPHA, N_NODES, B)[:, :, self.ERASED, :]
        return bool(self.torch.equal(self.out.view(self.P, ALPHA, e, B), want))

    erased_list = property(lambda self: list(self.ERASED))


class Clay104(Workload):
    """Config 4: shortened Clay(10,4) (Clay(12,4) with 2 virtual zero data nodes),
    single-node repair.  Its "1 MiB blocks" is read two ways: 1 MiB
    node blocks = 256 planes x 4 KiB sub-chunks (the default, b = 4096), or 1 MiB
    sub-chunks, CLAY_BLOCK_SIZE in the sense of PipelineUtil.kt:13-28 (b = 1 MiB, a
    256 MiB node block, --sub-bytes 1048576)."""
    k, m, v, b, alpha = 10, 4, 2, 4096, 256

    def __init__(self, ecx, torch, dev, P, erased, seed, sub_bytes=None):
        if sub_bytes:
            self.b = sub_bytes
        k, m, v, b, a = self.k, self.m, self.v, self.b, self.alpha
        n = k + m
        self.P, self.erased, self.torch, self.n = P, erased, torch, n
        self.pool = torch.empty((P, n * a, b), dtype=torch.uint8, device=dev)
        self.out = torch.empty((P, a, b), dtype=torch.uint8, device=dev)
        ecx.fill_random(self.pool, self.pool.numel(), seed)
        enc = ecx.ClayCodeErasureDecodingStep(list(range(k, n)), k, m, virtualUnits=v)
        par = torch.empty((P, m * a, b), dtype=torch.uint8, device=dev)
        enc.performCodingBatch(self.pool, n * a * b, b, par, m * a * b, b, P, b)
        self.pool.view(P, a, n, b)[:, :, k:, :] = par.view(P, a, m, b)
        del par
        self.step = ecx.ClayCodeErasureDecodingStep([erased], k, m, virtualUnits=v)
        info = self.step.map().info()
        self.unit_bytes = (info["n_in"] + info["n_out"]) * b  # 832 helper + 256 repaired sub-chunks
        self.write_bytes = info["n_out"] * b
        self.reads, self.writes = info["n_in"], info["n_out"]
        self.region = self.pool
        blocks = ("1 MiB node blocks = 256 x 4096-B sub-chunks" if b == 4096 else
                  "CLAY_BLOCK_SIZE=%d: %d-B sub-chunks, %d MiB node blocks" % (b, b, a * b >> 20))
        self.description = ("Clay(10,4) (shortened Clay(12,4), 2 virtual nodes) single-node repair (erased node %d), "
                            "%s" % (erased, blocks))

    def launch(self):
        n, a, b = self.n, self.alpha, self.b
        self.step.performCodingBatch(self.pool, n * a * b, b, self.out, a * b, b, self.P, b)

    def host_call(self, hin, hout, n_):
        n, a, b = self.n, self.alpha, self.b
        self.step.performCodingBatchHost(hin, n * a * b, b, hout, a * b, b, n_, b)

    def host_plan(self, n_):
        n, a, b = self.n, self.alpha, self.b
        return self.step.map().host_plan(n * a * b, b, a * b, b, n_, b)

    def verify(self):
        orig = self.pool.view(self.P, self.alpha, self.n, self.b)[:, :, self.erased, :]
        return bool(self.torch.equal(self.out, orig))

    def host_units(self, k):
        return [self.pool[i].cpu().numpy() for i in range(min(k, self.P))]

    def sample(self):
        return self.pool[self.P // 2].cpu().numpy(), self.out[self.P // 2].cpu().numpy()

    def oracle_check(self, stripe, got):
        import oracle as O
        n, a = self.n, self.alpha
        inputs = [None if (i % n) == self.erased else stripe[i].copy() for i in range(n * a)]
        ref = O.shortened_clay_perform_coding(self.k, self.m, self.v, [self.erased], inputs, self.b)
        return all(bool((got[z] == ref[z]).all()) for z in range(a))

    def cpu_spec(self):
        """The reference cannot build Clay(10,4) (integer t = (k+m)/m): its
        path for this config is Clay(12,4) with the 2 virtual data nodes zero-filled."""
        import numpy as np
        import oracle as O
        k, m, v, a = self.k, self.m, self.v, self.alpha
        n_r, n_u = k + m, k + v + m
        e_u = self.erased if self.erased < k else self.erased + v
        arena_slot, present = [], []
        for z in range(a):
            for u in range(n_u):
                virtual = k <= u < k + v
                r = u if u < k else u - v
                arena_slot.append(0 if virtual else z * n_r + r)
                present.append(2 if virtual else (0 if u == e_u else 1))

        def make(rng):  # random bytes: the oracle's work does not depend on the data
            return [rng.integers(0, 256, (n_r * a, self.b), dtype=np.uint8)
                    for _ in range(1 if n_r * a * self.b > CPU_ARENA_BYTES // 2 else 2)]
        return {"op": O.BENCH_CLAY, "data": k + v, "parity": m, "erased": [e_u], "make": make,
                "arena_slot": np.array(arena_slot, np.int64), "present": np.array(present, np.int64),
                "data_kind": "random-byte",
                "what": "Clay(10,4) repairs of node %d as the reference runs them: Clay(12,4) with the 2 virtual "
                        "data nodes zero-filled, 256 x %d-B sub-chunks; GiB/s over the shortened map's "
                        "algorithmic bytes" % (self.erased, self.b), "read_only_units": True}


def _resolve_pitch(rs, args_pitch, L, pad=0):
    """The natural layout's shard pitch: --pitch (bytes or 'recommended') or L + pad."""
    if args_pitch is None:
        return L + pad
    if str(args_pitch) == "recommended":
        return rs.recommendedPitch(L)
    p = int(args_pitch)
    if p < L:
        raise SystemExit("--pitch %d is below the shard size %d" % (p, L))
    return p


class _RsLayout:
    """A pool of RS stripes in the natural layout ([stripe][n][pitch], self.pool 3-D) or the
    blocked one (ecx_rs_blocked_layout, self.pool flat), with natural read-back."""
    layout, block = "natural", None

    def stripes(self, first, count, slots=None):
        """[count][slots][L] natural shards of stripes first.. (a device tensor)."""
        if self.layout == "blocked":
            return self.ecx.blocked_unpack(self.pool, self.P, self.n, self.L, self.block, slots, first, count)
        sl = slice(None) if slots is None else list(slots)
        return self.pool[first:first + count, sl, :self.L]

    def _layout_desc(self):
        if self.layout == "blocked":
            full, tail = divmod(self.L, self.block)
            return ("blocked layout: %d-B blocks block-major (%d full + a %d-B tail per shard, tails apart; "
                    "ecx_rs_blocked_layout)" % (self.block, full, tail))
        return "shard pitch %d B%s" % (self.pitch, "" if self.pitch != self.L else " (back to back)")

    def host_units(self, k):
        return [self.stripes(i, 1)[0].cpu().numpy() for i in range(min(k, self.P))]

    def host_stripe_bytes(self):
        return self.n * self.L if self.layout == "blocked" else self.pool[0].numel()

    def host_source(self, n):
        """Blocked: the full blocks of the first n stripes, then their tails (a blocked batch of
        n stripes in host memory, ecx.h's layout)."""
        if self.layout != "blocked":
            return [self.pool[:n].reshape(-1)]
        full, tail = divmod(self.L, self.block)
        body = full * self.n * self.block
        out = [self.pool[:n * body]] if full else []
        if tail:
            t0 = self.P * body
            out.append(self.pool[t0:t0 + n * self.n * tail])
        return out


class RS124(_RsLayout, Workload):
    """Config 5: RS(12,4), 4 MiB shards, erasures {0,1} decoded in place (the first 12
    present shards, ReedSolomon.decodeMissing)."""
    k, m, L, n = 12, 4, 4 << 20, 16
    reads, writes = 12, 2
    unit_bytes = 14 * (4 << 20)
    write_bytes = 2 * (4 << 20)

    def __init__(self, ecx, torch, dev, P, pad, seed, layout="natural", pitch=None):
        self.P, self.torch, self.ecx, self.layout = P, torch, ecx, layout
        rs = ecx.ReedSolomon.create(self.k, self.m)
        self.rs = rs
        L = self.L
        self.pitch = L if layout == "blocked" else _resolve_pitch(rs, pitch, L, pad)
        p = self.pitch
        nat = torch.empty((P, 16, p), dtype=torch.uint8, device=dev)
        ecx.fill_random(nat, nat.numel(), seed)
        rs.encode_map().apply_batch(nat, 16 * p, p, nat, 16 * p, p, P, L)
        self.orig = nat[:, 0:2, :L].clone()
        nat[:, 0:2, :L] = 0  # the erased shards
        self.present = [False, False] + [True] * 14
        self.dmap = rs.decode_map(self.present)
        if layout == "blocked":
            self.block = rs.blockedLayout(L)[0]
            self.pool = ecx.blocked_pack(nat[:, :, :L], self.block)
            del nat
            self.pitch = self.block  # the slot pitch the decode's launches see
        else:
            self.pool = nat
        self.region = self.pool
        self.description = "RS(12,4) 2-erasure decode {0,1} in place, 4 MiB shards, %s" % self._layout_desc()

    def launch(self):
        if self.layout == "blocked":
            self.rs.decodeMissingBlockedBatch(self.pool, self.present, self.P, self.L)
            return
        p = self.pitch
        self.dmap.apply_batch(self.pool, 16 * p, p, self.pool, 16 * p, p, self.P, self.L)

    def selected_map(self):
        return self.dmap, self.pitch

    def host_out_bytes(self):
        return 0

    def host_call(self, hin, hout, n):
        if self.layout == "blocked":
            # the full blocks, then the tails: two pipelined host batches (ecx_rs_*_blocked_batch_host)
            self.rs.decodeMissingBlockedBatchHost(hin, self.present, n, self.L, self.block)
            return
        p = self.pitch
        self.dmap.apply_batch_host(hin, 16 * p, p, hin, 16 * p, p, n, self.L)

    def host_plan(self, n):
        if self.layout == "blocked":
            return None  # two passes (full blocks, tails)
        p = self.pitch
        return self.dmap.host_plan(16 * p, p, 16 * p, p, n, self.L)

    def sub_bytes(self):
        return self.L

    def verify(self):
        return all(bool(self.torch.equal(self.stripes(s0, min(64, self.P - s0), [0, 1]), self.orig[s0:s0 + 64]))
                   for s0 in range(0, self.P, 64))

    def sample(self):
        s = self.P // 2
        st = self.stripes(s, 1)[0]
        return st.cpu().numpy(), st[0:2].cpu().numpy()

    def oracle_check(self, stripe, got):
        import numpy as np
        import oracle as O
        shards = [np.zeros(self.L, np.uint8) if i < 2 else stripe[i].copy() for i in range(16)]
        O.ReedSolomon(self.k, self.m).decode_missing(shards, [i >= 2 for i in range(16)], 0, self.L)
        return bool((shards[0] == got[0]).all() and (shards[1] == got[1]).all())

    def cpu_spec(self):
        import numpy as np
        import oracle as O

        def make(rng):  # random bytes: decodeMissing's work does not depend on the data
            return [rng.integers(0, 256, (16, self.L), dtype=np.uint8) for _ in range(2)]
        return {"op": O.BENCH_RS_DECODE, "data": self.k, "parity": self.m, "erased": [0, 1], "make": make,
                "arena_slot": np.arange(16), "present": np.ones(16, np.int64), "data_kind": "random-byte",
                "what": "RS(12,4) decodeMissing of shards {0, 1} in place (first-k-present rule, sub-matrix "
                        "inverted per call as ReedSolomon.java:224-244 does), 4 MiB shards"}


class RS173(_RsLayout, Workload):
    """The reference's published benchmark shape (rs/README.md:53, ReedSolomonBenchmark.java:
    25-33,104-124): RS(17,3) encodeParity over 200,000-byte shards, parity written in place.
    Natural layout: shards back to back (pitch 200,000 B), every other slot 64 B off a 128-B
    line and each shard ending in a 320-B partial chunk, as DESIGN.md section 4 measures; or a
    padded pitch (--pitch), or the blocked layout contract (--layout blocked)."""
    k, m, L, n = 17, 3, 200 * 1000, 20
    reads, writes = 17, 3
    unit_bytes = 20 * 200 * 1000        # 17 shards read + 3 written (roofline bytes)
    write_bytes = 3 * 200 * 1000
    metric_unit, metric_scale, metric_bytes = "MB/s", 1e6, 17 * 200 * 1000  # data bytes, 10^6
    data_desc = "synthetic (device splitmix64 data shards; the timed launch is the encode itself)"

    def __init__(self, ecx, torch, dev, P, seed, layout="natural", pitch=None):
        self.P, self.torch, self.ecx, self.layout = P, torch, ecx, layout
        L = self.L
        self.rs = ecx.ReedSolomon.create(self.k, self.m)
        if layout == "blocked":
            self.block = self.rs.blockedLayout(L)[0]
            self.pitch = self.block
            self.pool = torch.empty(P * 20 * L, dtype=torch.uint8, device=dev)
        else:
            self.pitch = _resolve_pitch(self.rs, pitch, L)
            self.pool = torch.empty((P, 20, self.pitch), dtype=torch.uint8, device=dev)
        ecx.fill_random(self.pool, self.pool.numel(), seed)
        self.region = self.pool
        self.description = ("RS(17,3) encodeParity in place, 200,000-B shards, %s%s" %
                            (self._layout_desc(), " (the published shape)" if self.pitch == L else ""))

    def launch(self):
        if self.layout == "blocked":
            self.rs.encodeParityBlockedBatch(self.pool, self.P, self.L)
            return
        p = self.pitch
        self.rs.encodeParityBatch(self.pool, 20 * p, p, self.P, 0, self.L)

    def selected_map(self):
        return self.rs.encode_map(), self.pitch

    def host_out_bytes(self):
        return 0

    def host_call(self, hin, hout, n):
        if self.layout == "blocked":
            self.rs.encodeParityBlockedBatchHost(hin, n, self.L, self.block)
            return
        p = self.pitch
        self.rs.encode_map().apply_batch_host(hin, 20 * p, p, hin, 20 * p, p, n, self.L)

    def host_plan(self, n):
        if self.layout == "blocked":
            return None  # two passes (full blocks, tails)
        p = self.pitch
        return self.rs.encode_map().host_plan(20 * p, p, 20 * p, p, n, self.L)

    def verify(self):
        """The parity the GPU wrote equals the oracle's on two stripes, and re-encoding
        leaves the whole pool unchanged (isParityCorrect over every stripe)."""
        before = self.pool.clone()
        self.launch()
        self.torch.cuda.synchronize()
        same = bool(self.torch.equal(before, self.pool))
        del before
        return same and all(self.oracle_check(*self._stripe_and_parity(s)) for s in (0, self.P - 1))

    def _stripe_and_parity(self, s):
        st = self.stripes(s, 1)[0]
        return st.cpu().numpy(), st[self.k:].cpu().numpy()

    def sample(self):
        return self._stripe_and_parity(self.P // 2)

    def oracle_check(self, stripe, got):
        import oracle as O
        shards = [stripe[i].copy() for i in range(20)]
        for i in range(self.k, 20):
            shards[i][:] = 0
        O.ReedSolomon(self.k, self.m).encode_parity(shards, 0, self.L)
        return all(bool((shards[self.k + j] == got[j]).all()) for j in range(self.m))

    def cpu_spec(self):
        import numpy as np
        import oracle as O

        def make(rng):  # random data shards: encodeParity's work does not depend on the data
            return [rng.integers(0, 256, (20, self.L), dtype=np.uint8) for _ in range(8)]
        return {"op": O.BENCH_RS_ENCODE, "data": self.k, "parity": self.m, "erased": [], "make": make,
                "arena_slot": np.arange(20), "present": np.ones(20, np.int64), "data_kind": "random-byte",
                "what": "RS(17,3) encodeParity (InputOutputByteTableCodingLoop, ReedSolomon.java:94-108), "
                        "200,000-B shards"}


class RS173Check(RS173):
    """ReedSolomonBenchmark's "Check" half (ReedSolomonBenchmark.java:73-87,126-149): RS(17,3)
    isParityCorrect (ReedSolomon.java:129-178) over the encoded pool of 200,000-B shards,
    read-only (k_gf_check: the syndromes OR-folded in registers, one verdict byte per stripe).
    The roofline prices the 20 shards read per stripe; nothing is written but the verdicts."""
    reads, writes = 20, 0
    unit_bytes = 20 * 200 * 1000        # 17 data + 3 parity shards read
    write_bytes = 0
    metric_bytes = 17 * 200 * 1000      # bytesChecked += BUFFER_SIZE * DATA_COUNT (:139)
    data_desc = "synthetic (device splitmix64 data shards, GPU encodeParity; the timed launch is the check itself)"

    def __init__(self, ecx, torch, dev, P, seed):
        super().__init__(ecx, torch, dev, P, seed)
        RS173.launch(self)  # valid parity everywhere, as the benchmark's encode pass leaves it
        self.verdict = torch.zeros(P, dtype=torch.uint8, device=dev)
        self.description = ("RS(17,3) isParityCorrect (read-only, one verdict per stripe), 200,000-B shards back to "
                             "back (the published shape)")

    def launch(self):
        self.rs.isParityCorrectBatch(self.pool, 20 * self.L, self.L, self.P, 0, self.L, self.verdict)

    def selected_map(self):
        return None

    def host_out_bytes(self):
        return 1  # one verdict byte per stripe comes back

    def host_call(self, hin, hout, n):  # pipelined H2D of the 20 shards, the check, the verdicts D2H
        self.rs.isParityCorrectBatchHost(hin, 20 * self.L, self.L, n, 0, self.L, hout)

    def host_expect(self, hin, hout, n):
        """Every host stripe (a copy of the valid pool) passes, as the device check says."""
        return bool((hout[:n] == 1).all()) and bool((self.verdict[:n] == 1).all())

    def pcie_bytes(self):
        return 20 * self.L, 1

    def verify(self):
        """Every stripe passes; a flipped byte in a data shard (stripe 1, byte 0), in a parity
        shard (stripe P-2, the 3,392-B partial last chunk) fails exactly that stripe; both are
        restored afterwards; the verdicts equal the oracle's isParityCorrect on those stripes."""
        import oracle as O
        self.launch()
        self.torch.cuda.synchronize()
        if not bool((self.verdict == 1).all()):
            return False
        bad = [(1, 0, 0), (self.P - 2, 18, self.L - 100)]
        for s_, sh, b in bad:
            self.pool[s_, sh, b] ^= 0x40
        self.launch()
        self.torch.cuda.synchronize()
        got = self.verdict.cpu().numpy()
        want = [0 if s_ in (1, self.P - 2) else 1 for s_ in range(self.P)]
        ok = got.tolist() == want
        for s_, _, _ in bad:
            shards = [x.copy() for x in self.pool[s_].cpu().numpy()]
            ok = ok and not O.ReedSolomon(self.k, self.m).is_parity_correct(shards, 0, self.L)
        for s_, sh, b in bad:
            self.pool[s_, sh, b] ^= 0x40
        self.launch()
        self.torch.cuda.synchronize()
        return ok and bool((self.verdict == 1).all())

    def sample(self):
        s_ = self.P // 2
        return self.pool[s_].cpu().numpy(), self.verdict[s_:s_ + 1].cpu().numpy()

    def oracle_check(self, stripe, got):
        import oracle as O
        shards = [stripe[i].copy() for i in range(20)]
        return bool(O.ReedSolomon(self.k, self.m).is_parity_correct(shards, 0, self.L)) == bool(got[0])

    def cpu_spec(self):
        import numpy as np
        import oracle as O

        def make(rng):  # valid stripes: the check must pass (the benchmark throws otherwise)
            out = []
            for _ in range(8):
                st = rng.integers(0, 256, (20, self.L), dtype=np.uint8)
                shards = [st[i] for i in range(20)]
                O.ReedSolomon(self.k, self.m).encode_parity(shards, 0, self.L)
                out.append(st)
            return out
        return {"op": O.BENCH_RS_CHECK, "data": self.k, "parity": self.m, "erased": [], "make": make,
                "arena_slot": np.arange(20), "present": np.ones(20, np.int64), "data_kind": "valid-stripe",
                "what": "RS(17,3) isParityCorrect with a temp buffer (ReedSolomon.java:159-178, "
                        "InputOutputByteTableCodingLoop.checkSomeShards), 200,000-B shards"}


class LRCEncode(Workload):
    """Config 3, encode half (LRCErasureCodeExample.kt:30-60): each local group of 3 data
    blocks gets its XOR parity (RS(3,1) encodeParity, parity row [1, 1, 1]), written in place
    into the stripe's [d d d p] x 4 layout, 64 KiB blocks."""
    b = 65536
    reads, writes = 12, 4
    unit_bytes = 16 * 65536
    write_bytes = 4 * 65536
    data_desc = "synthetic (device splitmix64 data blocks; the timed launch is the encode itself)"

    def __init__(self, ecx, torch, dev, P, seed):
        import numpy as np
        b = self.b
        self.P, self.torch = P, torch
        self.pool = torch.empty((P, 16, b), dtype=torch.uint8, device=dev)
        ecx.fill_random(self.pool, self.pool.numel(), seed)
        enc = np.zeros((4, 16), np.uint8)
        for g in range(4):
            enc[g, 4 * g:4 * g + 3] = 1
        self.emap = ecx.GfMap.from_matrix(enc, in_slot=list(range(16)), out_slot=[3, 7, 11, 15])
        self.region = self.pool
        self.description = "LRC(12 data, 4 XOR local parities) encode in place, 64 KiB blocks"

    def launch(self):
        b = self.b
        self.emap.apply_batch(self.pool, 16 * b, b, self.pool, 16 * b, b, self.P, b)

    def selected_map(self):
        return self.emap, self.b

    def host_out_bytes(self):
        return 0

    def host_call(self, hin, hout, n):
        b = self.b
        self.emap.apply_batch_host(hin, 16 * b, b, hin, 16 * b, b, n, b)

    def host_plan(self, n):
        b = self.b
        return self.emap.host_plan(16 * b, b, 16 * b, b, n, b)

    def verify(self):
        """Re-encoding leaves every stripe unchanged, and two stripes' parities equal the oracle's."""
        before = self.pool[:, 3::4].clone()
        self.launch()
        self.torch.cuda.synchronize()
        same = bool(self.torch.equal(before, self.pool[:, 3::4]))
        return same and all(self.oracle_check(self.pool[s].cpu().numpy(), self.pool[s, 3::4].cpu().numpy())
                            for s in (0, self.P - 1))

    def host_units(self, k):
        # CPU units are local groups (3 data blocks + parity), as the reference encodes them
        return [self.pool[i // 4, 4 * (i % 4):4 * (i % 4) + 4].cpu().numpy() for i in range(min(k, 4 * self.P))]

    def sample(self):
        s = self.P // 2
        return self.pool[s].cpu().numpy(), self.pool[s, 3::4].cpu().numpy()

    def oracle_check(self, stripe, got):
        import numpy as np
        import oracle as O
        for g in range(4):
            group = [stripe[4 * g + i].copy() for i in range(3)] + [np.zeros(self.b, np.uint8)]
            O.ReedSolomon(3, 1).encode_parity(group, 0, self.b)
            if not (group[3] == got[g]).all():
                return False
        return True

    def cpu_spec(self):
        import numpy as np
        import oracle as O

        def make(rng):  # one local group (3 data blocks + parity), random bytes
            return [rng.integers(0, 256, (4, self.b), dtype=np.uint8) for _ in range(8)]
        return {"op": O.BENCH_RS_ENCODE, "data": 3, "parity": 1, "erased": [], "make": make,
                "arena_slot": np.arange(4), "present": np.ones(4, np.int64), "data_kind": "random-byte",
                "unit_bytes": 4 * self.b,
                "what": "LRC local-parity encodes: RS(3,1).encodeParity per local group (LRCErasureCodeExample.kt:30-60), "
                        "64 KiB blocks"}


class LRC(Workload):
    """Config 3: LRC (LRCErasureCodeExample shapes: 12 data blocks in 4 local groups of 3,
    each with an XOR parity), 64 KiB blocks; repair of data block 2 from its group."""
    b = 65536
    reads, writes = 3, 1
    unit_bytes = 4 * 65536
    write_bytes = 65536

    def __init__(self, ecx, torch, dev, P, seed):
        import numpy as np
        b = self.b
        self.P, self.torch = P, torch
        self.pool = torch.empty((P, 16, b), dtype=torch.uint8, device=dev)
        ecx.fill_random(self.pool, self.pool.numel(), seed)
        enc = np.zeros((4, 16), np.uint8)
        for g in range(4):
            enc[g, 4 * g:4 * g + 3] = 1
        ecx.GfMap.from_matrix(enc, in_slot=list(range(16)), out_slot=[3, 7, 11, 15]).apply_batch(
            self.pool, 16 * b, b, self.pool, 16 * b, b, P, b)
        rs = ecx.ReedSolomon.create(3, 1)
        mat, _ins, _outs = rs.decode_map([True, True, False, True]).matrix()
        self.rmap = ecx.GfMap.from_matrix(mat, in_slot=[0, 1, 3], out_slot=[0])
        self.out = torch.empty((P, 1, b), dtype=torch.uint8, device=dev)
        self.region = self.pool
        self.description = "LRC(12 data, 4 XOR local parities) repair of data block 2, 64 KiB blocks"

    def launch(self):
        b = self.b
        self.rmap.apply_batch(self.pool, 16 * b, b, self.out, b, b, self.P, b)

    def host_call(self, hin, hout, n):
        b = self.b
        self.rmap.apply_batch_host(hin, 16 * b, b, hout, b, b, n, b)

    def host_plan(self, n):
        b = self.b
        return self.rmap.host_plan(16 * b, b, b, b, n, b)

    def verify(self):
        return bool(self.torch.equal(self.out[:, 0], self.pool[:, 2]))

    def host_units(self, k):
        return [self.pool[i, 0:4].cpu().numpy() for i in range(min(k, self.P))]

    def sample(self):
        s = self.P // 2
        return self.pool[s].cpu().numpy(), self.out[s].cpu().numpy()

    def oracle_check(self, stripe, got):
        import numpy as np
        import oracle as O
        group = [stripe[i].copy() for i in range(4)]
        group[2] = np.zeros(self.b, np.uint8)
        O.ReedSolomon(3, 1).decode_missing(group, [True, True, False, True], 0, self.b)
        return bool((group[2] == got[0]).all())

    def cpu_spec(self):
        import numpy as np
        import oracle as O

        def make(rng):  # the local group of block 2 (blocks 0-3), random bytes
            return [rng.integers(0, 256, (4, self.b), dtype=np.uint8) for _ in range(8)]
        return {"op": O.BENCH_RS_DECODE, "data": 3, "parity": 1, "erased": [2], "make": make,
                "arena_slot": np.arange(4), "present": np.ones(4, np.int64), "data_kind": "random-byte",
                "what": "LRC local-group repairs of data block 2: RS(3,1).decodeMissing over its group "
                        "(LRCErasureCodeExample.kt:100-131), 64 KiB blocks"}


def launch_ranks(args) -> int:
    """`--gpus N` (N > 1) without a launcher: start N fresh rank processes through
    torch.distributed.run as a CHILD process (this process never touches the GPU and
    never execs), with the same arguments.  Rank 0's JSON line reaches stdout through
    the inherited stream; the exit status is the launcher's, non-zero if any rank failed."""
    import socket
    import subprocess
    with socket.socket() as sk:  # a free rendezvous port on the loopback interface
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, str(Path(__file__).resolve())] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        raise SystemExit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d: launch one rank per GPU" % (args.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    import rpamd
    ecx = rpamd.load(shape_knobs=any(kv.partition("=")[0] not in DEPLOYMENT_KEYS for kv in args.tune))

    # ECX_BENCH_BACKEND=gloo rehearses the multi-process path on a box with fewer
    # GPUs than ranks (ranks share devices round-robin); the default is RCCL, which
    # needs one GPU per rank.
    backend = os.environ.get("ECX_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and world > max(1, ndev):
        raise SystemExit("bench.py: %d ranks but %d visible GPUs (RCCL needs one GPU per rank; "
                         "ECX_BENCH_BACKEND=gloo shares devices for a rehearsal)" % (world, ndev))
    local = local % max(1, ndev)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # Under a launcher (WORLD_SIZE set) the process group is created even for one rank, so
    # `torch.distributed.run --nproc-per-node 1` rehearses the RCCL init, barriers and
    # max-reduction of the N-GPU path on a one-GPU box; a plain `python bench.py` has none.
    grouped = "WORLD_SIZE" in os.environ
    if grouped:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    ecx.set_device(local)
    for kv in args.tune:
        key, _, val = kv.partition("=")
        ecx.tune(key, int(val))

    P = args.pool
    rss_stages = {"init": _peak_rss_bytes()}  # peak host RSS after each stage (the line's host_rss_MiB)
    passes = max(1, args.stripes_per_step // P)
    stripes_per_step = passes * P
    seed = 0x5EED + rank

    # ---- resident pool of valid stripes: random data + GPU encode
    if args.workload == "clay42":
        wl = Clay42(ecx, torch, dev, P, args.erased, seed)
    elif args.workload == "clay104":
        wl = Clay104(ecx, torch, dev, P, args.erased, seed, args.sub_bytes)
    elif args.workload == "clay42x2":
        wl = Clay42x2(ecx, torch, dev, P, args.erased, seed)
    elif args.workload == "rs124":
        wl = RS124(ecx, torch, dev, P, args.pitch_pad, seed, args.layout, args.pitch)
    elif args.workload == "rs173":
        wl = RS173(ecx, torch, dev, P, seed, args.layout, args.pitch)
    elif args.workload == "rs173check":
        wl = RS173Check(ecx, torch, dev, P, seed)
    elif args.workload == "lrcenc":
        wl = LRCEncode(ecx, torch, dev, P, seed)
    else:
        wl = LRC(ecx, torch, dev, P, seed)

    wl.launch()
    torch.cuda.synchronize()
    kernel = ecx.last_kernel()  # the instance launch_apply actually chose for this map and layout
    rss_stages["pool"] = _peak_rss_bytes()
    verified = None
    if not args.no_verify:
        verified = wl.verify()
        if not verified:
            raise SystemExit("repair output differs from the erased originals")

    # Maps whose launch shape is selected per batch layout (ecx_tune "layout_select") time
    # their candidate shapes on their first calls; those calls run here, untimed, until the
    # choice is made (at most 64 launches), so the timed region runs the kept shape.
    launch_shape = None
    sel = wl.selected_map()
    if sel is not None:
        gm, pitch = sel
        for _ in range(64):
            if gm.layout_choice(pitch) != -1:
                break
            wl.launch()
            torch.cuda.synchronize()
        wl.launch()  # the kept shape (or the static rules, if the layout is not selected per launch)
        torch.cuda.synchronize()
        kernel = ecx.last_kernel()
        choice, med = gm.layout_choice(pitch, with_times=True)
        state, dropped = gm.layout_state(pitch)
        launch_shape = {"layout_select": choice, "candidate_median_ms": med, "kernel": kernel,
                        "state": state, "probes_dropped": dropped}
        if not args.no_verify and not wl.verify():
            raise SystemExit("output differs from the erased originals after the layout selection")

    for _ in range(args.warmup):
        for _ in range(passes):
            wl.launch()
    torch.cuda.synchronize()
    if args.warmup:
        kernel = ecx.last_kernel()  # after the layout selection: the instance the timed region runs
    shape = ecx.last_launch_shape()  # the kernel instance plus the unit order (stagger, XCD runs)

    rss_stages["verify_warmup"] = _peak_rss_bytes()
    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps * passes)]
    if grouped:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    i = 0
    for _ in range(args.steps):
        for _ in range(passes):
            evs[i][0].record(stream)
            wl.launch()
            evs[i][1].record(stream)
            i += 1
    torch.cuda.synchronize()
    if grouped:
        dist.barrier()
    el = time.perf_counter() - t0
    own_el = el
    if grouped:
        t = torch.tensor([el], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    launch_times = [a.elapsed_time(b) for a, b in evs]
    launch_ms = sum(launch_times) / len(launch_times)
    # the spread of the timed launches, first and last step apart: a memory system still busy
    # with something else early in the run (e.g. the driver clearing VRAM a previous process
    # freed) shows as a slower first step
    per_step = [sum(launch_times[i * passes:(i + 1) * passes]) / passes for i in range(args.steps)]
    launch_spread = {"min": round(min(launch_times), 4), "max": round(max(launch_times), 4),
                     "first_step": round(per_step[0], 4), "last_step": round(per_step[-1], 4)}
    per_launch_bytes = P * wl.unit_bytes
    achieved = per_launch_bytes / (launch_ms * 1e-3) / 1e9
    total_stripes = stripes_per_step * args.steps * world
    metric_bytes = wl.metric_bytes or wl.unit_bytes
    value = total_stripes * metric_bytes / el / wl.metric_scale
    traffic, traffic_note = pmc_traffic(profile_key(args), P, kernel, shape)

    # per-rank rates, so an N-GPU efficiency shortfall can be attributed to a rank
    per_rank = [own_el]
    if grouped:
        g = [torch.zeros(1, dtype=torch.float64, device=dev if backend == "nccl" else "cpu") for _ in range(world)]
        dist.all_gather(g, torch.tensor([own_el], dtype=torch.float64, device=g[0].device))
        per_rank = [float(x.item()) for x in g]
    per_rank_gibs = [stripes_per_step * args.steps * metric_bytes / e / wl.metric_scale for e in per_rank]

    # the end-to-end leg: every rank at once (they share the host's PCIe and memory), after the
    # timed region; the line carries rank 0's figures and the whole-job sum
    e2e = None
    if args.e2e_seconds > 0:
        if grouped:
            dist.barrier()
        rss_before = _peak_rss_bytes()  # the process before the leg: torch + HIP runtime, the bench's own state
        mine = e2e_rate(ecx, torch, wl, args.e2e_seconds, world)
        if mine is not None:
            # (rate, peak host RSS before / after the leg) of every rank; a rank that skipped
            # the leg reports rate -1
            own = [mine.get("GiBps", -1.0), float(rss_before), float(_peak_rss_bytes())]
            rows = [own]
            if grouped:
                g = [torch.zeros(3, dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
                     for _ in range(world)]
                dist.all_gather(g, torch.tensor(own, dtype=torch.float64, device=g[0].device))
                rows = [[float(v) for v in x.tolist()] for x in g]
            rates = [r[0] for r in rows]
            rss = {"per_rank_MiB": [round(r[2] / 2**20) for r in rows], "max_MiB": round(max(r[2] for r in rows) / 2**20),
                   "before_leg_per_rank_MiB": [round(r[1] / 2**20) for r in rows]}
            if "skipped" in mine:
                e2e = dict(mine, peak_rss=rss)
            else:
                e2e = dict(mine, rank0_GiBps=mine["GiBps"], GiBps=round(sum(r for r in rates if r >= 0), 3),
                           per_rank_GiBps=[round(r, 3) for r in rates], peak_rss=rss)

    sample = units = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:  # the contract: rank 0 at N=1 only
        sample = wl.sample()  # one pool unit for the oracle check
        units = wl.host_units(8 if wl.unit_bytes < (64 << 20) else (2 if wl.unit_bytes < (1 << 30) else 1))
    probes = memory_probes(ecx, torch, wl.region, wl.reads, wl.writes) if not args.no_probes else None

    cpu = None
    if sample is not None:  # rank 0 at N=1 only, after the timed region
        cpu = cpu_baseline(wl, args.cpu_seconds, sample, units=units, protocol=args.cpu_protocol)
        if wl.metric_unit != "GiB/s":  # the line's own unit: metric bytes per metric_scale
            f = 2**30 / wl.metric_scale * metric_bytes / wl.unit_bytes
            cpu["algorithmic_GiBps"] = cpu["value"]
            cpu["value"], cpu["unit"] = round(cpu["value"] * f, 1), wl.metric_unit
            cpu["single_thread_value"] = round(cpu["single_thread_value"] * f, 1)

    if rank == 0 and args.meta:
        Path(args.meta).write_text(json.dumps({
            "workload": profile_key(args), "kernel": kernel, "launch_shape": shape, "tune": args.tune,
            "pool_stripes": P, "unit_bytes": wl.unit_bytes,
            "write_bytes_per_unit": wl.write_bytes, "algorithmic_bytes_per_launch": per_launch_bytes,
            "kernel_source_hash": kernel_source_hash(kernel), "avg_launch_ms": launch_ms}) + "\n")
    if rank == 0:
        line = {
            "metric": WORKLOADS[args.workload][0],
            "value": round(value, 3),
            "unit": wl.metric_unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / PUBLISHED[args.workload], 1) if args.workload in PUBLISHED else None,
            "dtype": "u8",
            "data": wl.data_desc,
            "config": {
                "workload": "%s, %d stripes per GPU per step over a resident pool of %d" % (wl.description,
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
                "traffic_note": traffic_note,
                "kernel": kernel,
                "kernel_source_hash": kernel_source_hash(kernel),
                "avg_launch_ms": round(launch_ms, 4), "launch_ms_spread": launch_spread,
                "algorithmic_bytes_per_launch": per_launch_bytes,
                "measured_ceilings": probes,
                "launch_shape": dict(launch_shape or {}, name=shape),
                "frac_of_mix_model": round(achieved / probes["mix_model_GBps"], 4) if probes else None,
            },
            "repaired_output_GiBps": round(total_stripes * wl.write_bytes / el / 2**30, 3),
            "per_rank_%s" % ("GiBps" if wl.metric_unit == "GiB/s" else "MBps"): {"min": round(min(per_rank_gibs), 3), "max": round(max(per_rank_gibs), 3),
                               "ranks": [round(v, 3) for v in per_rank_gibs]},
            "cpu_baseline": cpu,
            "e2e": e2e,
            "host_rss_MiB": {k: round(v / 2**20) for k, v in dict(rss_stages, end=_peak_rss_bytes()).items()},
            "verified": verified,
        }
        print(json.dumps(line), flush=True)
    if grouped:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
