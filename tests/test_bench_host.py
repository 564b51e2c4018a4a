"""Host logic of bench.py (no GPU): the kernel-source hash families behind
roofline.traffic, the staleness rules of pmc_traffic(), the --gpus / WORLD_SIZE guard,
and the self-launch of N ranks propagating a failing rank's status."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def test_source_hash_families_are_separate_and_stable():
    """Each kernel family hashes its own sources: a change to the generated Clay kernels
    does not stale the composed-map profile, and the other way round."""
    composed = bench.kernel_source_hash("k_gf_apply<false, true, 1, 20, false, 256, 8>")
    assert composed == bench.kernel_source_hash("k_gf_apply_wide<false, true, 1, 8>")
    assert composed == bench.kernel_source_hash("k_gf_lut<0, true>")  # launch_apply can pick it
    clay = bench.kernel_source_hash("k_clay_repair_grp")
    planes = bench.kernel_source_hash("k_map_planes")
    assert len({composed, clay, planes}) == 3
    assert all(len(h) == 16 for h in (composed, clay, planes))
    assert clay == bench.kernel_source_hash("k_clay_repair_grp")
    # every source a family names exists (a renamed file must not silently drop out)
    for name in bench.COMMON_SOURCES + bench.COMPOSED_SOURCES + bench.RTC_SOURCES + bench.PLANES_SOURCES:
        assert (ROOT / "repair-pipelining_amd" / "csrc" / name).is_file(), name


def test_committed_pmc_profile_matches_current_sources():
    """profiles/pmc_traffic.json was taken on the sources in this tree for every bench
    workload, so the bench line carries measured traffic (not a stale constant)."""
    d = json.loads((ROOT / "profiles" / "pmc_traffic.json").read_text())["workloads"]
    assert set(d) >= {"clay42", "clay104", "rs124", "lrc", "clay42x2"}
    stale = [w for w, e in d.items() if bench.pmc_traffic(w, e["pool_stripes"], e["kernel"])[1] is not None]
    if stale:  # kernel sources edited since the last PMC pass: the bench reports traffic null until re-profiled
        pytest.skip("PMC profile stale for %s: re-run scripts/pmc.sh + scripts/pmc_summary.py on a GPU" % stale)
    for w, e in d.items():
        traffic, note = bench.pmc_traffic(w, e["pool_stripes"], e["kernel"])
        assert note is None and traffic == e["hbm_bytes_per_launch"], (w, note)
        # within 0.1 % of the algorithmic bytes on the composed maps; Clay(10,4)'s plane-group
        # kernel measures 1.004-1.021x across rounds; RS(17,3)'s 200,000-B
        # shards leave every other slot 64 B off a 128-B line (reads ~1.035x)
        bound = {"clay104": 1.03, "clay104_sub1048576": 1.03, "rs173": 1.05, "rs173check": 1.05,
                 "rs173_pitchrecommended": 1.05}.get(w, 1.001)
        lo = 1.0
        if w.endswith("_blocked"):  # the profiled kernel is the full-block launch; the tails run apart
            L = {"rs173": 200000, "rs124": 4 << 20}[w.split("_")[0]]
            block, full, _tail = {"rs173": (32768, 6, 3392), "rs124": (65536, 64, 0)}[w.split("_")[0]]
            lo = full * block / L
        assert lo <= traffic / e["algorithmic_bytes_per_launch"] < bound * lo, w


def test_pmc_traffic_staleness_rules(monkeypatch):
    d = json.loads((ROOT / "profiles" / "pmc_traffic.json").read_text())["workloads"]["clay42"]
    pool, kernel = d["pool_stripes"], d["kernel"]
    # as if the tree's sources were the profiled ones (freshness itself is the test above)
    monkeypatch.setattr(bench, "kernel_source_hash", lambda kernel="": d["kernel_source_hash"])
    assert bench.pmc_traffic("clay42", pool, kernel)[0] == d["hbm_bytes_per_launch"]
    assert bench.pmc_traffic("clay42", pool * 2, kernel) == (
        None, "stale: PMC profile taken on another pool size or kernel instance")
    assert bench.pmc_traffic("no_such_workload", pool, kernel) == (None, "no PMC profile for this workload")
    monkeypatch.setattr(bench, "kernel_source_hash", lambda kernel="": "0" * 16)
    assert bench.pmc_traffic("clay42", pool, kernel) == (None, "stale: PMC profile taken on other kernel sources")


def _run_bench(args, env_extra, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, env=env, capture_output=True, text=True,
                          timeout=timeout, cwd=str(ROOT))


def test_gpus_must_match_world_size():
    """Under an external launcher, a --gpus that differs from WORLD_SIZE is refused
    before anything touches a device (a scaling record must never measure fewer GPUs
    than it claims)."""
    r = _run_bench(["--gpus", "2"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert r.returncode != 0
    assert "--gpus 2 but WORLD_SIZE=3" in r.stderr


def test_self_launch_propagates_a_failing_rank():
    """`bench.py --gpus 2` without a launcher starts 2 ranks through torch.distributed.run
    as a child process; with no usable GPU here every rank fails, and the failure must
    reach the exit status (not a silent one-GPU line)."""
    import torch
    if torch.cuda.device_count() > 0:  # counting devices does not initialise HIP on this image
        pytest.skip("a GPU is visible: the ranks would run the real bench")
    r = _run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--cpu-seconds", "0", "--no-probes"],
                   {"ECX_BENCH_BACKEND": "gloo", "MASTER_ADDR": "127.0.0.1"})
    assert r.returncode != 0
    assert '"n_gpus"' not in r.stdout


def _bare(cls, **attrs):
    """A workload object with only the attributes its oracle hooks read (no GPU pool)."""
    wl = object.__new__(cls)
    for k, v in attrs.items():
        setattr(wl, k, v)
    return wl


@pytest.mark.parametrize("case", ["clay42", "clay42x2", "clay104", "rs124", "lrc", "rs173", "lrcenc"])
def test_cpu_baseline_every_workload(case):
    """Every bench workload has an oracle baseline (the reference path
    restated by oracle/, timed by oracle/orc_bench.c orc_bench_run), here on a bounded
    arena: the line's fields are filled and the rate is positive."""
    if case == "clay42":
        wl = _bare(bench.Clay42, erased=1)
    elif case == "clay42x2":
        wl = _bare(bench.Clay42x2, erased=0, unit_bytes=48 * bench.B)
    elif case == "clay104":
        wl = _bare(bench.Clay104, erased=3, n=14, unit_bytes=1088 * 4096)
    elif case == "rs124":
        wl = _bare(bench.RS124)
    elif case == "rs173":
        wl = _bare(bench.RS173)
    elif case == "lrcenc":
        wl = _bare(bench.LRCEncode)
    else:
        wl = _bare(bench.LRC)
    cpu = bench.cpu_baseline(wl, 0.2, None, max_units=2)
    assert cpu["kind"] == "port" and cpu["unit"] == "GiB/s" and cpu["cores"] >= 1
    assert cpu["value"] > 0 and cpu["single_thread_value"] > 0
    assert cpu["oracle_check"] is None and "oracle/" in cpu["sample"]


def test_cpu_baseline_on_given_units_reference_protocol(monkeypatch):
    """The baseline runs on the units it is handed (the GPU pool's own stripes in bench.py)
    and, under protocol "reference", reports the mean of REF_MEASUREMENTS measurements after
    REF_WARMUPS warm-ups (shortened here)."""
    import numpy as np
    monkeypatch.setattr(bench, "REF_SECONDS", 0.02)
    wl = _bare(bench.LRC)
    shape = wl.cpu_spec()["make"](np.random.default_rng(0))[0].shape
    units = [np.random.default_rng(i).integers(0, 256, shape, dtype=np.uint8) for i in range(3)]
    cpu = bench.cpu_baseline(wl, 0.2, None, max_units=3, units=units, protocol="reference")
    assert cpu["protocol"] == "reference" and "GPU-pool" in cpu["sample"]
    assert len(cpu["measurements_GiBps"]["threads"]) == bench.REF_MEASUREMENTS
    assert len(cpu["measurements_GiBps"]["one"]) == bench.REF_MEASUREMENTS
    assert cpu["value"] > 0 and cpu["single_thread_value"] > 0


def test_oracle_checks_of_the_workloads():
    """The sampled byte-compare of each workload agrees with an oracle-made unit and
    rejects a corrupted output byte (rs124 / lrc / clay104 on small host stand-ins)."""
    import numpy as np
    import oracle as O
    rng = np.random.default_rng(1)
    # LRC: group [d0 d1 d2 p] with p = d0 ^ d1 ^ d2; repair of block 2
    lrc = _bare(bench.LRC, b=256)
    st = rng.integers(0, 256, (16, 256), dtype=np.uint8)
    st[3] = st[0] ^ st[1] ^ st[2]
    assert lrc.oracle_check(st, st[2:3].copy())
    bad = st[2:3].copy()
    bad[0, 7] ^= 1
    assert not lrc.oracle_check(st, bad)
    # RS(12,4) decode of {0, 1}
    rs = _bare(bench.RS124, L=512)
    shards = [rng.integers(0, 256, 512, dtype=np.uint8) for _ in range(12)] + [np.zeros(512, np.uint8)] * 4
    shards = [s.copy() for s in shards]
    O.ReedSolomon(12, 4).encode_parity(shards, 0, 512)
    stripe = np.stack(shards)
    assert rs.oracle_check(stripe, stripe[0:2].copy())
    assert not rs.oracle_check(stripe, stripe[1:3].copy())
    # RS(17,3) encodeParity (the published benchmark's shape, shortened shards)
    r17 = _bare(bench.RS173, L=640)
    shards = [rng.integers(0, 256, 640, dtype=np.uint8) for _ in range(17)] + [np.zeros(640, np.uint8)] * 3
    shards = [s.copy() for s in shards]
    O.ReedSolomon(17, 3).encode_parity(shards, 0, 640)
    stripe = np.stack(shards)
    assert r17.oracle_check(stripe, stripe[17:20].copy())
    bad = stripe[17:20].copy()
    bad[2, 639] ^= 0x80
    assert not r17.oracle_check(stripe, bad)
    # LRC encode: parity p_g = d_3g ^ d_3g+1 ^ d_3g+2 in slots 3, 7, 11, 15
    le = _bare(bench.LRCEncode, b=256)
    st = rng.integers(0, 256, (16, 256), dtype=np.uint8)
    par = np.stack([st[4 * g] ^ st[4 * g + 1] ^ st[4 * g + 2] for g in range(4)])
    assert le.oracle_check(st, par)
    par[1, 0] ^= 4
    assert not le.oracle_check(st, par)


def test_published_metric_conversion():
    """rs173 reports the published benchmark's own unit (MB/s of input data bytes,
    ReedSolomonBenchmark.java:116-121) and vs_baseline against rs/README.md:53's 525.7."""
    wl = bench.RS173
    assert wl.metric_unit == "MB/s" and wl.metric_scale == 1e6 and wl.metric_bytes == 17 * 200000
    assert wl.unit_bytes == 20 * 200000 and bench.PUBLISHED == {"rs173": 525.7}
    assert bench.WORKLOADS["rs173"][0].startswith("MB/s RS(17,3) encodeParity")
    assert all(getattr(bench, c).metric_unit == "GiB/s" for c in ("Clay42", "Clay104", "RS124", "LRC"))


def test_round_scripts_cover_every_workload():
    """scripts/pmc.sh (the PMC traffic behind roofline.traffic) and scripts/gpu_round.sh
    (the per-workload bench lines) name every bench.py workload, and pmc.sh profiles each
    at the pool size bench.py uses by default, so no workload's line loses its traffic."""
    import re
    pmc = (ROOT / "scripts" / "pmc.sh").read_text()
    rnd = (ROOT / "scripts" / "gpu_round.sh").read_text()
    lists = [m.split() for m in re.findall(r'WORKLOADS="\$\{\*:-([^}]*)\}"', pmc)]
    default = max(lists, key=len)  # (the other list: --candidates, the layout-selected workloads)
    assert sorted(min(lists, key=len)) == ["lrcenc", "rs124", "rs173"]
    assert sorted(default) == sorted(bench.WORKLOADS)
    loop = re.search(r"for W in ([a-z0-9 ]+); do", rnd).group(1).split()
    assert sorted(loop + ["clay42"]) == sorted(bench.WORKLOADS)
    pools = {}
    for names, pool in re.findall(r"((?:[a-z0-9]+\|?)+)\) POOL=(\d+)", pmc):
        for w in names.split("|"):
            pools[w] = int(pool)
    assert pools == {w: v[1] for w, v in bench.WORKLOADS.items()}


def test_e2e_host_expect_in_place_and_separate():
    """The end-to-end leg's verification (Workload.host_expect): written-in-place workloads
    compare the whole host stripes with the device pool, the others the host outputs with the
    device outputs; one differing byte is caught either way (CPU tensors stand in for HBM)."""
    import numpy as np
    import torch
    pool = torch.randint(0, 256, (3, 20, 64), dtype=torch.uint8)
    r = _bare(bench.RS173, pool=pool, L=64)
    hin = pool.numpy().reshape(-1).copy()
    assert r.host_out_bytes() == 0 and r.host_stripe_bytes() == 20 * 64
    assert r.host_expect(hin, np.empty(0, np.uint8), 3)
    hin[2 * 20 * 64 + 17 * 64 + 5] ^= 1  # a parity byte of the last stripe
    assert not r.host_expect(hin, np.empty(0, np.uint8), 3)
    out = torch.randint(0, 256, (3, 8, 32), dtype=torch.uint8)
    c = _bare(bench.Clay42, pool=torch.zeros((3, 48, 32), dtype=torch.uint8), out=out)
    hout = out.numpy().reshape(-1).copy()
    assert c.host_expect(np.empty(0, np.uint8), hout, 3)
    hout[-1] ^= 0x80
    assert not c.host_expect(np.empty(0, np.uint8), hout, 3)
    assert c.pcie_bytes() == (20 * 32768, 8 * 32768)


def test_e2e_host_budget_shrinks_with_world():
    """The end-to-end leg's pinned host input per rank: E2E_HOST_BYTES for
    one rank, a share of E2E_NODE_BYTES when the ranks of a node run it at once, and within
    E2E_MEM_FRACTION of the free host memory in every case."""
    per = [bench.e2e_host_budget(w) for w in (1, 2, 4, 8)]
    assert per[0] == bench.E2E_HOST_BYTES
    assert all(a >= b for a, b in zip(per, per[1:])) and per[3] < per[2] < per[1]
    assert all(p * w <= max(bench.E2E_NODE_BYTES, bench.E2E_HOST_BYTES) for p, w in zip(per, (1, 2, 4, 8)))
    free = 16 << 30  # a tight lease: 16 GiB free -> 4 GiB for all ranks together
    capped = [bench.e2e_host_budget(w, free) for w in (1, 2, 4, 8)]
    assert all(c * w <= free * bench.E2E_MEM_FRACTION for c, w in zip(capped, (1, 2, 4, 8)))
    assert capped[3] == (4 << 30) // 8
    mem = bench.host_memory_free()  # this container: MemAvailable is readable
    assert mem["mem_available"] and mem["free"] and mem["free"] <= mem["mem_available"]


class _FakeHostBuffer:
    def __init__(self, nbytes):
        import numpy as np
        self.array = np.zeros(nbytes, np.uint8)


def test_e2e_leg_fills_in_chunks_within_the_budget(monkeypatch):
    """e2e_rate fills the pinned input from the pool in E2E_COPY_CHUNK steps (no full-size
    .cpu() of the pool), takes at most the per-rank budget, verifies, and reports the cap
    and the peak RSS (CPU tensors and a numpy HostBuffer stand in for HBM and pinned memory)."""
    import numpy as np
    import torch
    monkeypatch.setattr(bench, "E2E_COPY_CHUNK", 1000)  # several steps per stripe
    pool = torch.randint(0, 256, (40, 20, 64), dtype=torch.uint8)
    wl = _bare(bench.RS173, pool=pool, L=64, P=40)
    calls = []
    wl.host_call = lambda ha, ho, n: calls.append(n)  # in place, so the host copy is already "encoded"
    wl.host_plan = lambda n: None  # no map behind this stand-in
    full = pool.numel()

    class Ecx:
        HostBuffer = _FakeHostBuffer
    stripe = 20 * 64
    monkeypatch.setattr(bench, "E2E_HOST_BYTES", 25 * stripe)
    monkeypatch.setattr(bench, "E2E_NODE_BYTES", 50 * stripe)
    r1 = bench.e2e_rate(Ecx, torch, wl, 0.01, world=1)
    assert r1["verified"] and r1["stripes_per_call"] == 25 and r1["host_bytes"] == 25 * stripe < full
    assert r1["host_cap"]["budget_bytes_per_rank"] == 25 * stripe and r1["peak_rss_bytes"] > 0
    r8 = bench.e2e_rate(Ecx, torch, wl, 0.01, world=8)
    assert r8["verified"] and r8["stripes_per_call"] == 50 // 8 and r8["host_bytes"] < r1["host_bytes"]
    assert set(calls) == {25, 6}
    # a stripe larger than a rank's share at N > 1 is skipped, with the reason and the cap
    monkeypatch.setattr(bench, "E2E_NODE_BYTES", stripe)
    r = bench.e2e_rate(Ecx, torch, wl, 0.01, world=8)
    assert "skipped" in r and r["host_cap"]["world"] == 8


def test_copy_chunked_round_trip():
    import torch
    src = torch.randint(0, 256, (12345,), dtype=torch.uint8)
    dst = torch.zeros_like(src)
    bench._copy_chunked(dst, src, chunk=1000)
    assert torch.equal(dst, src)


def test_clay104_sub_bytes_reading(monkeypatch):
    """Config 4's other reading: --sub-bytes sets CLAY_BLOCK_SIZE for
    clay104 and scales the pool / stripes per step to the same bytes per step; its CPU
    baseline aliases read-only multi-GiB units instead of copying one per thread (a 64 KiB
    stand-in with a small arena cap here)."""
    monkeypatch.setattr(sys, "argv", ["bench.py", "--workload", "clay104", "--sub-bytes", "1048576"])
    a = bench.parse()
    assert a.sub_bytes == 1 << 20 and a.pool == 16 and a.stripes_per_step == 128
    monkeypatch.setattr(sys, "argv", ["bench.py", "--workload", "clay104"])
    a = bench.parse()
    assert a.pool == 2048 and a.stripes_per_step == 1 << 15
    monkeypatch.setattr(sys, "argv", ["bench.py", "--workload", "rs173", "--sub-bytes", "4096"])
    with pytest.raises(SystemExit):
        bench.parse()
    monkeypatch.setattr(bench, "CPU_ARENA_BYTES", 300 << 20)
    b = 65536
    wl = _bare(bench.Clay104, erased=3, n=14, unit_bytes=1088 * b, b=b)
    cpu = bench.cpu_baseline(wl, 0.2, None, max_units=2)
    assert cpu["value"] > 0 and "alias 1 distinct" in cpu["sample"] and "65536-B sub-chunks" in cpu["sample"]


def test_e2e_blocked_layout_host_batch_order(monkeypatch):
    """The blocked RS layout's end-to-end leg: the host input of n stripes is the
    full blocks of the first n pool stripes followed by their tails -- itself the blocked layout
    of those n stripes (blocked_pack of their natural shards) -- and the leg verifies region by
    region (CPU tensors and a numpy HostBuffer stand in for HBM and pinned memory)."""
    import torch
    import rpamd
    ecx = rpamd.load()
    monkeypatch.setattr(bench, "E2E_COPY_CHUNK", 777)
    S, n, L, b = 7, 20, 1000, 256  # 3 full blocks + a 232-B tail per shard
    nat = torch.randint(0, 256, (S, n, L), dtype=torch.uint8)
    wl = _bare(bench.RS173, pool=ecx.blocked_pack(nat, b), L=L, P=S, n=n, layout="blocked", block=b, ecx=ecx)
    k = 4
    src = torch.cat(wl.host_source(k))
    assert torch.equal(src, ecx.blocked_pack(nat[:k].contiguous(), b))
    assert wl.host_stripe_bytes() == n * L
    wl.host_call = lambda ha, ho, m: None  # the host map itself runs on the GPU box

    class Ecx:
        HostBuffer = _FakeHostBuffer
    monkeypatch.setattr(bench, "E2E_HOST_BYTES", k * n * L)
    r = bench.e2e_rate(Ecx, torch, wl, 0.01, world=1)
    assert r["verified"] and r["stripes_per_call"] == k


def test_e2e_leg_reports_the_host_plan():
    """The e2e leg's `plan` (ecx_map_host_plan, host-only) for the bench's own layouts: the headline
    keeps 64 MiB chunks with its runs of 5 planes in one 3D copy, Clay(10,4) node 3 takes 3 copies a
    chunk, the two-node repair one folded copy, RS(17,3) natural one merged run, and the blocked
    layouts (two passes) report none."""
    import rpamd
    ecx = rpamd.load()
    ecx.tune("host_chunk_kib", 65536)
    c42 = _bare(bench.Clay42, step=ecx.ClayCodeErasureDecodingStep([1], 4, 2), erased=1)
    p = c42.host_plan(2048)
    assert (p["chunk"], p["h2d_copies"], p["h2d_3d"], p["slices"]) == (102, 3, 1, 1)
    c2 = _bare(bench.Clay42x2, step=ecx.ClayCodeErasureDecodingStep([0, 3], 4, 2))
    assert (c2.host_plan(2048)["h2d_copies"], c2.host_plan(2048)["h2d_rows"]) == (1, 16)
    c104 = _bare(bench.Clay104, step=ecx.ClayCodeErasureDecodingStep([3], 10, 4, virtualUnits=2), n=14, alpha=256,
                 b=4096)
    assert (c104.host_plan(219)["h2d_copies"], c104.host_plan(219)["chunk"]) == (3, 19)
    big = _bare(bench.Clay104, step=c104.step, n=14, alpha=256, b=1 << 20)
    assert big.host_plan(1)["slices"] == 13
    rs = ecx.ReedSolomon.create(17, 3)
    r173 = _bare(bench.RS173, rs=rs, layout="natural", pitch=200000, L=200000)
    assert r173.host_plan(805)["h2d_copies"] == 1
    assert _bare(bench.RS173, rs=rs, layout="blocked", pitch=32768, L=200000).host_plan(805) is None
