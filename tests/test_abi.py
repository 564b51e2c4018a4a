"""The C-ABI library loads and exports every symbol include/ecx.h declares
(no compute calls: this container has no GPU)."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def declared_symbols(header="ecx.h"):
    text = (ROOT / "include" / header).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ecx_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for must in ["ecx_code_some_shards", "ecx_check_some_shards", "ecx_code_single", "ecx_rs_encode_parity",
                 "ecx_rs_decode_missing", "ecx_rs_decode_missing_single", "ecx_rs_encode_parity_single",
                 "ecx_rs_is_parity_correct", "ecx_clay_perform_coding", "ecx_clay_decode_single_helper",
                 "ecx_clay_perform_coding_batch", "ecx_map_apply_batch"]:
        assert must in syms


def test_library_exports_every_declared_symbol(ecx):
    """Every function declared by every header under include/ is exported."""
    lib = ctypes.CDLL(str(ecx.LIB_PATH))
    headers = sorted(p.name for p in (ROOT / "include").glob("*.h"))
    assert headers == ["ecx.h", "ecx_tune.h"]
    missing = [s for h in headers for s in declared_symbols(h) if not hasattr(lib, s)]
    assert not missing, missing
    assert len(declared_symbols("ecx_tune.h")) == 18


def test_binding_table_matches_header(ecx):
    from importlib import import_module
    sigs = import_module("repair_pipelining_amd._lib").SIGNATURES
    assert sorted(sigs) == declared_symbols()


def test_no_gpu_fails_loudly(ecx):
    """Without a HIP device the arithmetic entry points raise (no CPU fallback)."""
    import numpy as np
    if ecx.device_count() if _has_device(ecx) else 0:
        pytest.skip("a device is present")
    rs = ecx.ReedSolomon.create(4, 2)
    with pytest.raises(ecx.EcxError) as e:
        rs.encodeParity([np.zeros(16, np.uint8) for _ in range(6)], 0, 16)
    assert e.value.code == -10
    # the host-memory batch path has no CPU fallback either
    step = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
    host_in, host_out = np.zeros((2, 48, 64), np.uint8), np.zeros((2, 8, 64), np.uint8)
    with pytest.raises(ecx.EcxError) as e:
        step.performCodingBatchHost(host_in, 48 * 64, 64, host_out, 8 * 64, 64, 2, 64)
    assert e.value.code == -10
    with pytest.raises(ecx.EcxError) as e:
        ecx.HostBuffer(4096)
    assert e.value.code == -10


def _has_device(ecx):
    try:
        return ecx.device_count() > 0
    except ecx.EcxError:
        return False


def test_status_strings(ecx):
    lib = ecx.lib()
    assert lib.ecx_status_string(-3) == b"Matrix is singular"
    assert lib.ecx_version() >= 100


def test_host_planner_errors(ecx):
    """Exceptions of the reference map to status codes before any device work."""
    with pytest.raises(ecx.EcxError) as e:
        ecx.ReedSolomon.create(200, 57)
    assert e.value.code == -4
    with pytest.raises(ecx.EcxError) as e:
        ecx.Matrix.invert([[1, 1], [1, 1]])
    assert e.value.code == -3
    with pytest.raises(ecx.EcxError) as e:
        ecx.Galois.divide(3, 0)
    assert e.value.code == -1
    rs = ecx.ReedSolomon.create(4, 2)
    with pytest.raises(ecx.EcxError) as e:
        rs.decode_map([True, False, False, False, True, True])
    assert e.value.code == -2
    # Clay(10,4): t = 14 // 4 = 3 -> nodes 12, 13 are off the grid (bug B7)
    step = ecx.ClayCodeErasureDecodingStep([13], 10, 4)
    with pytest.raises(ecx.EcxError) as e:
        step.getHelperPlanesIndexes(13)
    assert e.value.code == -5


def test_roctx_ranges_keep_results_and_status(ecx):
    """ecx_tune("roctx", 1) wraps every C-ABI call in a roctx range named after the entry
    point: host results and exception status codes are unchanged, with or without the
    marker library and with no profiler attached."""
    ecx.tune("roctx", 1)
    try:
        rs = ecx.ReedSolomon.create(4, 2)
        m = rs.decode_map([False, True, True, True, True, False])
        assert m.info()["n_out"] == 2  # data shard 0 and parity shard 5
        with pytest.raises(ecx.EcxError) as e:
            ecx.Matrix.invert([[1, 1], [1, 1]])
        assert e.value.code == -3
        with pytest.raises(ecx.EcxError) as e:
            rs.decode_map([True, False, False, False, True, True])
        assert e.value.code == -2
    finally:
        ecx.tune("roctx", 0)


def test_batch_layout_checked_before_any_device_work(ecx):
    """A batch layout that addresses past the end of its buffer fails loudly
    (ArrayIndexOutOfBoundsException) instead of reaching a kernel."""
    import numpy as np
    import torch
    step = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
    B, S = 512, 3
    inp, out = np.zeros((S, 48, B), np.uint8), np.zeros((S, 8, B), np.uint8)
    with pytest.raises(ecx.EcxError) as e:
        step.performCodingBatchHost(inp, 48 * B, B, out, 8 * B, B, S + 1, B)  # one stripe too many
    assert e.value.code == -5
    with pytest.raises(ecx.EcxError) as e:
        step.performCodingBatchHost(inp[1:], 48 * B, B, out, 8 * B, B, S, B)  # view: less room left
    assert e.value.code == -5
    with pytest.raises(ecx.EcxError) as e:
        step.performCodingBatchHost(inp, 48 * B, B, out, 8 * B, 2 * B, S, B)  # output slot stride too wide
    assert e.value.code == -5
    t_in = torch.zeros((S, 48, B), dtype=torch.uint8)
    mat, ins, outs = step.map().matrix()
    gm = ecx.GfMap.from_matrix(mat, in_slot=ins, out_slot=outs)
    assert gm.max_slots() == (int(ins.max()), int(outs.max()))
    with pytest.raises(ecx.EcxError) as e:
        gm.apply_batch_host(t_in[:, :40], 48 * B, B, out, 8 * B, B, S, B + 1)
    assert e.value.code == -5
    if not _has_device(ecx):  # a valid layout gets as far as the (absent) device
        with pytest.raises(ecx.EcxError) as e:
            gm.apply_batch_host(t_in, 48 * B, B, out, 8 * B, B, S, B)
        assert e.value.code == -10


def test_tuning_keys(ecx):
    """ecx_tune (include/ecx_tune.h) accepts every documented knob with its valid
    values, rejects unknown keys and out-of-range values, and is host-only."""
    lib = ecx.lib()
    tune = lib.ecx_tune
    tune.argtypes, tune.restype = [ctypes.c_char_p, ctypes.c_int], ctypes.c_int
    header = (ROOT / "include" / "ecx_tune.h").read_text()
    documented = re.findall(r'^ \*\s+"([a-z_]+)"', header, flags=re.M)
    lab = re.findall(r'^ \*\s+\[DIAG\] "([a-z_]+)"', header, flags=re.M)
    assert sorted(lab) == sorted(["wave_groups", "occ_lds", "bitslice", "lds_lut", "rtc_diag", "rtc_units", "rtc_persist",
                                  "units"])
    for key in lab:  # the product library refuses them; the diagnostic one takes its defaults
        assert tune(key.encode(), 1 if key in ("rtc_units", "units") else 0) == (0 if ecx.is_diag() else -1), key
    defaults = {"depth": 0, "nontemporal": 1, "xcd_group": 0, "lds_tables": 1, "store_scope": 0,
                "chunk_major": 0, "stagger": 0, "block_threads": 0, "small_tiles": 2, "host_zero_copy": 1, "wide_tiles": 1, "skew_chunks": 1, "layout_select": 1, "plan_cache": 256, "roctx": 0, "host_contexts": 1, "clay_rtc": 1, "rtc_lookahead": 1, "rtc_waves": 3, "rtc_xcd": 2, "rtc_group": 1, "rtc_sched": 2, "rtc_nt": 5, "rtc_wide": 0, "xcd_run": 8, "xcd_misaligned": 1,
                "map_planes": 1, "planes_lookahead": 12, "planes_waves": 2,
                "host_chunk_kib": 65536, "host_buffers": 3, "host_gather_kib": 512, "host_exec_kib": 1024}
    assert sorted(documented) == sorted(defaults)
    integration = (ROOT / "INTEGRATION.md").read_text()
    assert all("`%s`" % k in integration for k in documented), "INTEGRATION.md must list every tuning key"
    for key, val in defaults.items():
        assert tune(key.encode(), val) == 0, key
    assert tune(b"no_such_knob", 1) == -1
    for key, bad in (("depth", 3), ("depth", 6), ("nontemporal", 3), ("xcd_group", -1), ("xcd_group", 4), ("xcd_run", 0), ("xcd_misaligned", 2), ("stagger", -1), ("stagger", 65), ("lds_tables", 3), ("host_buffers", 9), ("block_threads", 128), ("small_tiles", 3), ("wave_groups", 3), ("wide_tiles", 3), ("skew_chunks", 3), ("layout_select", 2), ("plan_cache", -1), ("bitslice", 3), ("lds_lut", 3), ("lds_lut", -1), ("roctx", 2), ("host_contexts", 2), ("clay_rtc", 3), ("rtc_lookahead", 32), ("rtc_waves", 1), ("rtc_persist", 9), ("rtc_units", 0), ("rtc_units", 3), ("rtc_sched", 3), ("rtc_nt", -1), ("rtc_nt", 16), ("rtc_wide", 2), ("occ_lds", -2), ("occ_lds", 65537), ("rtc_diag", 1), ("rtc_diag", 32), ("map_planes", 3), ("planes_lookahead", 16), ("planes_waves", 0), ("planes_waves", 5), ("host_exec_kib", -1)):
        assert tune(key.encode(), bad) == -1, key
    for key, val in defaults.items():  # restore
        tune(key.encode(), val)


def test_last_kernel_label_before_any_launch(ecx):
    """ecx_last_kernel (include/ecx_tune.h): empty before any launch on this thread,
    and a too-short buffer is refused rather than truncated."""
    import ctypes as C
    f = ecx.lib().ecx_last_kernel
    f.argtypes, f.restype = [C.c_char_p, C.c_int], C.c_int
    assert f(C.create_string_buffer(8), 8) == 0
    assert f(None, 0) == -1


def test_codec_registry_refcounts_and_bounds_idle(ecx):
    """ecx_rs_create / ecx_clay_create share one reference-counted codec per key (ecx.h):
    creates of an equal codec return the same object, destroy drops one reference, the
    last one parks the codec in a bounded idle cache (a later create revives it with its
    plans), and past 64 idle codecs the least recently released are freed -- so a caller
    cycling through many distinct codecs (one Clay decoding step per erasure pattern) does
    not grow the process without bound.  Host-only: codec creation needs no device."""
    lib = ecx.lib()
    stats = lib.ecx_codec_stats
    stats.argtypes, stats.restype = [ctypes.POINTER(ctypes.c_int)] * 4, ctypes.c_int
    create, destroy = lib.ecx_rs_create, lib.ecx_rs_destroy

    def counts():
        v = [ctypes.c_int() for _ in range(4)]
        assert stats(*[ctypes.byref(x) for x in v]) == 0
        return [x.value for x in v]

    def rs(k, m):
        h = ctypes.c_void_p()
        assert create(k, m, ctypes.byref(h)) == 0
        return h.value

    live0, idle0, _, _ = counts()
    a, b = rs(29, 3), rs(29, 3)
    assert a == b and counts()[0] == live0 + 1
    destroy(a)
    assert counts()[:2] == [live0 + 1, idle0]        # one reference left
    destroy(b)
    parked = min(idle0 + 1, 64)  # (an idle cache already full evicts its oldest entry instead)
    assert counts()[:2] == [live0, parked]           # parked idle, not freed
    destroy(b)                                        # a second destroy holds no reference: ignored
    assert counts()[:2] == [live0, parked]
    assert rs(29, 3) == a and counts()[:2] == [live0 + 1, parked - 1]  # revived: same object
    destroy(a)
    # many distinct codecs created and released: the idle cache stays bounded
    for k in range(100):
        destroy(rs(30 + k, 2))
    live, idle, _, _ = counts()
    assert live == live0 and idle == 64
    # Clay steps: the same rules per (k, m, virtual nodes, erased list)
    er = (ctypes.c_int * 1)(3)
    h1, h2 = ctypes.c_void_p(), ctypes.c_void_p()
    assert lib.ecx_clay_create(4, 2, er, 1, ctypes.byref(h1)) == 0
    assert lib.ecx_clay_create(4, 2, er, 1, ctypes.byref(h2)) == 0
    assert h1.value == h2.value
    cl_live = counts()[2]
    lib.ecx_clay_destroy(h1)
    lib.ecx_clay_destroy(h2)
    assert counts()[2] == cl_live - 1


def test_host_batch_devices_argument_checks(ecx):
    """The multi-GPU host batches refuse an empty or null device list before touching a
    device (ECX_E_ILLEGAL_ARGUMENT / ECX_E_NULL); without a device, a valid list reaches the
    device query and fails loudly (ECX_E_DEVICE), never a CPU path."""
    import numpy as np
    if _has_device(ecx):
        pytest.skip("a device is present (the GPU tests cover the calls)")
    lib = ecx.lib()
    step = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
    hin, hout = np.zeros((2, 48, 64), np.uint8), np.zeros((2, 8, 64), np.uint8)
    args = (step._h, hin.ctypes.data, 48 * 64, 64, hout.ctypes.data, 8 * 64, 64, 2, 64)
    assert lib.ecx_clay_perform_coding_batch_host_devices(*args, None, 1) == -6
    devs = (ctypes.c_int * 2)(0, 0)
    assert lib.ecx_clay_perform_coding_batch_host_devices(*args, devs, 0) == -1
    assert lib.ecx_clay_perform_coding_batch_host_devices(*args, devs, -3) == -1
    assert lib.ecx_clay_perform_coding_batch_host_devices(*args, devs, 2) == -10
    m = step.map()
    margs = (m._h, hin.ctypes.data, 48 * 64, 64, hout.ctypes.data, 8 * 64, 64, 2, 64)
    assert lib.ecx_map_apply_batch_host_devices(*margs, None, 1) == -6
    assert lib.ecx_map_apply_batch_host_devices(*margs, devs, 0) == -1
    assert lib.ecx_map_apply_batch_host_devices(*margs, devs, 2) == -10
    assert (hout == 0).all()


def test_is_parity_correct_batch_argument_checks(ecx):
    """ecx_rs_is_parity_correct_batch: negative counts are IllegalArgumentException, a null
    codec or pointer NullPointerException; an empty batch is a no-op; no CPU path."""
    lib = ecx.lib()
    rs = ecx.ReedSolomon.create(17, 3)
    assert lib.ecx_rs_is_parity_correct_batch(rs._h, 16, 20 * 64, 64, -1, 0, 64, 16, None) == -1
    assert lib.ecx_rs_is_parity_correct_batch(rs._h, 16, 20 * 64, 64, 1, -1, 64, 16, None) == -1
    assert lib.ecx_rs_is_parity_correct_batch(rs._h, 16, 20 * 64, 64, 1, 0, -64, 16, None) == -1
    assert lib.ecx_rs_is_parity_correct_batch(None, 16, 20 * 64, 64, 1, 0, 64, 16, None) == -6
    assert lib.ecx_rs_is_parity_correct_batch(rs._h, None, 20 * 64, 64, 1, 0, 64, 16, None) == -6
    assert lib.ecx_rs_is_parity_correct_batch(rs._h, 16, 20 * 64, 64, 1, 0, 64, None, None) == -6
    assert lib.ecx_rs_is_parity_correct_batch(rs._h, None, 20 * 64, 64, 0, 0, 64, None, None) == 0
    if not _has_device(ecx):
        assert lib.ecx_rs_is_parity_correct_batch(rs._h, 16, 20 * 64, 64, 1, 0, 64, 16, None) == -10


def test_host_check_batch_argument_checks(ecx):
    """ecx_rs_is_parity_correct_batch_host(_devices): negative counts or strides are
    IllegalArgumentException, a null codec, stripe or verdict pointer NullPointerException, an
    empty or null device list is refused before any device is touched; an empty batch is a
    no-op; with bytes to check and no device the call fails loudly (ECX_E_DEVICE) -- no CPU path."""
    import numpy as np
    lib = ecx.lib()
    rs = ecx.ReedSolomon.create(17, 3)
    shards, verdict = np.zeros((2, 20, 64), np.uint8), np.full(2, 7, np.uint8)
    base, v = shards.ctypes.data, verdict.ctypes.data
    f = lib.ecx_rs_is_parity_correct_batch_host
    assert f(rs._h, base, 20 * 64, 64, -1, 0, 64, v) == -1
    assert f(rs._h, base, 20 * 64, 64, 2, -1, 64, v) == -1
    assert f(rs._h, base, 20 * 64, 64, 2, 0, -64, v) == -1
    assert f(rs._h, base, -1, 64, 2, 0, 64, v) == -1
    assert f(None, base, 20 * 64, 64, 2, 0, 64, v) == -6
    assert f(rs._h, None, 20 * 64, 64, 2, 0, 64, v) == -6
    assert f(rs._h, base, 20 * 64, 64, 2, 0, 64, None) == -6
    assert f(rs._h, None, 20 * 64, 64, 0, 0, 64, None) == 0
    g = lib.ecx_rs_is_parity_correct_batch_host_devices
    devs = (ctypes.c_int * 2)(0, 0)
    assert g(rs._h, base, 20 * 64, 64, 2, 0, 64, v, None, 1) == -6
    assert g(rs._h, base, 20 * 64, 64, 2, 0, 64, v, devs, 0) == -1
    assert g(rs._h, base, 20 * 64, 64, -2, 0, 64, v, devs, 2) == -1
    if not _has_device(ecx):
        assert f(rs._h, base, 20 * 64, 64, 2, 0, 64, v) == -10
        assert g(rs._h, base, 20 * 64, 64, 2, 0, 64, v, devs, 2) == -10
        assert (verdict == 7).all()  # nothing was decided on the host


def test_shape_knobs_need_the_opt_in():
    """Round-4 verdict item 7: in a process without ECX_SHAPE_KNOBS=1 the product library
    accepts only the deployment keys (layout_select, plan_cache, roctx, host_*) and refuses
    every launch-shape key; with the opt-in it accepts them (a fresh process each way: the
    library reads the variable once)."""
    import os
    import subprocess
    import sys
    code = r'''
import sys, ctypes
sys.path.insert(0, %r)
import rpamd
lib = rpamd.load().lib()
f = lib.ecx_tune
f.argtypes, f.restype = [ctypes.c_char_p, ctypes.c_int], ctypes.c_int
out = {}
for k, v in [("layout_select", 1), ("plan_cache", 256), ("roctx", 0), ("host_chunk_kib", 65536),
             ("host_buffers", 3), ("host_gather_kib", 512), ("host_zero_copy", 1), ("host_contexts", 1),
             ("host_exec_kib", 1024),
             ("depth", 0), ("nontemporal", 1), ("xcd_group", 0), ("stagger", 0), ("block_threads", 0),
             ("skew_chunks", 1), ("wide_tiles", 1), ("lds_tables", 1), ("store_scope", 0), ("rtc_nt", 5),
             ("clay_rtc", 1), ("map_planes", 1), ("small_tiles", 2), ("chunk_major", 0)]:
    out[k] = f(k.encode(), v)
print(out)
''' % str(ROOT)
    env = {k: v for k, v in os.environ.items() if k != "ECX_SHAPE_KNOBS"}
    deploy = {"layout_select", "plan_cache", "roctx", "host_chunk_kib", "host_buffers", "host_gather_kib",
              "host_zero_copy", "host_contexts", "host_exec_kib"}
    for opt_in in (False, True):
        e = dict(env, ECX_SHAPE_KNOBS="1") if opt_in else env
        r = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        got = eval(r.stdout.strip().splitlines()[-1])
        for k, st in got.items():
            assert st == (0 if (k in deploy or opt_in) else -1), (opt_in, k, st)


def test_multi_gpu_host_batch_split_matches_shard_stripes(ecx):
    """The multi-GPU host batches split a batch exactly as shard_stripes partitions stripes
    across ranks (ecx_stripe_range, the split run_host_batch_devices uses): contiguous, covering,
    the remainder on the first entries; bad requests are refused."""
    f = ecx.lib().ecx_stripe_range
    f.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int64),
                  ctypes.POINTER(ctypes.c_int64)]
    f.restype = ctypes.c_int
    b, e = ctypes.c_int64(), ctypes.c_int64()
    for n in (0, 1, 5, 7, 8, 1023, 1 << 20, (1 << 33) + 3):
        for parts in (1, 2, 3, 7, 8, 13):
            prev = 0
            for j in range(parts):
                assert f(n, parts, j, ctypes.byref(b), ctypes.byref(e)) == 0
                assert (b.value, e.value) == ecx.shard_stripes(n, parts, j)
                assert b.value == prev
                prev = e.value
            assert prev == n
    for bad in ((-1, 2, 0), (5, 0, 0), (5, 2, 2), (5, 2, -1)):
        assert f(*bad, ctypes.byref(b), ctypes.byref(e)) == -1


def test_rs_blocked_layout_contract(ecx):
    """The RS layout contract (ecx_rs_blocked_layout / ecx_rs_recommended_pitch):
    64 KiB blocks (one block below that), the full / tail split, the plain layout's pitch; and
    blocked_pack / blocked_unpack, the torch helpers that lay a [stripes][n][L] batch out that
    way, are exact inverses over exactly stripes * n * L bytes (CPU tensors here)."""
    import torch
    r173, r124 = ecx.ReedSolomon.create(17, 3), ecx.ReedSolomon.create(12, 4)
    assert r173.blockedLayout(200000) == (32768, 6, 200000 - 6 * 32768)
    assert r124.blockedLayout(4 << 20) == (65536, 64, 0)
    assert ecx.ReedSolomon.create(4, 2).blockedLayout(32768) == (32768, 1, 0)  # 6 shards: 128 KiB blocks
    assert r173.blockedLayout(34) == (34, 1, 0) and r173.blockedLayout(0) == (0, 0, 0)
    assert ecx.ReedSolomon.create(128, 128).blockedLayout(1 << 20)[0] == 4096  # never below 4 KiB
    for L in (200000, 4 << 20, 104449, 34816, 1, 4096):
        p = r173.recommendedPitch(L)
        assert p >= L and p % 4096 == 0 and (p // 4096) % 2 == 1 and p - L < 8192, (L, p)
    assert r124.recommendedPitch(4 << 20) == (4 << 20) + 4096 and r173.recommendedPitch(200000) == 200704
    with pytest.raises(ecx.EcxError):
        r173.blockedLayout(-1)
    g = torch.Generator().manual_seed(3)
    for S, n, L, b in ((3, 20, 200000, 65536), (2, 16, 3 * 4096, 4096), (2, 5, 1001, 64), (1, 4, 64, 64)):
        x = torch.randint(0, 256, (S, n, L), dtype=torch.uint8, generator=g)
        flat = ecx.blocked_pack(x, b)
        assert flat.numel() == S * n * L
        full, tail = divmod(L, b)
        if full:  # stripe 0, block 1 (or 0), shard 2 sits where the layout says
            t = min(1, full - 1)
            at = (t * n + 2) * b
            assert torch.equal(flat[at:at + b], x[0, 2, t * b:(t + 1) * b])
        assert torch.equal(ecx.blocked_unpack(flat, S, n, L, b), x)
