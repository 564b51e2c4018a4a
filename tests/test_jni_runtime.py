"""The JNI binding EXECUTED: the generated forwarders of jni/ecx_jni.c, compiled with a
fake JNIEnv over C memory (tests/native/jni_fake_env.c; no JDK in this image) and linked
to libecx.so, are called the way EcxNative's natives would be.

CPU: every argument check the forwarders run before pinning returns the status of the
exception the reference throws (ReedSolomon.checkBuffersAndSizes, ReedSolomon.java:338-363;
"Invalid inputs/outputs length", ClayCodeErasureDecodingStep.java:76-82;
ArrayIndexOutOfBoundsException of the CodingLoop byte loop, InputOutputByteTableCodingLoop
.java:34-41) without reaching the export, null Clay sub-chunks pass, the planner entry
points return the reference's values through the binding, and every pin is released
with no JNI call made inside a critical region.
The host batches over direct ByteBuffers (clayPerformCodingBatchHostBuffer,
mapApplyBatchHostBuffer): a buffer shorter than the batch's extent, a heap buffer or a
null one is refused before anything is pinned or read.
GPU: codeSomeShards (RS(4,2) parity rows), the RS codec calls, decodeMissingSingle,
clayPerformCoding (Clay(4,2), e = 1) and the two ByteBuffer host batches through the
binding equal the oracle, with array positions (ByteBuffer.arrayOffset + position) applied."""
import re

import numpy as np
import pytest

import oracle as O
from jni_harness import Jni

OK, ILL, NSH, IDX, NUL, DEV = 0, -1, -2, -5, -6, -10


@pytest.fixture(scope="module")
def jni():
    j = Jni()
    yield j
    j.free_all()


@pytest.fixture
def J(jni):
    jni.reset()
    yield jni
    c = jni.counters()
    assert c["pins_now"] == 0 and c["pins"] == c["unpins"], c
    assert c["violations"] == 0 and c["calls_while_pinned"] == 0, c


def has_device(J):
    n = np.zeros(1, np.int32)
    return J.call("deviceCount", J.array(n)) == OK and n[0] > 0


def handle(J, fn, *args):
    h = np.zeros(1, np.int64)
    assert J.call(fn, *args, J.array(h)) == OK
    assert h[0] != 0
    return int(h[0])


def rnd(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


# ---------------------------------------------------------------- CPU: argument checks
def test_code_some_shards_argument_checks(J):
    rows = np.ones(2 * 4, np.uint8)
    ins = [rnd(64, i) for i in range(4)]
    outs = [np.zeros(64, np.uint8) for _ in range(2)]
    call = lambda rows_, ins_, outs_, nin=4, nout=2, off=0, bc=64, ipos=None, opos=None: J.call(  # noqa: E731
        "codeSomeShards", J.array(rows_), J.array2d(ins_), J.ints(ipos) if ipos is not None else None, nin,
        J.array2d(outs_), J.ints(opos) if opos is not None else None, nout, off, bc)
    assert call(rows[:7], ins, outs) == IDX                       # matrixRows too short
    assert call(rows, ins[:3], outs) == IDX                       # fewer inputs than inputCount
    assert call(rows, ins[:3] + [rnd(63, 9)], outs) == IDX        # an input shorter than offset + byteCount
    assert call(rows, ins, outs[:1] + [np.zeros(10, np.uint8)]) == IDX  # a short output
    assert call(rows, ins, outs, off=8, bc=57) == IDX             # offset + byteCount past the shards
    assert call(rows, ins, outs, ipos=[0, 0, 1, 0]) == IDX       # position + byteCount past a shard
    assert call(rows, ins, outs, ipos=[0, -1, 0, 0]) == IDX      # negative position
    assert call(rows, ins, outs, ipos=[0, 0]) == ILL             # positions shorter than the list
    assert call(rows, ins[:2] + [None] + ins[3:], outs) == NUL    # null input shard
    assert call(rows, ins, outs, off=-1) == ILL
    assert call(rows, ins, outs, bc=-1) == ILL
    assert call(None, ins, outs) == NUL
    assert J.counters()["pins"] == 0  # nothing above was pinned: rejected before the export
    assert all((o == 0).all() for o in outs)


def test_rs_codec_argument_checks(J):
    rs = handle(J, "rsCreate", 4, 2)
    try:
        shards = [rnd(100, i) for i in range(6)]
        enc = lambda sh, count=6, length=100, off=0, bc=100, pos=None: J.call(  # noqa: E731
            "rsEncodeParity", rs, J.array2d(sh), J.ints(pos) if pos is not None else None, count, length, off, bc)
        assert enc(shards[:5]) == ILL                             # wrong number of shards (:341-343)
        assert enc(shards[:5] + [rnd(99, 7)]) == ILL              # shards of different sizes (:346-351)
        assert enc(shards, pos=[0, 0, 0, 0, 0, 1]) == ILL         # position leaves fewer than shardLength bytes
        assert enc(shards[:5] + [None]) == NUL
        assert enc(shards, off=-1) == ILL and enc(shards, bc=-1) == ILL
        present = np.ones(6, np.uint8)
        assert J.call("rsDecodeMissing", rs, J.array2d(shards), None, J.array(present[:5]), 6, 100, 0, 100) == IDX
        assert J.call("rsIsParityCorrect", rs, J.array2d(shards), None, 6, 100, 0, 100, J.array(rnd(50, 1)), 100) == ILL
        # encodeParitySingle (EcxPartialSums): outputs the caller supplies are checked too
        assert J.call("rsEncodeParitySingle", rs, J.array(rnd(100, 1)), J.array(np.zeros(99, np.uint8)), 0, 0, 0,
                      100) == IDX
        assert J.call("rsEncodeParitySingle", rs, J.array(rnd(10, 1)), J.array(np.zeros(100, np.uint8)), 0, 0, 0,
                      100) == IDX
        pres = np.array([0, 1, 1, 1, 1, 1], np.uint8)
        outs = [np.zeros(100, np.uint8)]
        assert J.call("rsDecodeMissingSingle", rs, J.array(rnd(100, 2)), 1, 0, J.array(pres[:4]), J.array2d(outs),
                      None, 1, 0, 100, 1) == IDX
        assert J.call("rsDecodeMissingSingle", rs, J.array(rnd(100, 2)), 1, 0, J.array(pres),
                      J.array2d([np.zeros(50, np.uint8)]), None, 1, 0, 100, 1) == IDX
        assert J.call("rsMatrix", rs, J.array(np.zeros(6 * 4 - 1, np.uint8))) == IDX
        assert J.call("rsEncodeParity", 0, J.array2d(shards), None, 6, 100, 0, 100) == NUL  # handle 0
        assert J.counters()["pins"] == 0
    finally:
        J.call("rsDestroy", rs)


def test_clay_perform_coding_argument_checks(J):
    clay = handle(J, "clayCreate", 4, 2, J.ints([1]), 1)
    J.reset()
    try:
        n, a, B = 6, 8, 64
        ins = [None if i % n == 1 else rnd(B, i) for i in range(n * a)]
        outs = [np.zeros(B, np.uint8) for _ in range(a)]
        pc = lambda i, o, bs=B, ipos=None: J.call("clayPerformCoding", clay, J.array2d(i),  # noqa: E731
                                                 J.ints(ipos) if ipos is not None else None, J.array2d(o), None, bs)
        assert pc(ins[:-1], outs) == ILL                  # Invalid inputs length (:76-78)
        assert pc(ins + [rnd(B, 0)], outs) == ILL         # ... not fewer, not more
        assert pc(ins, outs[:-1]) == ILL                  # Invalid outputs length (:80-82)
        assert pc(ins, outs[:-1] + [np.zeros(B - 1, np.uint8)]) == IDX
        assert pc(ins, outs[:-1] + [None]) == NUL
        short = list(ins)
        short[2] = rnd(B - 1, 3)
        assert pc(short, outs) == IDX                     # a helper sub-chunk shorter than bufSize
        assert pc(ins, outs, ipos=[0] * (n * a - 1) + [1]) == IDX
        assert pc(ins, outs, bs=-1) == ILL
        assert J.counters()["pins"] == 0
        # null inputs (absent sub-chunks) pass the checks and reach the device
        st = pc(ins, outs)
        assert st == (OK if has_device(J) else DEV), st
        hp = np.zeros(1, np.int32)
        assert J.call("clayHelperPlanes", clay, 1, J.array(hp)) == IDX  # needs alpha/q = 4 entries
    finally:
        J.call("clayDestroy", clay)


def test_clay_nothing_erased_returns_before_length_checks(J):
    """performCoding with no erased index returns at once (:54-56), even for arrays of
    the wrong length."""
    clay = handle(J, "clayCreate", 4, 2, J.ints([]), 0)
    try:
        assert J.call("clayPerformCoding", clay, J.array2d([rnd(8, 1)]), None, J.array2d([]), None, 8) == OK
    finally:
        J.call("clayDestroy", clay)


def test_handles_and_out_arrays(J):
    assert J.call("rsCreate", 4, 2, J.array(np.zeros(0, np.int64))) == IDX  # long[0] for the handle
    assert J.call("rsCreate", 4, 2, None) == NUL
    assert J.call("mapInfo", 0, None, None, None) == NUL
    assert J.call("clayGeometry", 0, None, None, None) == NUL
    assert J.call("matrixTimes", J.array(np.ones(6, np.uint8)), -2, -3, J.array(np.ones(6, np.uint8)), 3, 2,
                  J.array(np.zeros(4, np.uint8))) == ILL
    assert J.call("matrixInvert", J.array(np.ones(8, np.uint8)), 3, J.array(np.zeros(9, np.uint8))) == IDX


# ---------------------------------------------------------------- CPU: planner through the binding
def test_planner_calls_through_binding(J, kats):
    assert J.call("gfMultiply", 3, 7) == O.gf_multiply(3, 7)
    t = kats["matrix"]["times"]
    a, b = np.array(t["a"], np.uint8), np.array(t["b"], np.uint8)
    out = np.zeros((a.shape[0], b.shape[1]), np.uint8)
    assert J.call("matrixTimes", J.array(a), a.shape[0], a.shape[1], J.array(b), b.shape[0], b.shape[1],
                  J.array(out)) == OK
    assert out.tolist() == t["out"]
    case = kats["matrix"]["invert"][0]
    m = np.array(case["m"], np.uint8)
    inv = np.zeros_like(m)
    assert J.call("matrixInvert", J.array(m), m.shape[0], J.array(inv)) == OK
    assert inv.tolist() == case["inv"]
    log, exp, mul = np.zeros(256, np.int16), np.zeros(510, np.uint8), np.zeros(65536, np.uint8)
    assert J.call("gfTables", J.array(log), J.array(exp), J.array(mul)) == OK
    assert log.tolist() == kats["galois"]["log_table"] and (mul.reshape(256, 256) == O.mul_table()).all()
    assert J.string(J.call("statusString", -5)).startswith("ArrayIndexOutOfBounds") or J.string(
        J.call("statusString", -5))

    rs = handle(J, "rsCreate", 17, 3)
    try:
        k, m_ = np.zeros(1, np.int32), np.zeros(1, np.int32)
        assert J.call("rsShape", rs, J.array(k), J.array(m_)) == OK and (k[0], m_[0]) == (17, 3)
        mat = np.zeros((20, 17), np.uint8)
        assert J.call("rsMatrix", rs, J.array(mat)) == OK
        assert (mat == O.ReedSolomon(17, 3).matrix).all()
    finally:
        J.call("rsDestroy", rs)

    clay = handle(J, "clayCreateShortened", 10, 4, 2, J.ints([3]), 1)
    try:
        q, t_, al = (np.zeros(1, np.int32) for _ in range(3))
        assert J.call("clayGeometry", clay, J.array(q), J.array(t_), J.array(al)) == OK
        assert (q[0], t_[0], al[0]) == (4, 4, 256)
        nodes, ne = np.zeros(1, np.int32), np.zeros(1, np.int32)
        assert J.call("clayShape", clay, J.array(nodes), J.array(ne), J.array(al)) == OK
        assert (nodes[0], ne[0], al[0]) == (14, 1, 256)
        hp = np.zeros(64, np.int32)
        assert J.call("clayHelperPlanes", clay, 3, J.array(hp)) == 64
    finally:
        J.call("clayDestroy", clay)

    mat = np.arange(1, 13, dtype=np.uint8).reshape(3, 4)
    mp = handle(J, "mapCreate", J.array(mat), 3, 4, J.ints([0, 2, 4, 6]), J.ints([1, 3, 5]))
    try:
        no, ni, nnz = (np.zeros(1, np.int32) for _ in range(3))
        assert J.call("mapInfo", mp, J.array(no), J.array(ni), J.array(nnz)) == OK
        assert (no[0], ni[0], nnz[0]) == (3, 4, 12)
        got, ins, outs = np.zeros((3, 4), np.uint8), np.zeros(4, np.int32), np.zeros(3, np.int32)
        assert J.call("mapMatrix", mp, J.array(got[:2]), J.array(ins), J.array(outs)) == IDX
        assert J.call("mapMatrix", mp, J.array(got), J.array(ins), J.array(outs)) == OK
        assert (got == mat).all() and ins.tolist() == [0, 2, 4, 6] and outs.tolist() == [1, 3, 5]
    finally:
        J.call("mapDestroy", mp)


def test_valid_per_call_reaches_the_export(J):
    """Well-formed arguments pass every check and reach the device (ECX_E_DEVICE without
    one: there is no CPU fallback), with every pin released and the outputs released
    with mode 0 (copy back) and the read-only inputs with JNI_ABORT."""
    rows = O.ReedSolomon(4, 2).parity_rows.astype(np.uint8).copy()
    ins = [rnd(64, i) for i in range(4)]
    outs = [np.zeros(64, np.uint8) for _ in range(2)]
    st = J.call("codeSomeShards", J.array(rows), J.array2d(ins), None, 4, J.array2d(outs), None, 2, 0, 64)
    c = J.counters()
    assert st == (OK if has_device(J) else DEV), st
    assert c["pins"] == 1 + 4 + 2 and c["last_mode"] == 2  # matrixRows released last, JNI_ABORT


# ---------------------------------------------------------------- host batches over direct ByteBuffers
# EcxNative.clayPerformCodingBatchHostBuffer / mapApplyBatchHostBuffer read each buffer's
# address and capacity themselves (GetDirectBufferAddress / GetDirectBufferCapacity) and
# refuse a layout that addresses past the capacity, as the reference's ByteBuffer get/put
# would throw (ClayCoordinator.kt:378-390), before anything reaches the device.
def clay_batch_layout(S, B, n=6, a=8, ne=1):
    """Stripe-major Clay(4,2) host batch: [S][n*a][B] in, [S][ne*a][B] out."""
    return n * a * B, B, ne * a * B, B, S, B


def test_clay_batch_host_buffer_extent_checks(J):
    clay = handle(J, "clayCreate", 4, 2, J.ints([1]), 1)
    try:
        S, B = 3, 256
        iss, isl, oss, osl, _, _ = clay_batch_layout(S, B)
        inp, out = rnd(S * iss, 1), np.zeros(S * oss, np.uint8)
        mi, mo = np.zeros(1, np.int32), np.zeros(1, np.int32)
        cm = np.zeros(1, np.int64)
        assert J.call("clayMap", clay, J.array(cm)) == OK
        assert J.call("mapSlotExtent", int(cm[0]), J.array(mi), J.array(mo)) == OK
        # node 1 erased: the last slot read is plane 7's node 5 (47), the last written plane 7's (7)
        assert (int(mi[0]), int(mo[0])) == (47, 7)
        need_in = (S - 1) * iss + 47 * isl + B
        need_out = (S - 1) * oss + 7 * osl + B
        J.reset()  # count the pins of the batch calls below only
        call = lambda i, o, **kw: J.call("clayPerformCodingBatchHostBuffer", clay, i, kw.get("iss", iss), isl, o,  # noqa: E731
                                         oss, osl, kw.get("S", S), kw.get("B", B))
        assert call(J.direct(inp, need_in - 1), J.direct(out)) == IDX      # input one byte short
        assert call(J.direct(inp), J.direct(out, need_out - 1)) == IDX     # output one byte short
        assert call(J.direct(inp), J.direct(out), S=4) == IDX              # one stripe too many
        assert call(J.direct(inp), J.direct(out), B=B + 1) == IDX          # sub-chunks past the stride
        assert call(J.direct(inp), J.direct(out), iss=1 << 62) == IDX      # extent overflows int64
        assert call(J.direct(inp), J.direct(out), iss=-1) == ILL           # negative stride
        assert call(J.direct(inp), J.direct(out), S=-1) == ILL
        assert call(J.array(inp), J.direct(out)) == NUL                    # heap buffer: no address
        assert call(None, J.direct(out)) == NUL
        assert call(J.direct(inp), None) == NUL
        assert J.call("clayPerformCodingBatchHostBuffer", 0, J.direct(inp), iss, isl, J.direct(out), oss, osl,
                      S, B) == NUL
        assert J.counters()["pins"] == 0 and (out == 0).all()  # nothing pinned, nothing written
        # exactly the extent: reaches the export (the device, or ECX_E_DEVICE without one)
        st = call(J.direct(inp, need_in), J.direct(out, need_out))
        assert st == (OK if has_device(J) else DEV), st
        assert call(J.direct(inp), J.direct(out), S=0) == OK  # an empty batch touches nothing
    finally:
        J.call("clayDestroy", clay)
    # nothing erased: performCoding returns before any check (ClayCodeErasureDecodingStep.java:54-56)
    none = handle(J, "clayCreate", 4, 2, J.ints([]), 0)
    try:
        assert J.call("clayPerformCodingBatchHostBuffer", none, None, 0, 0, None, 0, 0, 3, 64) == OK
    finally:
        J.call("clayDestroy", none)


def test_map_batch_host_buffer_extent_checks(J):
    mat = np.arange(1, 13, dtype=np.uint8).reshape(3, 4)
    mp = handle(J, "mapCreate", J.array(mat), 3, 4, J.ints([0, 2, 4, 6]), J.ints([1, 3, 5]))
    try:
        S, L, pitch = 5, 100, 128
        inp, out = rnd(S * 8 * pitch, 2), np.zeros(S * 8 * pitch, np.uint8)
        need_in, need_out = (S - 1) * 8 * pitch + 6 * pitch + L, (S - 1) * 8 * pitch + 5 * pitch + L
        J.reset()
        call = lambda i, o: J.call("mapApplyBatchHostBuffer", mp, i, 8 * pitch, pitch, o, 8 * pitch, pitch, S, L)  # noqa: E731
        assert call(J.direct(inp, need_in - 1), J.direct(out)) == IDX
        assert call(J.direct(inp), J.direct(out, need_out - 1)) == IDX
        assert call(J.array(inp), J.direct(out)) == NUL
        assert J.counters()["pins"] == 0 and (out == 0).all()
        st = call(J.direct(inp, need_in), J.direct(out, need_out))
        assert st == (OK if has_device(J) else DEV), st
    finally:
        J.call("mapDestroy", mp)


def test_clay_batch_host_devices_buffer_checks(J):
    """clayPerformCodingBatchHostDevicesBuffer: the same capacity checks as the one-GPU form,
    plus the device list -- shorter than ndev, null, or ndev < 0 -- refused before anything is
    pinned or copied; a valid call reaches the export (the devices, or ECX_E_DEVICE)."""
    clay = handle(J, "clayCreate", 4, 2, J.ints([1]), 1)
    try:
        S, B = 3, 256
        iss, isl, oss, osl, _, _ = clay_batch_layout(S, B)
        inp, out = rnd(S * iss, 1), np.zeros(S * oss, np.uint8)
        need_in = (S - 1) * iss + 47 * isl + B
        J.reset()
        call = lambda i, o, devs, nd: J.call("clayPerformCodingBatchHostDevicesBuffer", clay, i, iss, isl, o,  # noqa: E731
                                             oss, osl, S, B, devs, nd)
        assert call(J.direct(inp, need_in - 1), J.direct(out), J.ints([0]), 1) == IDX
        assert call(J.direct(inp), J.direct(out), J.ints([0]), 2) == ILL   # list shorter than ndev
        assert call(J.direct(inp), J.direct(out), None, 1) == NUL
        assert call(J.direct(inp), J.direct(out), J.ints([0]), -1) == ILL
        assert call(J.array(inp), J.direct(out), J.ints([0]), 1) == NUL     # heap buffer
        assert J.counters()["pins"] == 0 and (out == 0).all()
        st = call(J.direct(inp), J.direct(out), J.ints([0, 0]), 2)
        assert st == (OK if has_device(J) else DEV), st
        if has_device(J):
            assert call(J.direct(inp), J.direct(out), J.ints([1 << 20]), 1) == ILL  # unknown device id
    finally:
        J.call("clayDestroy", clay)


def test_rs_check_batch_host_buffer_checks(J):
    """rsIsParityCorrectBatchHost(Devices)Buffer: the stripes' ByteBuffer must hold every shard
    of every stripe up to offset + byteCount, the verdict ByteBuffer one byte per stripe; short,
    heap or null buffers and a bad device list are refused before anything is read or written."""
    rs = handle(J, "rsCreate", 17, 3)
    try:
        S, L = 3, 512
        ss, sl = 20 * L, L
        shards, verdict = rnd(S * ss, 21), np.full(S, 7, np.uint8)
        need = (S - 1) * ss + 19 * sl + L
        J.reset()
        call = lambda b, v, **kw: J.call("rsIsParityCorrectBatchHostBuffer", rs, b, ss, sl, kw.get("S", S),  # noqa: E731
                                         kw.get("off", 0), kw.get("L", L), v)
        assert call(J.direct(shards, need - 1), J.direct(verdict)) == IDX     # stripes one byte short
        assert call(J.direct(shards), J.direct(verdict, S - 1)) == IDX         # verdict one byte short
        assert call(J.direct(shards), J.direct(verdict), off=1) == IDX         # window past the shard pitch end
        assert call(J.direct(shards), J.direct(verdict), off=-1) == ILL
        assert call(J.direct(shards), J.direct(verdict), S=-1) == ILL
        assert call(J.array(shards), J.direct(verdict)) == NUL                 # heap buffer
        assert call(J.direct(shards), None) == NUL
        dcall = lambda devs, nd: J.call("rsIsParityCorrectBatchHostDevicesBuffer", rs, J.direct(shards), ss, sl,  # noqa: E731
                                        S, 0, L, J.direct(verdict), devs, nd)
        assert dcall(J.ints([0]), 2) == ILL and dcall(None, 1) == NUL and dcall(J.ints([0]), -1) == ILL
        assert J.counters()["pins"] == 0 and (verdict == 7).all()
        st = call(J.direct(shards, need), J.direct(verdict, S))
        assert st == (OK if has_device(J) else DEV), st
    finally:
        J.call("rsDestroy", rs)


def _np_blocked(nat, block):
    """[S][n][L] -> the blocked layout (include/ecx.h): body [S][full][n][block], tails [S][n][tail]."""
    S, n, L = nat.shape
    full, tail = divmod(L, block)
    body = nat[:, :, :full * block].reshape(S, n, full, block).transpose(0, 2, 1, 3).reshape(-1)
    return np.concatenate([body, nat[:, :, full * block:].reshape(-1)])


def test_rs_blocked_batch_host_buffer_checks(J):
    """rsEncodeParityBlockedBatchHostBuffer / rsDecodeMissingBlockedBatchHostBuffer (round 6): the
    ByteBuffer must hold nstripes whole stripes (n * byteCount bytes each, blocks and tails), the
    shardPresent flags n bytes (copied, never pinned); short, heap or null buffers, short flags and
    an overflowing stripe size are refused before anything is touched; on the GPU the blocked
    stripes come back equal to the oracle's encodeParity / decodeMissing."""
    k, m, S, L, blk = 5, 3, 3, 1000, 256
    n = k + m
    rs = handle(J, "rsCreate", k, m)
    try:
        nat = np.random.default_rng(61).integers(0, 256, (S, n, L), dtype=np.uint8)
        buf = _np_blocked(nat, blk)
        need = S * n * L
        pres = np.ones(n, np.uint8)
        pres[[0, 6]] = 0
        J.reset()
        enc = lambda b, **kw: J.call("rsEncodeParityBlockedBatchHostBuffer", rs, b, kw.get("S", S), kw.get("L", L),  # noqa: E731
                                     blk)
        dec = lambda p, b, **kw: J.call("rsDecodeMissingBlockedBatchHostBuffer", rs, p, b, kw.get("S", S),  # noqa: E731
                                        kw.get("L", L), blk)
        before = buf.copy()
        assert enc(J.direct(buf, need - 1)) == IDX and dec(J.array(pres), J.direct(buf, need - 1)) == IDX
        assert enc(J.direct(buf), S=S + 1) == IDX                          # one stripe too many
        assert enc(J.direct(buf), L=1 << 62) == ILL                        # n * byteCount overflows
        assert enc(J.direct(buf), S=-1) == ILL and enc(J.direct(buf), L=-1) == ILL
        assert enc(J.array(buf)) == NUL and enc(None) == NUL               # heap / null buffer
        assert dec(J.array(pres[:n - 1]), J.direct(buf)) == IDX            # flags one short
        assert dec(None, J.direct(buf)) == NUL
        assert J.call("rsEncodeParityBlockedBatchHostBuffer", 0, J.direct(buf), S, L, blk) == NUL
        denc = lambda b, devs, nd: J.call("rsEncodeParityBlockedBatchHostDevicesBuffer", rs, b, S, L, blk,  # noqa: E731
                                          devs, nd)
        ddec = lambda p, devs, nd: J.call("rsDecodeMissingBlockedBatchHostDevicesBuffer", rs, p, J.direct(buf),  # noqa: E731
                                          S, L, blk, devs, nd)
        assert denc(J.direct(buf, need - 1), J.ints([0]), 1) == IDX
        assert denc(J.direct(buf), J.ints([0]), 2) == ILL and denc(J.direct(buf), None, 1) == NUL
        assert denc(J.direct(buf), J.ints([0]), -1) == ILL and denc(J.array(buf), J.ints([0]), 1) == NUL
        assert ddec(J.array(pres[:n - 1]), J.ints([0]), 1) == IDX and ddec(J.array(pres), J.ints([0]), 2) == ILL
        assert J.counters()["pins"] == 0 and (buf == before).all()
        st = enc(J.direct(buf))
        assert st == (OK if has_device(J) else DEV), st
        if st == OK:
            assert (buf == _np_blocked(_oracle_rs(k, m, nat, "encode"), blk)).all()
            buf[:] = _np_blocked(nat, blk)
            assert dec(J.array(pres), J.direct(buf)) == OK
            assert (buf == _np_blocked(_oracle_rs(k, m, nat, "decode", pres), blk)).all()
            buf[:] = _np_blocked(nat, blk)
            assert denc(J.direct(buf), J.ints([0, 0]), 2) == OK
            assert (buf == _np_blocked(_oracle_rs(k, m, nat, "encode"), blk)).all()
            buf[:] = _np_blocked(nat, blk)
            assert ddec(J.array(pres), J.ints([0, 0]), 2) == OK
            assert (buf == _np_blocked(_oracle_rs(k, m, nat, "decode", pres), blk)).all()
    finally:
        J.call("rsDestroy", rs)


def _oracle_rs(k, m, nat, op, pres=None):
    out = nat.copy()
    for s in range(nat.shape[0]):
        shards = [out[s, i] for i in range(k + m)]  # views: the oracle writes in place
        if op == "encode":
            O.ReedSolomon(k, m).encode_parity(shards, 0, nat.shape[2])
        else:
            O.ReedSolomon(k, m).decode_missing(shards, [bool(x) for x in pres], 0, nat.shape[2])
    return out


def test_codec_reference_survives_other_releases(J):
    """The registry side of ADVICE r04 (EcxPartialSums / EcxClayCodeErasureDecodingStep close):
    two handles of one (k, m) codec are one shared object; releasing one and then more than
    64 other codecs (the idle cache) leaves the other usable -- which is why the Java close()
    now releases at most once (asserted on the Java sources below)."""
    a = handle(J, "rsCreate", 6, 3)
    b = handle(J, "rsCreate", 6, 3)
    assert a == b
    J.call("rsDestroy", a)
    for k in range(2, 2 + 70):
        h = handle(J, "rsCreate", k, 1)
        J.call("rsDestroy", h)
    k_, m_ = np.zeros(1, np.int32), np.zeros(1, np.int32)
    assert J.call("rsShape", b, J.array(k_), J.array(m_)) == OK and (k_[0], m_[0]) == (6, 3)
    mat = np.zeros(9 * 6, np.uint8)
    assert J.call("rsMatrix", b, J.array(mat)) == OK
    assert (mat.reshape(9, 6)[:6] == np.eye(6, dtype=np.uint8)).all()
    J.call("rsDestroy", b)
    from pathlib import Path
    root = Path(__file__).resolve().parents[1] / "jni"
    for f, field in (("com/backblaze/erasure/ecx/EcxPartialSums.java", "rs"),
                     ("com/backblaze/erasure/ecx/EcxParityCheck.java", "rs"),
                     ("com/backblaze/erasure/ecx/EcxBlockedStripes.java", "rs"),
                     ("distributed/erasure/coding/clay/EcxClayCodeErasureDecodingStep.java", "clay")):
        src = (root / f).read_text()
        close = src[src.index("public synchronized void close()"):]
        close = close[:close.index("\n    }\n")]
        assert "if (%s == 0)" % field in close and "%s = 0;" % field in close, f
        assert "private long %s;" % field in src and "IllegalStateException" in src, f


def test_parity_check_wrapper_uses_the_checked_variants():
    """EcxParityCheck (the batch isParityCorrect for JVM callers) reaches libecx only through
    the capacity-checked ByteBuffer natives, and checks the same extents in Java first."""
    from pathlib import Path
    src = (Path(__file__).resolve().parents[1] / "jni" / "com" / "backblaze" / "erasure" / "ecx" /
           "EcxParityCheck.java").read_text()
    used = set(re.findall(r"EcxNative\.(\w+)\(", src))
    assert used == {"rsIsParityCorrectBatchHostBuffer", "rsIsParityCorrectBatchHostDevicesBuffer", "rsDestroy"}
    assert src.count("checkExtent(stripes") == 2 and "ArrayIndexOutOfBoundsException" in src


def test_java_wrapper_uses_the_checked_variant():
    """EcxClayCodeErasureDecodingStep.performCodingBatchHost goes through the capacity-checked
    native and checks the same extent in Java first (ArrayIndexOutOfBoundsException /
    NullPointerException), so a short or heap buffer never reaches the address-taking path."""
    from pathlib import Path
    src = (Path(__file__).resolve().parents[1] / "jni" / "distributed" / "erasure" / "coding" / "clay" /
           "EcxClayCodeErasureDecodingStep.java").read_text()
    body = src[src.index("public void performCodingBatchHost"):]
    body = body[:body.index("\n    }\n")]
    assert "clayPerformCodingBatchHostBuffer" in body and "directAddress" not in body
    assert "checkExtent(in" in body and "checkExtent(out" in body
    assert "ArrayIndexOutOfBoundsException" in src and "isDirect()" in src


# ---------------------------------------------------------------- GPU: results through the binding
@pytest.mark.gpu
def test_code_some_shards_via_jni_vs_oracle(J):
    rows = O.ReedSolomon(4, 2).parity_rows.astype(np.uint8).copy()
    L, off, pos = 5000, 7, 3
    ins = [rnd(pos + off + L, 10 + i) for i in range(4)]
    outs = [rnd(pos + off + L + 5, 20 + i) for i in range(2)]
    before = [o.copy() for o in outs]
    st = J.call("codeSomeShards", J.array(rows), J.array2d(ins), J.ints([pos] * 4), 4, J.array2d(outs),
                J.ints([pos] * 2), 2, off, L)
    assert st == OK, st
    ref = [np.zeros(L, np.uint8) for _ in range(2)]
    O.code_some_shards(rows, [i[pos + off:pos + off + L] for i in ins], ref, 0, L)
    for o, b, r in zip(outs, before, ref):
        assert (o[pos + off:pos + off + L] == r).all()
        assert (o[:pos + off] == b[:pos + off]).all() and (o[pos + off + L:] == b[pos + off + L:]).all()
    chk = np.zeros(1, np.int32)
    assert J.call("checkSomeShards", J.array(rows), J.array2d(ins), J.ints([pos] * 4), 4, J.array2d(outs),
                  J.ints([pos] * 2), 2, off, L, None) == 1
    outs[1][pos + off + 100] ^= 1
    assert J.call("checkSomeShards", J.array(rows), J.array2d(ins), J.ints([pos] * 4), 4, J.array2d(outs),
                  J.ints([pos] * 2), 2, off, L, None) == 0
    del chk


@pytest.mark.gpu
def test_rs_codec_via_jni_vs_oracle(J):
    rs = handle(J, "rsCreate", 4, 2)
    try:
        L = 4097
        shards = [rnd(L, 30 + i) for i in range(4)] + [np.zeros(L, np.uint8) for _ in range(2)]
        assert J.call("rsEncodeParity", rs, J.array2d(shards), None, 6, L, 0, L) == OK
        ref = [s.copy() for s in shards]
        ref[4][:] = 0
        ref[5][:] = 0
        O.ReedSolomon(4, 2).encode_parity(ref, 0, L)
        assert all((a == b).all() for a, b in zip(shards, ref))
        assert J.call("rsIsParityCorrect", rs, J.array2d(shards), None, 6, L, 0, L, None, 0) == 1
        lost = [s.copy() for s in shards]
        lost[1][:] = 0
        lost[4][:] = 0
        present = np.array([1, 0, 1, 1, 0, 1], np.uint8)
        assert J.call("rsDecodeMissing", rs, J.array2d(lost), None, J.array(present), 6, L, 0, L) == OK
        assert all((a == b).all() for a, b in zip(lost, ref))
        three = np.array([1, 0, 0, 1, 0, 1], np.uint8)
        assert J.call("rsDecodeMissing", rs, J.array2d(lost), None, J.array(three), 6, L, 0, L) == NSH
        # decodeMissingSingle: helper 2's share of the missing data shard 1 (ClayCodeNode chain hop)
        pres = np.array([1, 0, 1, 1, 1, 1], np.uint8)
        got = [rnd(L, 5)]
        want = [np.zeros(L, np.uint8)]
        assert J.call("rsDecodeMissingSingle", rs, J.array(shards[2]), 2, 1, J.array(pres), J.array2d(got), None, 1,
                      0, L, 1) == OK
        O.ReedSolomon(4, 2).decode_missing_single(shards[2], 2, 1, [bool(p) for p in pres], want, 0, L, True)
        assert (got[0] == want[0]).all()
    finally:
        J.call("rsDestroy", rs)


@pytest.mark.gpu
@pytest.mark.parametrize("B,pos", [(4096, 0), (1000, 3)])
def test_clay_perform_coding_via_jni_vs_oracle(J, B, pos):
    clay = handle(J, "clayCreate", 4, 2, J.ints([1]), 1)
    try:
        n, a = 6, 8
        ins = [None if i % n == 1 else rnd(pos + B, 40 + i) for i in range(n * a)]
        outs = [np.full(pos + B, 0x77, np.uint8) for _ in range(a)]
        st = J.call("clayPerformCoding", clay, J.array2d(ins), J.ints([pos] * (n * a)), J.array2d(outs),
                    J.ints([pos] * a), B)
        assert st == OK, st
        ref = [np.zeros(B, np.uint8) for _ in range(a)]
        O.Clay(4, 2, [1]).perform_coding([None if x is None else x[pos:].copy() for x in ins], ref, B)
        for o, r in zip(outs, ref):
            assert (o[pos:] == r).all() and (o[:pos] == 0x77).all()
    finally:
        J.call("clayDestroy", clay)


@pytest.mark.gpu
def test_clay_batch_host_buffer_via_jni_vs_oracle(J):
    """Clay(4,2), e = 1, three stripes of 4 KiB sub-chunks in direct host buffers, through the
    capacity-checked forwarder: every repaired sub-chunk equals the oracle's performCoding."""
    clay = handle(J, "clayCreate", 4, 2, J.ints([1]), 1)
    try:
        S, B, n, a = 3, 4096, 6, 8
        iss, isl, oss, osl, _, _ = clay_batch_layout(S, B)
        inp = rnd(S * iss, 3)
        out = np.full(S * oss, 0x5A, np.uint8)
        st = J.call("clayPerformCodingBatchHostBuffer", clay, J.direct(inp), iss, isl, J.direct(out), oss, osl, S, B)
        assert st == OK, st
        for s_ in range(S):
            ins = [None if i % n == 1 else inp[s_ * iss + i * B:s_ * iss + (i + 1) * B].copy() for i in range(n * a)]
            ref = [np.zeros(B, np.uint8) for _ in range(a)]
            O.Clay(4, 2, [1]).perform_coding(ins, ref, B)
            for z in range(a):
                assert (out[s_ * oss + z * B:s_ * oss + (z + 1) * B] == ref[z]).all(), (s_, z)
    finally:
        J.call("clayDestroy", clay)


@pytest.mark.gpu
def test_clay_batch_host_devices_buffer_via_jni_vs_oracle(J):
    """The multi-GPU forwarder over device list [0, 0] (two workers), a ragged 5 stripes:
    every repaired sub-chunk equals the oracle's performCoding."""
    clay = handle(J, "clayCreate", 4, 2, J.ints([4]), 1)
    try:
        S, B, n, a = 5, 4096, 6, 8
        iss, isl, oss, osl, _, _ = clay_batch_layout(S, B)
        inp = rnd(S * iss, 13)
        out = np.full(S * oss, 0x5A, np.uint8)
        st = J.call("clayPerformCodingBatchHostDevicesBuffer", clay, J.direct(inp), iss, isl, J.direct(out), oss, osl,
                    S, B, J.ints([0, 0]), 2)
        assert st == OK, st
        for s_ in range(S):
            ins = [None if i % n == 4 else inp[s_ * iss + i * B:s_ * iss + (i + 1) * B].copy() for i in range(n * a)]
            ref = [np.zeros(B, np.uint8) for _ in range(a)]
            O.Clay(4, 2, [4]).perform_coding(ins, ref, B)
            for z in range(a):
                assert (out[s_ * oss + z * B:s_ * oss + (z + 1) * B] == ref[z]).all(), (s_, z)
    finally:
        J.call("clayDestroy", clay)


@pytest.mark.gpu
def test_rs_check_batch_host_buffer_via_jni_vs_oracle(J):
    """RS(17,3) isParityCorrect over 7 host stripes through the checked ByteBuffer forwarders,
    one device and the list [0, 0]: stripes encoded by the oracle pass, a stripe with one byte
    flipped (a data shard, a parity shard's last byte) fails, as the oracle's isParityCorrect says."""
    rs = handle(J, "rsCreate", 17, 3)
    try:
        S, L = 7, 3000
        ss, sl = 20 * L, L
        shards = rnd(S * ss, 31)
        for s_ in range(S):
            sh = [shards[s_ * ss + i * L:s_ * ss + (i + 1) * L].copy() for i in range(20)]
            O.ReedSolomon(17, 3).encode_parity(sh, 0, L)
            shards[s_ * ss:(s_ + 1) * ss] = np.concatenate(sh)
        shards[2 * ss + 5 * L + 17] ^= 1         # stripe 2: data shard 5
        shards[6 * ss + 19 * L + L - 1] ^= 0x80  # stripe 6: parity shard 19's last byte
        want = []
        for s_ in range(S):
            sh = [shards[s_ * ss + i * L:s_ * ss + (i + 1) * L].copy() for i in range(20)]
            want.append(1 if O.ReedSolomon(17, 3).is_parity_correct(sh, 0, L) else 0)
        assert want == [1, 1, 0, 1, 1, 1, 0]
        for devs in (None, [0, 0]):
            verdict = np.full(S, 7, np.uint8)
            if devs is None:
                st = J.call("rsIsParityCorrectBatchHostBuffer", rs, J.direct(shards), ss, sl, S, 0, L, J.direct(verdict))
            else:
                st = J.call("rsIsParityCorrectBatchHostDevicesBuffer", rs, J.direct(shards), ss, sl, S, 0, L,
                            J.direct(verdict), J.ints(devs), len(devs))
            assert st == OK, st
            assert verdict.tolist() == want, (devs, verdict.tolist())
    finally:
        J.call("rsDestroy", rs)


@pytest.mark.gpu
def test_map_batch_host_buffer_via_jni_vs_oracle(J):
    mat = np.random.default_rng(4).integers(0, 256, (3, 4), dtype=np.uint8)
    mp = handle(J, "mapCreate", J.array(mat), 3, 4, J.ints([0, 2, 4, 6]), J.ints([1, 3, 5]))
    try:
        S, L, pitch = 5, 1000, 1024
        inp, out = rnd(S * 8 * pitch, 5), np.zeros(S * 8 * pitch, np.uint8)
        st = J.call("mapApplyBatchHostBuffer", mp, J.direct(inp), 8 * pitch, pitch, J.direct(out), 8 * pitch, pitch,
                    S, L)
        assert st == OK, st
        for s_ in range(S):
            base = s_ * 8 * pitch
            ins = [inp[base + j * pitch:base + j * pitch + L] for j in (0, 2, 4, 6)]
            ref = [np.zeros(L, np.uint8) for _ in range(3)]
            O.code_some_shards(mat, ins, ref, 0, L)
            for r, slot in zip(ref, (1, 3, 5)):
                assert (out[base + slot * pitch:base + slot * pitch + L] == r).all()
    finally:
        J.call("mapDestroy", mp)


def test_round6_entry_points_through_binding(J):
    """Round 6's exports through their generated forwarders (CPU, no device work): the RS layout
    contract's long[] outputs (rsBlockedLayout / rsRecommendedPitch, pinned and released, a short
    array refused with ArrayIndexOutOfBounds before any pin), and clayCreateEx with the isTest
    flag (its int[] erased list copied, not pinned) -- a distinct shared codec from clayCreate's."""
    lay = np.zeros(3, np.int64)
    assert J.call("rsBlockedLayout", 17, 3, 200000, J.array(lay)) == OK
    assert lay.tolist() == [32768, 6, 200000 - 6 * 32768]
    pitch = np.zeros(1, np.int64)
    assert J.call("rsRecommendedPitch", 12, 4, 4 << 20, J.array(pitch)) == OK and pitch[0] == (4 << 20) + 4096
    J.reset()
    assert J.call("rsBlockedLayout", 17, 3, 200000, J.array(np.zeros(2, np.int64))) == IDX
    assert J.call("rsBlockedLayout", 17, 3, 200000, None) == NUL
    assert J.counters()["pins"] == 0
    c = J.counters()
    assert c["violations"] == 0 and c["pins_now"] == 0
    test = handle(J, "clayCreateEx", 4, 2, 0, J.ints([2]), 1, 1)
    std = handle(J, "clayCreate", 4, 2, J.ints([2]), 1)
    try:
        assert test != std
        assert J.counters()["pins_now"] == 0
        assert J.call("clayCreateEx", 4, 2, 0, J.ints([2]), 1, 2, J.array(np.zeros(1, np.int64))) == ILL  # unknown flag
    finally:
        J.call("clayDestroy", test)
        J.call("clayDestroy", std)
