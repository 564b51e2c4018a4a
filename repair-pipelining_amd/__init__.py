"""repair_pipelining_amd -- MI355X-native GF(256) erasure engine.

Host-side mirror of the reference's coding API (krishnarb3/repair-pipelining:
rs/ ``com.backblaze.erasure``, clay/ ``distributed.erasure.coding.clay``,
lrc/ ``distributed.erasure.coding``) over the C ABI of libecx.so
(include/ecx.h).  Method names, argument meaning and error behaviour follow
the Java classes; byte[] becomes a 1-D ``numpy.uint8`` array and Java
exceptions become :class:`EcxError` carrying the ecx_status code.

All arithmetic runs in hand-written HIP kernels on the MI355X; the host side
only plans (GF tables, matrix inverses, the composed Clay map).  There is no
CPU fallback.

Batch (device-resident) APIs take torch CUDA tensors or raw device pointers.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Optional, Sequence

import numpy as np

from ._lib import EcxError, build, check, lib, LIB_PATH, HEADER  # noqa: F401

__all__ = [
    "EcxError", "Galois", "Matrix", "CodingLoop", "InputOutputByteTableCodingLoop",
    "InputOutputByteTableCodingLoopSingle", "ReedSolomon", "GfMap", "ClayCodeUtil",
    "ClayCodeErasureDecodingStep", "ClayCode", "LRCErasureCode", "LRCErasureUtil", "JavaRandom",
    "lrc_encode", "lrc_encode_using_single", "lrc_decode", "sample_encode", "sample_decode",
    "device_count", "set_device", "fill_random", "count_mismatch", "shard_stripes",
    "ECChunk", "ECBlock", "ClayCodeHelper", "write_subchunk", "read_subchunk",
]


def shard_stripes(n_stripes: int, world: int, rank: int):
    """Stripe range [begin, end) that rank `rank` of `world` owns.  Stripes are
    independent (every repair reads only its own stripe), so the batch is split
    into contiguous ranges with no data exchange between GPUs."""
    if world <= 0 or not 0 <= rank < world or n_stripes < 0:
        raise ValueError("invalid partition request")
    base, extra = divmod(n_stripes, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


# ---------------------------------------------------------------- ECChunk.java / ECBlock.java
class ECChunk:
    """Hadoop-style chunk wrapper (ECChunk.java:37-109); the buffer may be None."""

    def __init__(self, buffer=None, offset: int = 0, length: Optional[int] = None):
        if buffer is not None and (offset or length is not None):
            buffer = buffer[offset:offset + (len(buffer) - offset if length is None else length)]
        self.buffer = buffer
        self.allZero = False

    def getBuffer(self):
        return self.buffer

    def isAllZero(self):
        return self.allZero

    def setAllZero(self, v: bool):
        self.allZero = v

    def toBytesArray(self) -> np.ndarray:
        return np.array(self.buffer, np.uint8)

    @staticmethod
    def toBuffers(chunks):
        """ECChunk.toBuffers (ECChunk.java:81-95): null chunks map to null buffers."""
        return [None if c is None else c.getBuffer() for c in chunks]


class ECBlock:
    """ECBlock.java:36-99 -- flags are carried but, as in the reference, unused by the math."""

    def __init__(self, chunk: Optional[ECChunk] = None, isParity: bool = False, isErased: bool = False):
        self.chunk, self.isParity, self.isErased = chunk, isParity, isErased

    def getChunk(self):
        return self.chunk

    def setChunk(self, c):
        self.chunk = c


def _buffers(items):
    """Accept ndarray / None / ECChunk / ECBlock entries (the reference passes ECChunk[])."""
    out = []
    for it in items:
        if isinstance(it, ECBlock):
            it = it.chunk
        if isinstance(it, ECChunk):
            it = it.buffer
        out.append(it)
    return out


# ---------------------------------------------------------------- helpers
def _u8(a) -> np.ndarray:
    if not (isinstance(a, np.ndarray) and a.dtype == np.uint8 and a.flags.c_contiguous):
        raise TypeError("byte buffers must be C-contiguous numpy.uint8 arrays")
    return a


def _addr(a: np.ndarray) -> int:
    """Data address of a checked uint8 array.  ctypes' from_buffer is about 3x cheaper
    than ndarray.ctypes.data (which builds a helper object per call) -- it matters
    for per-call APIs that take 50+ buffers; read-only or empty arrays take the slow
    path."""
    try:
        return ctypes.addressof(ctypes.c_char.from_buffer(a))
    except (TypeError, ValueError):
        return a.ctypes.data


def _ptr_array(bufs) -> ctypes.Array:
    arr = (ctypes.c_void_p * max(1, len(bufs)))()
    arr[:len(bufs)] = [None if b is None else _addr(_u8(b)) for b in bufs]
    return arr


def _bytes(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.int64) & 0xFF, dtype=np.uint8)


def _dev_ptr(x) -> int:
    """Device pointer of a torch CUDA tensor or an int."""
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        if not x.is_cuda:
            raise TypeError("batch APIs take device (CUDA/HIP) tensors")
        return int(x.data_ptr())
    raise TypeError("expected a device tensor or an integer pointer")


def _host_ptr(x) -> int:
    """Host address of a numpy array, a CPU torch tensor (pinned or not) or an int."""
    if isinstance(x, int):
        return x
    if isinstance(x, np.ndarray):
        return int(x.ctypes.data)
    if hasattr(x, "data_ptr"):
        if x.is_cuda:
            raise TypeError("host batch APIs take host (CPU) buffers")
        return int(x.data_ptr())
    raise TypeError("expected a host array/tensor or an integer pointer")


def _avail_bytes(x) -> Optional[int]:
    """Bytes addressable from the buffer's first byte to the end of its allocation:
    torch tensors use their storage, numpy arrays their outermost base array.
    None for raw integer pointers (the caller vouches for those)."""
    if isinstance(x, int):
        return None
    if isinstance(x, np.ndarray):
        base = x
        while isinstance(base.base, np.ndarray):
            base = base.base
        hi = base.ctypes.data + base.nbytes if base.flags.c_contiguous else None
        return None if hi is None else hi - x.ctypes.data
    if hasattr(x, "untyped_storage"):
        st = x.untyped_storage()
        return st.data_ptr() + st.nbytes() - x.data_ptr()
    return None


def _check_layout(buf, stripe_stride, slot_stride, max_slot, nstripes, nbytes, what):
    """Fail loudly (ArrayIndexOutOfBoundsException, as a Java ByteBuffer would)
    instead of letting a kernel address past the end of `buf`."""
    if nstripes <= 0 or nbytes <= 0:
        return
    if stripe_stride < 0 or slot_stride < 0:
        raise EcxError(-1, f"{what}: negative stride")
    avail = _avail_bytes(buf)
    need = (nstripes - 1) * stripe_stride + max(0, max_slot) * slot_stride + nbytes
    if avail is not None and need > avail:
        raise EcxError(-5, f"{what}: the batch layout addresses {need} bytes but the buffer holds {avail}")


def _check_extent(buf, nbytes, what):
    avail = _avail_bytes(buf)
    if nbytes > 0 and avail is not None and nbytes > avail:
        raise EcxError(-5, f"{what}: the batch addresses {nbytes} bytes but the buffer holds {avail}")


def blocked_pack(shards, block_bytes: int, out=None):
    """The blocked layout (include/ecx.h ecx_rs_blocked_layout) of a [stripes][n][L] uint8
    tensor, as a flat tensor of stripes * n * L bytes: body [stripe][block][shard][block_bytes],
    then tails [stripe][shard][L % block_bytes] (torch copies on the tensor's device)."""
    S, n, L = shards.shape
    full, tail = divmod(L, block_bytes)
    if out is None:
        out = shards.new_empty(S * n * L)
    body = full * n * block_bytes
    if full:
        out[:S * body].view(S, full, n, block_bytes).copy_(
            shards[:, :, :full * block_bytes].reshape(S, n, full, block_bytes).permute(0, 2, 1, 3))
    if tail:
        out[S * body:].view(S, n, tail).copy_(shards[:, :, full * block_bytes:])
    return out


def blocked_unpack(flat, stripes: int, n: int, byte_count: int, block_bytes: int, slots=None, first: int = 0,
                   count: int = None):
    """The natural [count][len(slots)][byte_count] shards (default: every stripe, every slot) of
    stripes first..first+count-1 of a blocked-layout buffer of `stripes` stripes (a copy)."""
    import torch
    count = stripes - first if count is None else count
    slots = list(range(n)) if slots is None else list(slots)
    full, tail = divmod(byte_count, block_bytes)
    body = full * n * block_bytes
    parts = []
    if full:
        b = flat[:stripes * body].view(stripes, full, n, block_bytes)[first:first + count][:, :, slots, :]
        parts.append(b.permute(0, 2, 1, 3).reshape(count, len(slots), full * block_bytes))
    if tail:
        t = flat[stripes * body:stripes * n * byte_count].view(stripes, n, tail)[first:first + count]
        parts.append(t[:, slots, :])
    return torch.cat(parts, dim=2) if len(parts) > 1 else parts[0].clone()


class HostBuffer:
    """Page-locked host memory from ecx_host_alloc, viewed as a numpy uint8 array."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        check(lib().ecx_host_alloc(nbytes, ctypes.byref(p)))
        self._p = p
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * max(1, nbytes)).from_address(p.value))[:nbytes]

    def __del__(self):
        if getattr(self, "_p", None) and lib is not None:
            lib().ecx_host_free(self._p)
            self._p = None


def host_register(arr) -> None:
    """Page-lock an existing host buffer (hipHostRegister) for PCIe-rate host batches."""
    check(lib().ecx_host_register(_host_ptr(arr), int(arr.nbytes)))


def host_unregister(arr) -> None:
    check(lib().ecx_host_unregister(_host_ptr(arr)))


def tune(key: str, value: int) -> None:
    """Launch-shape knobs (include/ecx_tune.h); results are bit-identical for every setting."""
    f = lib().ecx_tune
    f.argtypes, f.restype = [ctypes.c_char_p, ctypes.c_int], ctypes.c_int
    check(f(key.encode(), int(value)))


def tune_value(key: str) -> int:
    """The current value of a deployment knob (ecx_tune_value, include/ecx_tune.h)."""
    f = lib().ecx_tune_value
    f.argtypes, f.restype = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)], ctypes.c_int
    v = ctypes.c_int()
    check(f(key.encode(), ctypes.byref(v)))
    return v.value


def is_diag() -> bool:
    """True for the diagnostic library (make DIAG=1, libecx_diag.so): it also holds the
    measured-and-rejected kernels, whose ecx_tune keys the product library refuses."""
    f = lib().ecx_build_diag
    f.argtypes, f.restype = [], ctypes.c_int
    return f() == 1


def last_kernel() -> str:
    """The kernel instance of this thread's last full-chunk launch, as rocprofv3 names it
    (ecx_last_kernel, include/ecx_tune.h); "" before the first launch."""
    f = lib().ecx_last_kernel
    f.argtypes, f.restype = [ctypes.c_char_p, ctypes.c_int], ctypes.c_int
    buf = ctypes.create_string_buffer(256)
    return buf.value.decode() if check(f(buf, len(buf))) > 0 else ""


def last_launch_shape() -> str:
    """That launch's full shape: kernel instance plus the unit order its name does not encode
    ("... stagger=G xcd_group=X xcd_run=R"; ecx_last_launch_shape)."""
    f = lib().ecx_last_launch_shape
    f.argtypes, f.restype = [ctypes.c_char_p, ctypes.c_int], ctypes.c_int
    buf = ctypes.create_string_buffer(512)
    return buf.value.decode() if check(f(buf, len(buf))) > 0 else ""


def probe_bandwidth(kind: int, src, dst, nbytes: int, nontemporal: bool = True, stream=None) -> None:
    """Pure-bandwidth probe kernels (include/ecx_tune.h): kind 0 = read-only stream of
    `src`, kind 1 = copy src -> dst; nbytes a multiple of 16 KiB.  Diagnostics only."""
    f = lib().ecx_probe_bandwidth
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    f.restype = ctypes.c_int
    check(f(kind, _dev_ptr(src), _dev_ptr(dst), nbytes, 1 if nontemporal else 0, _stream(stream)))


def _stream(stream) -> Optional[int]:
    if stream is None:
        try:
            import torch
            return int(torch.cuda.current_stream().cuda_stream)
        except Exception:  # pragma: no cover - no torch / no device
            return None
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)


def device_count() -> int:
    n = ctypes.c_int(0)
    check(lib().ecx_device_count(ctypes.byref(n)))
    return n.value


def set_device(device: int) -> None:
    check(lib().ecx_set_device(device))


def fill_random(dst, nbytes: int, seed: int, stream=None) -> None:
    """Deterministic counter-based synthetic bytes on the device (splitmix64)."""
    check(lib().ecx_fill_random(_dev_ptr(dst), nbytes, seed & 0xFFFFFFFFFFFFFFFF, _stream(stream)))


def count_mismatch(a, a_stride, b, b_stride, nrows, row_bytes, d_count, stream=None) -> None:
    """Accumulate into the device uint64 ``d_count`` the bytes that differ."""
    check(lib().ecx_count_mismatch(_dev_ptr(a), a_stride, None if b is None else _dev_ptr(b), b_stride, nrows,
                                   row_bytes, _dev_ptr(d_count), _stream(stream)))


# ---------------------------------------------------------------- Galois.java
class Galois:
    """GF(2^8) with generating polynomial 29 (Galois.java:43)."""
    FIELD_SIZE = 256
    GENERATING_POLYNOMIAL = 29

    @staticmethod
    def multiply(a: int, b: int) -> int:
        return lib().ecx_gf_multiply(a & 0xFF, b & 0xFF)

    @staticmethod
    def divide(a: int, b: int) -> int:
        return check(lib().ecx_gf_divide(a & 0xFF, b & 0xFF))

    @staticmethod
    def exp(a: int, n: int) -> int:
        return check(lib().ecx_gf_exp(a & 0xFF, n))

    @staticmethod
    def add(a: int, b: int) -> int:
        return (a ^ b) & 0xFF

    subtract = add

    @staticmethod
    def tables():
        log = np.zeros(256, np.int16)
        exp = np.zeros(510, np.uint8)
        mul = np.zeros((256, 256), np.uint8)
        check(lib().ecx_gf_tables(log.ctypes.data, exp.ctypes.data, mul.ctypes.data))
        return log, exp, mul


# ---------------------------------------------------------------- Matrix.java
class Matrix:
    @staticmethod
    def times(a, b) -> np.ndarray:
        a, b = _bytes(a), _bytes(b)
        out = np.zeros((a.shape[0], b.shape[1]), np.uint8)
        check(lib().ecx_matrix_times(a.ctypes.data, a.shape[0], a.shape[1], b.ctypes.data, b.shape[0], b.shape[1],
                                     out.ctypes.data))
        return out

    @staticmethod
    def invert(m) -> np.ndarray:
        m = _bytes(m)
        out = np.zeros_like(m)
        check(lib().ecx_matrix_invert(m.ctypes.data, m.shape[0], out.ctypes.data))
        return out


# ---------------------------------------------------------------- CodingLoop.java
class CodingLoop:
    """The reference's operator/plugin interface (CodingLoop.java:79-117),
    implemented by one fused HIP kernel launch per call."""

    def codeSomeShards(self, matrixRows, inputs, inputCount, outputs, outputCount, offset, byteCount):
        m = _bytes([list(matrixRows[o])[:inputCount] for o in range(outputCount)]).reshape(outputCount, inputCount)
        check(lib().ecx_code_some_shards(m.ctypes.data, _ptr_array(inputs[:inputCount]), inputCount,
                                         _ptr_array(outputs[:outputCount]), outputCount, offset, byteCount))

    def checkSomeShards(self, matrixRows, inputs, inputCount, toCheck, checkCount, offset, byteCount,
                        tempBuffer=None) -> bool:
        m = _bytes([list(matrixRows[o])[:inputCount] for o in range(checkCount)]).reshape(checkCount, inputCount)
        return bool(check(lib().ecx_check_some_shards(m.ctypes.data, _ptr_array(inputs[:inputCount]), inputCount,
                                                      _ptr_array(toCheck[:checkCount]), checkCount, offset,
                                                      byteCount, None)))


InputOutputByteTableCodingLoop = CodingLoop  # the default loop of ReedSolomon.create (ReedSolomon.java:35)


class InputOutputByteTableCodingLoopSingle:
    """InputOutputByteTableCodingLoopSingle.java:4-20."""

    def codeSomeShards(self, matrixRows, input, index, output, outputIndex, offset, byteCount, isFirstTime):
        rows = [list(r) for r in matrixRows]
        width = max(len(r) for r in rows)
        m = _bytes([r + [0] * (width - len(r)) for r in rows])
        check(lib().ecx_code_single(m.ctypes.data, width, _u8(input).ctypes.data, index, _u8(output).ctypes.data,
                                    outputIndex, offset, byteCount, 1 if isFirstTime else 0))


# ---------------------------------------------------------------- compiled maps
class GfMap:
    """A compiled GF(256) linear map resident on the device (ecx_map)."""

    def __init__(self, handle, owner=None, owned=False):
        self._h = handle
        self._owner = owner  # keeps a codec alive while its maps are used
        self._owned = owned

    @classmethod
    def from_matrix(cls, matrix, in_slot=None, out_slot=None) -> "GfMap":
        m = _bytes(matrix)
        n_out, n_in = m.shape
        ins = None if in_slot is None else np.ascontiguousarray(in_slot, np.int32)
        outs = None if out_slot is None else np.ascontiguousarray(out_slot, np.int32)
        h = ctypes.c_void_p()
        check(lib().ecx_map_create(m.ctypes.data, n_out, n_in, None if ins is None else ins.ctypes.data,
                                   None if outs is None else outs.ctypes.data, ctypes.byref(h)))
        g = cls(h, owned=True)
        g._keep = (ins, outs)
        return g

    def __del__(self):
        if getattr(self, "_owned", False) and self._h and lib is not None:
            lib().ecx_map_destroy(self._h)
            self._h = None

    def info(self):
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib().ecx_map_info(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return {"n_out": a.value, "n_in": b.value, "nnz": c.value}

    def accumulate_batch(self, inp, in_stripe_stride, in_slot_stride, out, out_stripe_stride, out_slot_stride,
                         nstripes, byte_count, stream=None):
        """out ^= M * in (partial sums)."""
        self._check(inp, in_stripe_stride, in_slot_stride, out, out_stripe_stride, out_slot_stride, nstripes,
                    byte_count)
        check(lib().ecx_map_accumulate_batch(self._h, _dev_ptr(inp), in_stripe_stride, in_slot_stride,
                                             _dev_ptr(out), out_stripe_stride, out_slot_stride, nstripes,
                                             byte_count, _stream(stream)))

    def matrix(self):
        """(dense matrix n_out x n_in, in_slot, out_slot) of the composed map."""
        inf = self.info()
        m = np.zeros((inf["n_out"], inf["n_in"]), np.uint8)
        ins = np.zeros(max(1, inf["n_in"]), np.int32)
        outs = np.zeros(max(1, inf["n_out"]), np.int32)
        check(lib().ecx_map_matrix(self._h, m.ctypes.data, ins.ctypes.data, outs.ctypes.data))
        return m, ins[:inf["n_in"]].copy(), outs[:inf["n_out"]].copy()

    def max_slots(self):
        """(largest input slot, largest output slot) of the map (cached)."""
        if getattr(self, "_max_slots", None) is None:
            _, ins, outs = self.matrix()
            self._max_slots = (int(ins.max()) if len(ins) else 0, int(outs.max()) if len(outs) else 0)
        return self._max_slots

    def selftest(self, seed: int = 1) -> None:
        """Host-only check that the compiled plan (tables, tiles, tile-group unions)
        reproduces the dense map (ecx_map_selftest, include/ecx_tune.h)."""
        f = lib().ecx_map_selftest
        f.argtypes, f.restype = [ctypes.c_void_p, ctypes.c_uint64], ctypes.c_int
        check(f(self._h, seed))

    def planes_compile_check(self, accumulate: bool = False) -> int:
        """Generate this map's bit-plane kernel (k_map_planes) and compile it with hiprtc
        for gfx950; returns the code-object size (ecx_map_planes_compile_check)."""
        f = lib().ecx_map_planes_compile_check
        f.argtypes, f.restype = [ctypes.c_void_p, ctypes.c_int], ctypes.c_int
        return check(f(self._h, int(accumulate)))

    def planes_source(self, accumulate: bool = False) -> str:
        """The generated k_map_planes source (ecx_map_planes_source)."""
        f = lib().ecx_map_planes_source
        f.argtypes, f.restype = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int], ctypes.c_int
        n = check(f(self._h, int(accumulate), None, 0))
        buf = ctypes.create_string_buffer(n + 1)
        check(f(self._h, int(accumulate), buf, n + 1))
        return buf.value.decode()

    def plan_stats(self) -> dict:
        """Shape of the compiled plan (ecx_map_plan_stats, include/ecx_tune.h)."""
        f = lib().ecx_map_plan_stats
        f.argtypes, f.restype = [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_int)] * 4, ctypes.c_int
        v = [ctypes.c_int() for _ in range(4)]
        check(f(self._h, *[ctypes.byref(x) for x in v]))
        return dict(zip(["tiles", "entries", "groups", "union_total"], [x.value for x in v]))

    def layout_choice(self, slot_pitch: int, with_times: bool = False):
        """The launch shape "layout_select" kept for the latest selected batch layout of this
        map at an input slot pitch (ecx_map_layout_choice, include/ecx_tune.h): -1 none yet,
        0x100 the static rules' shape, else shape + 8 * stagger (shape 0 256-thread / 4 KiB
        workgroups, 1 skewed chunks, 2 one-wave / 1 KiB workgroups).  with_times: also the
        per-candidate median launch times (ms, -1 unsampled)."""
        f = lib().ecx_map_layout_choice
        f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_float), ctypes.c_int]
        f.restype = ctypes.c_int
        ms = (ctypes.c_float * 8)()
        c = check(f(self._h, int(slot_pitch), ms if with_times else None, 8 if with_times else 0))
        if c == 0x200:
            c = -1  # none chosen yet
        return (c, [round(float(x), 4) for x in ms]) if with_times else c

    def host_plan(self, in_stripe_stride, in_slot_stride, out_stripe_stride, out_slot_stride, nstripes, byte_count):
        """How apply_batch_host would move this batch (ecx_map_host_plan, host-only): a dict of the
        stripes per chunk, the chunk count, the buffer sets, and per chunk the H2D / D2H strided
        copies with the most rows per stripe one copy moves (> 1 where runs are folded or copied in
        3D) and how many of them are 3D."""
        f = lib().ecx_map_host_plan
        f.argtypes = [ctypes.c_void_p] + [ctypes.c_int64] * 6 + [ctypes.c_void_p]
        f.restype = ctypes.c_int
        out = np.zeros(10, np.int64)
        check(f(self._h, in_stripe_stride, in_slot_stride, out_stripe_stride, out_slot_stride, nstripes, byte_count,
                out.ctypes.data))
        keys = ("chunk", "chunks", "buffers", "h2d_copies", "h2d_rows", "d2h_copies", "d2h_rows", "h2d_3d", "d2h_3d",
                "slices")
        return {k: int(v) for k, v in zip(keys, out)}

    def layout_state(self, slot_pitch: int):
        """(state, dropped probes) of that layout's selection (ecx_map_layout_state): state -1
        none yet, 0 exploring, 1 chosen, 2 re-validating, 3 re-validated, 4 contended."""
        f = lib().ecx_map_layout_state
        f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        f.restype = ctypes.c_int
        st, dr = ctypes.c_int(), ctypes.c_int()
        check(f(self._h, int(slot_pitch), ctypes.byref(st), ctypes.byref(dr)))
        return st.value, dr.value

    def _check(self, inp, iss, isl, out, oss, osl, nstripes, nbytes):
        mi, mo = self.max_slots()
        _check_layout(inp, iss, isl, mi, nstripes, nbytes, "input")
        _check_layout(out, oss, osl, mo, nstripes, nbytes, "output")

    def apply_batch(self, inp, in_stripe_stride, in_slot_stride, out, out_stripe_stride, out_slot_stride, nstripes,
                    byte_count, stream=None):
        self._check(inp, in_stripe_stride, in_slot_stride, out, out_stripe_stride, out_slot_stride, nstripes,
                    byte_count)
        check(lib().ecx_map_apply_batch(self._h, _dev_ptr(inp), in_stripe_stride, in_slot_stride, _dev_ptr(out),
                                        out_stripe_stride, out_slot_stride, nstripes, byte_count, _stream(stream)))

    def apply_batch_host(self, inp, in_stripe_stride, in_slot_stride, out, out_stripe_stride, out_slot_stride,
                         nstripes, byte_count):
        """apply_batch over host buffers: pipelined H2D -> kernel -> D2H, synchronous."""
        self._check(inp, in_stripe_stride, in_slot_stride, out, out_stripe_stride, out_slot_stride, nstripes,
                    byte_count)
        check(lib().ecx_map_apply_batch_host(self._h, _host_ptr(inp), in_stripe_stride, in_slot_stride,
                                             _host_ptr(out), out_stripe_stride, out_slot_stride, nstripes,
                                             byte_count))

    def apply_batch_host_devices(self, inp, in_stripe_stride, in_slot_stride, out, out_stripe_stride,
                                 out_slot_stride, nstripes, byte_count, devices):
        """apply_batch_host split over several GPUs (ecx_map_apply_batch_host_devices): device j
        of ``devices`` takes the contiguous stripe range shard_stripes(nstripes, len(devices), j)
        on a worker thread of its own -- or, with fewer stripes than entries, a contiguous range of
        every slot's bytes (4 KiB units); synchronous."""
        self._check(inp, in_stripe_stride, in_slot_stride, out, out_stripe_stride, out_slot_stride, nstripes,
                    byte_count)
        devs = list(devices)
        arr = np.ascontiguousarray(devs + [0], np.int32)  # never a null list: an empty one is ndev 0
        check(lib().ecx_map_apply_batch_host_devices(self._h, _host_ptr(inp), in_stripe_stride, in_slot_stride,
                                                     _host_ptr(out), out_stripe_stride, out_slot_stride, nstripes,
                                                     byte_count, arr.ctypes.data, len(devs)))


# ---------------------------------------------------------------- ReedSolomon.java
class ReedSolomon:
    """ReedSolomon.java: systematic RS over GF(2^8), Vandermonde-derived."""

    def __init__(self, dataShardCount: int, parityShardCount: int, codingLoop=None):
        h = ctypes.c_void_p()
        check(lib().ecx_rs_create(dataShardCount, parityShardCount, ctypes.byref(h)))
        self._h = h
        self.dataShardCount = dataShardCount
        self.parityShardCount = parityShardCount
        self.totalShardCount = dataShardCount + parityShardCount

    @classmethod
    def create(cls, dataShardCount: int, parityShardCount: int) -> "ReedSolomon":
        return cls(dataShardCount, parityShardCount)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().ecx_rs_destroy(self._h)
            self._h = None

    def getDataShardCount(self):
        return self.dataShardCount

    def getParityShardCount(self):
        return self.parityShardCount

    def getTotalShardCount(self):
        return self.totalShardCount

    @property
    def matrix(self) -> np.ndarray:
        out = np.zeros((self.totalShardCount, self.dataShardCount), np.uint8)
        check(lib().ecx_rs_matrix(self._h, out.ctypes.data))
        return out

    @property
    def parityRows(self) -> np.ndarray:
        return self.matrix[self.dataShardCount:]

    @staticmethod
    def _len(shards):
        return len(shards[0]) if len(shards) and shards[0] is not None else 0

    def encodeParity(self, shards, offset: int, byteCount: int) -> None:
        check(lib().ecx_rs_encode_parity(self._h, _ptr_array(shards), len(shards), self._len(shards), offset,
                                         byteCount))

    def encodeParitySingle(self, shard, output, inputIndex, outputIndex, offset, byteCount) -> None:
        check(lib().ecx_rs_encode_parity_single(self._h, _u8(shard).ctypes.data, _u8(output).ctypes.data,
                                                inputIndex, outputIndex, offset, byteCount))

    def isParityCorrect(self, shards, firstByte: int, byteCount: int, tempBuffer=None) -> bool:
        t = None if tempBuffer is None else _u8(tempBuffer).ctypes.data
        tl = 0 if tempBuffer is None else len(tempBuffer)
        return bool(check(lib().ecx_rs_is_parity_correct(self._h, _ptr_array(shards), len(shards),
                                                         self._len(shards), firstByte, byteCount, t, tl)))

    def decodeMissing(self, shards, shardPresent, offset: int, byteCount: int) -> None:
        pres = np.array([1 if p else 0 for p in shardPresent], np.uint8)
        check(lib().ecx_rs_decode_missing(self._h, _ptr_array(shards), pres.ctypes.data, len(shards),
                                          self._len(shards), offset, byteCount))

    def decodeMissingSingle(self, shard, shardIndex, index, shardPresent, outputs, offset, byteCount,
                            isFirst) -> None:
        pres = np.array([1 if p else 0 for p in shardPresent], np.uint8)
        check(lib().ecx_rs_decode_missing_single(self._h, _u8(shard).ctypes.data, shardIndex, index,
                                                 pres.ctypes.data, _ptr_array(outputs), len(outputs), offset,
                                                 byteCount, 1 if isFirst else 0))

    # batched, device-resident
    def encodeParityBatch(self, shards, stripe_stride, shard_stride, nstripes, offset, byteCount, stream=None):
        """encodeParity over nstripes device-resident stripes, in place (ecx_rs_encode_parity_batch)."""
        _check_layout(shards, stripe_stride, shard_stride, self.getTotalShardCount() - 1, nstripes, offset + byteCount,
                      "shards")
        check(lib().ecx_rs_encode_parity_batch(self._h, _dev_ptr(shards), stripe_stride, shard_stride, nstripes,
                                               offset, byteCount, _stream(stream)))

    # ---- the blocked layout contract (ecx_rs_blocked_layout, include/ecx.h)
    def blockedLayout(self, byteCount: int):
        """(block_bytes, full blocks, tail bytes) of the recommended blocked layout of this
        code's stripes for a shard size (ecx_rs_blocked_layout)."""
        out = np.zeros(3, np.int64)
        check(lib().ecx_rs_blocked_layout(self.dataShardCount, self.parityShardCount, byteCount, out.ctypes.data))
        return int(out[0]), int(out[1]), int(out[2])

    def recommendedPitch(self, byteCount: int) -> int:
        """The recommended shard pitch of the plain [stripe][shard][pitch] layout (ecx_rs_recommended_pitch)."""
        out = np.zeros(1, np.int64)
        check(lib().ecx_rs_recommended_pitch(self.dataShardCount, self.parityShardCount, byteCount,
                                             out.ctypes.data))
        return int(out[0])

    def encodeParityBlockedBatch(self, base, nstripes, byteCount, blockBytes=0, stream=None):
        """encodeParity over nstripes stripes in the blocked layout, in place
        (ecx_rs_encode_parity_blocked_batch; blockBytes 0 = the recommended block)."""
        _check_extent(base, nstripes * self.getTotalShardCount() * byteCount, "base")
        check(lib().ecx_rs_encode_parity_blocked_batch(self._h, _dev_ptr(base), nstripes, byteCount, blockBytes,
                                                       _stream(stream)))

    def decodeMissingBlockedBatch(self, base, shardPresent, nstripes, byteCount, blockBytes=0, stream=None):
        """decodeMissing over nstripes stripes in the blocked layout, in place
        (ecx_rs_decode_missing_blocked_batch)."""
        pres = np.array([1 if p else 0 for p in shardPresent], np.uint8)
        if len(pres) != self.getTotalShardCount():
            raise EcxError(-1, "wrong number of shardPresent flags")
        _check_extent(base, nstripes * self.getTotalShardCount() * byteCount, "base")
        check(lib().ecx_rs_decode_missing_blocked_batch(self._h, pres.ctypes.data, _dev_ptr(base), nstripes,
                                                        byteCount, blockBytes, _stream(stream)))

    def encodeParityBlockedBatchHost(self, base, nstripes, byteCount, blockBytes=0):
        """encodeParityBlockedBatch over HOST-memory stripes in the blocked layout, in place
        (ecx_rs_encode_parity_blocked_batch_host: the full blocks, then the tails, each a
        pipelined host batch)."""
        _check_extent(base, nstripes * self.getTotalShardCount() * byteCount, "base")
        check(lib().ecx_rs_encode_parity_blocked_batch_host(self._h, _host_ptr(base), nstripes, byteCount,
                                                            blockBytes))

    def decodeMissingBlockedBatchHost(self, base, shardPresent, nstripes, byteCount, blockBytes=0):
        """decodeMissingBlockedBatch over HOST-memory stripes, in place
        (ecx_rs_decode_missing_blocked_batch_host)."""
        pres = np.array([1 if p else 0 for p in shardPresent], np.uint8)
        if len(pres) != self.getTotalShardCount():
            raise EcxError(-1, "wrong number of shardPresent flags")
        _check_extent(base, nstripes * self.getTotalShardCount() * byteCount, "base")
        check(lib().ecx_rs_decode_missing_blocked_batch_host(self._h, pres.ctypes.data, _host_ptr(base), nstripes,
                                                             byteCount, blockBytes))

    def encodeParityBlockedBatchHostDevices(self, base, nstripes, byteCount, devices, blockBytes=0):
        """encodeParityBlockedBatchHost split over several GPUs of this process
        (ecx_rs_encode_parity_blocked_batch_host_devices): contiguous stripe ranges, one worker
        thread and pipe per device entry."""
        _check_extent(base, nstripes * self.getTotalShardCount() * byteCount, "base")
        devs = list(devices)
        arr = np.ascontiguousarray(devs + [0], np.int32)  # never a null list: an empty one is ndev 0
        check(lib().ecx_rs_encode_parity_blocked_batch_host_devices(self._h, _host_ptr(base), nstripes, byteCount,
                                                                    blockBytes, arr.ctypes.data, len(devs)))

    def decodeMissingBlockedBatchHostDevices(self, base, shardPresent, nstripes, byteCount, devices, blockBytes=0):
        """decodeMissingBlockedBatchHost split over several GPUs of this process
        (ecx_rs_decode_missing_blocked_batch_host_devices)."""
        pres = np.array([1 if p else 0 for p in shardPresent], np.uint8)
        if len(pres) != self.getTotalShardCount():
            raise EcxError(-1, "wrong number of shardPresent flags")
        _check_extent(base, nstripes * self.getTotalShardCount() * byteCount, "base")
        devs = list(devices)
        arr = np.ascontiguousarray(devs + [0], np.int32)
        check(lib().ecx_rs_decode_missing_blocked_batch_host_devices(self._h, pres.ctypes.data, _host_ptr(base),
                                                                     nstripes, byteCount, blockBytes,
                                                                     arr.ctypes.data, len(devs)))

    def isParityCorrectBatch(self, shards, stripe_stride, shard_stride, nstripes, firstByte, byteCount, verdict,
                             stream=None) -> None:
        """isParityCorrect over nstripes device-resident stripes, read-only
        (ecx_rs_is_parity_correct_batch): the device uint8 array ``verdict`` (nstripes bytes)
        receives 1 for each stripe whose parity is correct over [firstByte, firstByte +
        byteCount), else 0.  Enqueued on ``stream``; read verdict after synchronising."""
        _check_layout(shards, stripe_stride, shard_stride, self.getTotalShardCount() - 1, nstripes,
                      firstByte + byteCount, "shards")
        _check_layout(verdict, 1, 0, 0, nstripes, 1, "verdict")
        check(lib().ecx_rs_is_parity_correct_batch(self._h, _dev_ptr(shards), stripe_stride, shard_stride, nstripes,
                                                   firstByte, byteCount, _dev_ptr(verdict), _stream(stream)))

    def isParityCorrectBatchHost(self, shards, stripe_stride, shard_stride, nstripes, firstByte, byteCount,
                                 verdict) -> None:
        """isParityCorrectBatch over HOST-memory stripes (ecx_rs_is_parity_correct_batch_host):
        chunks of stripes are pipelined H2D through the read-only check kernel and only the
        verdict bytes come back into the host uint8 array ``verdict`` (nstripes bytes)."""
        _check_layout(shards, stripe_stride, shard_stride, self.getTotalShardCount() - 1, nstripes,
                      firstByte + byteCount, "shards")
        _check_layout(verdict, 1, 0, 0, nstripes, 1, "verdict")
        check(lib().ecx_rs_is_parity_correct_batch_host(self._h, _host_ptr(shards), stripe_stride, shard_stride,
                                                        nstripes, firstByte, byteCount, _host_ptr(verdict)))

    def isParityCorrectBatchHostDevices(self, shards, stripe_stride, shard_stride, nstripes, firstByte, byteCount,
                                        verdict, devices) -> None:
        """isParityCorrectBatchHost split over several GPUs of this process
        (ecx_rs_is_parity_correct_batch_host_devices): contiguous stripe ranges, one worker
        thread and pipe per device entry."""
        _check_layout(shards, stripe_stride, shard_stride, self.getTotalShardCount() - 1, nstripes,
                      firstByte + byteCount, "shards")
        _check_layout(verdict, 1, 0, 0, nstripes, 1, "verdict")
        devs = list(devices)
        arr = np.ascontiguousarray(devs + [0], np.int32)  # never a null list: an empty one is ndev 0
        check(lib().ecx_rs_is_parity_correct_batch_host_devices(self._h, _host_ptr(shards), stripe_stride,
                                                                shard_stride, nstripes, firstByte, byteCount,
                                                                _host_ptr(verdict), arr.ctypes.data, len(devs)))

    def decodeMissingBatch(self, shards, shardPresent, stripe_stride, shard_stride, nstripes, offset, byteCount,
                           stream=None):
        """decodeMissing over nstripes device-resident stripes, in place (ecx_rs_decode_missing_batch)."""
        pres = np.array([1 if p else 0 for p in shardPresent], np.uint8)
        if len(pres) != self.getTotalShardCount():
            raise EcxError(-1, "wrong number of shardPresent flags")
        _check_layout(shards, stripe_stride, shard_stride, self.getTotalShardCount() - 1, nstripes, offset + byteCount,
                      "shards")
        check(lib().ecx_rs_decode_missing_batch(self._h, pres.ctypes.data, _dev_ptr(shards), stripe_stride,
                                                shard_stride, nstripes, offset, byteCount, _stream(stream)))

    def decodePartialBatch(self, shardPresent, shardIndex, inp, in_stripe_stride, acc, acc_stripe_stride,
                           acc_row_stride, nstripes, byteCount, isFirst, stream=None):
        """Batched decodeMissingSingle for every missing shard (data and parity)."""
        pres = np.array([1 if p else 0 for p in shardPresent], np.uint8)
        _check_layout(inp, in_stripe_stride, 0, 0, nstripes, byteCount, "input")
        _check_layout(acc, acc_stripe_stride, acc_row_stride, int((pres == 0).sum()) - 1, nstripes, byteCount, "acc")
        check(lib().ecx_rs_decode_partial_batch(self._h, pres.ctypes.data, shardIndex, _dev_ptr(inp),
                                                in_stripe_stride, _dev_ptr(acc), acc_stripe_stride, acc_row_stride,
                                                nstripes, byteCount, 1 if isFirst else 0, _stream(stream)))

    def encodePartialBatch(self, inputIndex, inp, in_stripe_stride, acc, acc_stripe_stride, acc_row_stride,
                           nstripes, byteCount, isFirst, stream=None):
        """Batched encodeParitySingle into every parity row."""
        _check_layout(inp, in_stripe_stride, 0, 0, nstripes, byteCount, "input")
        _check_layout(acc, acc_stripe_stride, acc_row_stride, self.parityShardCount - 1, nstripes, byteCount, "acc")
        check(lib().ecx_rs_encode_partial_batch(self._h, inputIndex, _dev_ptr(inp), in_stripe_stride,
                                                _dev_ptr(acc), acc_stripe_stride, acc_row_stride, nstripes,
                                                byteCount, 1 if isFirst else 0, _stream(stream)))

    def encode_map(self) -> GfMap:
        h = ctypes.c_void_p()
        check(lib().ecx_rs_encode_map(self._h, ctypes.byref(h)))
        return GfMap(h, owner=self)

    def decode_map(self, shardPresent) -> GfMap:
        pres = np.array([1 if p else 0 for p in shardPresent], np.uint8)
        h = ctypes.c_void_p()
        check(lib().ecx_rs_decode_map(self._h, pres.ctypes.data, ctypes.byref(h)))
        return GfMap(h, owner=self)


# ---------------------------------------------------------------- Clay
class ClayCodeUtil:
    """ClayCodeErasureDecodingStep.ClayCodeUtil (:676-944) index arithmetic."""

    def __init__(self, erasedIndexes, numDataUnits, numParityUnits):
        self.q = numParityUnits
        self.t = (numParityUnits + numDataUnits) // numParityUnits
        self.erasedIndexes = list(erasedIndexes)
        self.subPacketSize = self.q ** self.t

    def getSubPacketSize(self):
        return self.subPacketSize

    def getZVector(self, z):
        v = [0] * self.t
        for i in range(self.t - 1, -1, -1):
            v[i] = z % self.q
            z //= self.q
        return v

    def getZ(self, v):
        z = 0
        for x in v:
            z = z * self.q + x
        return z

    def getNodeIndex(self, x, y):
        return x + self.q * y

    def getNodeCoordinates(self, i):
        return [i % self.q, i // self.q]

    def getCouplePlaneIndex(self, coordinates, z):
        v = self.getZVector(z)
        v[coordinates[1]] = coordinates[0]
        return self.getZ(v)

    def getHelperPlanesIndexes(self, k):
        x, y = self.getNodeCoordinates(k)
        return [z for z in range(self.subPacketSize) if self.getZVector(z)[y] == x]


class ClayCodeErasureDecodingStep:
    """new ClayCodeErasureDecodingStep(erasedIndexes, RS(2,2), RS(k,m)) (:43-51)."""

    def __init__(self, erasedIndexes, numDataUnits: int, numParityUnits: int, virtualUnits: int = 0,
                 isTest: bool = False):
        """virtualUnits > 0: shortened code, Clay(k+v, m) with v virtual zero data nodes
        (e.g. Clay(10,4) = ClayCodeErasureDecodingStep(e, 10, 4, virtualUnits=2)).  isTest: the
        reference run with -DisTest=true (decodeDecoupledPlane :571-581, ecx_clay_create_ex)."""
        er = np.ascontiguousarray(list(erasedIndexes), np.int32)
        h = ctypes.c_void_p()
        if isTest:
            check(lib().ecx_clay_create_ex(numDataUnits, numParityUnits, virtualUnits, er.ctypes.data, len(er),
                                           1, ctypes.byref(h)))
        elif virtualUnits:
            check(lib().ecx_clay_create_shortened(numDataUnits, numParityUnits, virtualUnits, er.ctypes.data,
                                                  len(er), ctypes.byref(h)))
        else:
            check(lib().ecx_clay_create(numDataUnits, numParityUnits, er.ctypes.data, len(er), ctypes.byref(h)))
        self.isTest = isTest
        self._h = h
        self.erasedIndexes = list(erasedIndexes)
        self.numDataUnits, self.numParityUnits = numDataUnits, numParityUnits
        self.numTotalUnits = numDataUnits + numParityUnits
        q, t, a = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib().ecx_clay_geometry(h, ctypes.byref(q), ctypes.byref(t), ctypes.byref(a)))
        self.q, self.t, self.subPacketSize = q.value, t.value, a.value
        self.virtualUnits = virtualUnits
        self.util = ClayCodeUtil(erasedIndexes, numDataUnits + virtualUnits, numParityUnits)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().ecx_clay_destroy(self._h)
            self._h = None

    def rtcCompileCheck(self) -> int:
        """Build this single-node repair's per-helper-plane program (checked against the
        composed reference map), generate its kernel and compile it with hiprtc for
        gfx950; returns the code-object size (ecx_clay_rtc_compile_check, include/ecx_tune.h)."""
        f = lib().ecx_clay_rtc_compile_check
        f.argtypes, f.restype = [ctypes.c_void_p], ctypes.c_int
        return check(f(self._h))

    def rtcSource(self) -> str:
        """The generated k_clay_repair source (ecx_clay_rtc_source)."""
        f = lib().ecx_clay_rtc_source
        f.argtypes, f.restype = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int], ctypes.c_int
        n = check(f(self._h, None, 0))
        buf = ctypes.create_string_buffer(n + 1)
        check(f(self._h, buf, n + 1))
        return buf.value.decode()

    def getHelperPlanesIndexes(self, erasedIndex: int):
        out = np.zeros(self.subPacketSize, np.int32)
        n = check(lib().ecx_clay_helper_planes(self._h, erasedIndex, out.ctypes.data))
        return [int(x) for x in out[:n]]

    def performCoding(self, inputs, outputs, bufSize: Optional[int] = None) -> None:
        """inputs: n*alpha (plane-major, None = absent); outputs: |E|*alpha arrays.
        Entries may be numpy arrays, None, ECChunk or ECBlock (ECChunk.toBuffers)."""
        inputs, outputs = _buffers(inputs), _buffers(outputs)
        if len(inputs) != self.numTotalUnits * self.subPacketSize:
            raise EcxError(-1, "Invalid inputs length")
        if len(outputs) != len(self.erasedIndexes) * self.subPacketSize:
            raise EcxError(-1, "Invalid outputs length")
        if bufSize is None:
            first = next((b for b in inputs if b is not None), None)
            if first is None:
                raise EcxError(-1, "Invalid inputs are found, all being null")
            bufSize = len(first)
        check(lib().ecx_clay_perform_coding(self._h, _ptr_array(inputs), _ptr_array(outputs), bufSize))

    def doDecodeSingleHelper(self, helperCoupledPlanes, helperIndex: int, outputs, erasedIndex: int,
                             bufSize: int) -> None:
        """doDecodeSingle overload 2 (:225-282): helperCoupledPlanes[nh][n], outputs[alpha]."""
        flat = [b for row in helperCoupledPlanes for b in row]
        check(lib().ecx_clay_decode_single_helper(self._h, _ptr_array(flat), helperIndex, _ptr_array(outputs),
                                                  erasedIndex, bufSize))

    def map(self) -> GfMap:
        h = ctypes.c_void_p()
        check(lib().ecx_clay_map(self._h, ctypes.byref(h)))
        return GfMap(h, owner=self)

    def _check_batch(self, inp, iss, isl, out, oss, osl, nstripes, nbytes):
        if not self.erasedIndexes:
            return
        if getattr(self, "_map", None) is None:
            self._map = self.map()
        self._map._check(inp, iss, isl, out, oss, osl, nstripes, nbytes)

    def performCodingBatch(self, inp, in_stripe_stride, in_sub_stride, out, out_stripe_stride, out_sub_stride,
                           nstripes, bufSize, stream=None) -> None:
        self._check_batch(inp, in_stripe_stride, in_sub_stride, out, out_stripe_stride, out_sub_stride, nstripes,
                          bufSize)
        check(lib().ecx_clay_perform_coding_batch(self._h, _dev_ptr(inp), in_stripe_stride, in_sub_stride,
                                                  _dev_ptr(out), out_stripe_stride, out_sub_stride, nstripes,
                                                  bufSize, _stream(stream)))

    def performCodingBatchHost(self, inp, in_stripe_stride, in_sub_stride, out, out_stripe_stride, out_sub_stride,
                               nstripes, bufSize) -> None:
        """performCodingBatch over host-memory stripes (ecx_clay_perform_coding_batch_host)."""
        self._check_batch(inp, in_stripe_stride, in_sub_stride, out, out_stripe_stride, out_sub_stride, nstripes,
                          bufSize)
        check(lib().ecx_clay_perform_coding_batch_host(self._h, _host_ptr(inp), in_stripe_stride, in_sub_stride,
                                                       _host_ptr(out), out_stripe_stride, out_sub_stride, nstripes,
                                                       bufSize))

    def performCodingBatchHostDevices(self, inp, in_stripe_stride, in_sub_stride, out, out_stripe_stride,
                                      out_sub_stride, nstripes, bufSize, devices) -> None:
        """performCodingBatchHost split over several GPUs of this process
        (ecx_clay_perform_coding_batch_host_devices): contiguous stripe ranges (byte ranges of
        every sub-chunk when there are fewer stripes than entries), one worker thread and pipe per
        device entry."""
        self._check_batch(inp, in_stripe_stride, in_sub_stride, out, out_stripe_stride, out_sub_stride, nstripes,
                          bufSize)
        devs = list(devices)
        arr = np.ascontiguousarray(devs + [0], np.int32)  # never a null list: an empty one is ndev 0
        check(lib().ecx_clay_perform_coding_batch_host_devices(self._h, _host_ptr(inp), in_stripe_stride,
                                                               in_sub_stride, _host_ptr(out), out_stripe_stride,
                                                               out_sub_stride, nstripes, bufSize, arr.ctypes.data,
                                                               len(devs)))


class JavaRandom:
    """java.util.Random (JDK specification), for ClayCode.getInputs."""

    def __init__(self, seed: int):
        self.seed = (seed ^ 0x5DEECE66D) & ((1 << 48) - 1)

    def _next(self, bits):
        self.seed = (self.seed * 0x5DEECE66D + 0xB) & ((1 << 48) - 1)
        r = self.seed >> (48 - bits)
        return r - (1 << bits) if r >= 1 << (bits - 1) else r

    def nextInt(self):
        return self._next(32)

    def nextBytes(self, n: int) -> np.ndarray:
        out = np.zeros(n, np.uint8)
        i = 0
        while i < n:
            rnd = self.nextInt() & 0xFFFFFFFF
            for _ in range(min(4, n - i)):
                out[i] = rnd & 0xFF
                rnd >>= 8
                i += 1
        return out


class ClayCode:
    """ClayCode.java facade: RS(2,2) pair transform + RS(k,m) per plane.
    Buffers are numpy arrays inside ECChunk/ECBlock wrappers, as in the reference."""

    def __init__(self, numDataUnits, numParityUnits, blockSize, erasedIndexes):
        self.numDataUnits, self.numParityUnits, self.blockSize = numDataUnits, numParityUnits, blockSize
        self.erasedIndexes = list(erasedIndexes)
        self.erasureDecodingStep = ClayCodeErasureDecodingStep(erasedIndexes, numDataUnits, numParityUnits)
        self.clayCodeUtil = ClayCodeUtil(erasedIndexes, numDataUnits, numParityUnits)

    def performCoding(self, inputs, outputs):
        """ClayCode.performCoding (:43-45) -> ClayCodeErasureDecodingStep.performCoding."""
        self.erasureDecodingStep.performCoding(inputs, outputs, self.blockSize)

    def getInputs(self):
        """ClayCode.getInputs (ClayCode.java:47-77): one Random(123456), nextBytes per data
        sub-chunk in flat order k; sub-chunk k is data iff k % n < numDataUnits."""
        n = self.numDataUnits + self.numParityUnits
        a = self.clayCodeUtil.getSubPacketSize()
        r = JavaRandom(123456)
        out = [None] * (n * a)
        counter = 0
        for i in range(n):
            for j in range(a):
                k = i * a + j
                if counter < self.numDataUnits:
                    out[k] = ECBlock(ECChunk(r.nextBytes(self.blockSize)), False, False)
                else:
                    out[k] = ECBlock(ECChunk(None), True, True)
                counter = (counter + 1) % n
        return out

    def getOutputs(self):
        """ClayCode.getOutputs (:79-87)."""
        return [ECBlock(ECChunk(np.zeros(self.blockSize, np.uint8)), True, True)
                for _ in range(len(self.erasedIndexes) * self.clayCodeUtil.getSubPacketSize())]

    def encode(self, inputs, outputs):
        """ClayCode.encode (:89-99): performCoding with erasedIndexes = the parity nodes;
        returns [inputChunks, outputChunks]."""
        step = ClayCodeErasureDecodingStep(self.erasedIndexes, self.numDataUnits, self.numParityUnits)
        ic, oc = self.getChunks(inputs), self.getChunks(outputs)
        step.performCoding(ic, oc, self.blockSize)
        return [ic, oc]

    def getChunks(self, blocks):
        """ClayCode.getChunks (:168-177)."""
        return [None if b is None else b.getChunk() for b in blocks]

    def getTestOutputs(self, erasedIndexesSize: int):
        """ClayCode.getTestOutputs (:157-166)."""
        return [ECBlock(ECChunk(np.zeros(self.blockSize, np.uint8)), False, True)
                for _ in range(erasedIndexesSize * self.clayCodeUtil.getSubPacketSize())]

    def getTestInputs(self, inputChunks, outputChunks, testErasedIndexes, blockId: str = "LP", write_dir=None):
        """ClayCode.getTestInputs (:101-155), restated faithfully -- including the
        reference's index quirk (SURVEY.md A.2 bug B1): the outer loop variable is
        treated as the node although the flat index a*alpha+b is plane-major, so
        the zeroed sub-chunks are not the erased node's for every e.  With
        write_dir, also writes the per-sub-chunk files "<blockId> <node> <plane>"
        (and "ORIGINAL ..." for erased nodes) as the reference does in its CWD."""
        n = self.numDataUnits + self.numParityUnits
        a = self.clayCodeUtil.getSubPacketSize()
        erased = list(testErasedIndexes)
        ib, ob = ECChunk.toBuffers(inputChunks), ECChunk.toBuffers(outputChunks)
        test, k = [None] * (n * a), 0
        for aa in range(n):
            for b in range(a):
                i = aa * a + b
                if aa not in erased:
                    if ib[i] is not None:
                        buf = np.array(ib[i], np.uint8)
                    else:
                        buf = np.array(ob[k], np.uint8)
                        k += 1
                    test[i] = ECBlock(ECChunk(buf), False, True)
                else:
                    if ib[i] is None:
                        k += 1
                    test[i] = ECBlock(ECChunk(np.zeros(self.blockSize, np.uint8)), False, True)
        if write_dir is not None:
            k = 0
            for i in range(a):
                for j in range(n):
                    idx = i * n + j
                    data = ib[idx] if ib[idx] is not None else ob[k]
                    if ib[idx] is None:
                        k += 1
                    write_subchunk(write_dir, blockId, j, i, data, original=j in erased)
        return test


class ClayCodeHelper:
    """ClayCodeHelper.kt:11-76 -- coordinator-side single repair, one helper plane at a time
    (doDecodeSingle overload 2)."""

    def __init__(self, NUM_DATA_UNITS, NUM_PARITY_UNITS, SUBPACKET_SIZE, inputs):
        self.k, self.m, self.alpha = NUM_DATA_UNITS, NUM_PARITY_UNITS, SUBPACKET_SIZE
        self.n = NUM_DATA_UNITS + NUM_PARITY_UNITS
        self.inputs = _buffers(inputs)

    def getHelperPlanesAndDecode(self, util, blockId, outputs, erasedIndex, bufSize, isDirect=False):
        """outputs: [alpha][|E|] arrays (|E| = 1)."""
        step = ClayCodeErasureDecodingStep([erasedIndex], self.k, self.m)
        hidx = util.getHelperPlanesIndexes(erasedIndex)
        rows = [[self.inputs[z * self.n + j] for j in range(self.n)] for z in hidx]
        flat_out = [outputs[z][0] for z in range(self.alpha)]
        for i in range(len(hidx)):
            step.doDecodeSingleHelper(rows, i, flat_out, erasedIndex, bufSize)


# ---------------------------------------------------------------- per-sub-chunk files
def _subchunk_path(directory, blockId, node, plane, original=False):
    import os
    return os.path.join(str(directory), f"{'ORIGINAL ' if original else ''}{blockId} {node} {plane}")


def write_subchunk(directory, blockId: str, node: int, plane: int, data, original: bool = False) -> str:
    """The reference's on-disk unit: one file "<blockId> <node> <plane>" holding exactly
    B bytes (ClayCode.java:140-152, ClayCodeNode.kt:105,147,245,257)."""
    path = _subchunk_path(directory, blockId, node, plane, original)
    np.asarray(data, np.uint8).tofile(path)
    return path


def read_subchunk(directory, blockId: str, node: int, plane: int, blockSize: Optional[int] = None,
                  original: bool = False) -> np.ndarray:
    data = np.fromfile(_subchunk_path(directory, blockId, node, plane, original), dtype=np.uint8)
    return data if blockSize is None else data[:blockSize].copy()


# ---------------------------------------------------------------- LRC (lrc/)
class LRCErasureUtil:
    N = 16
    K = 12
    R = 3


class LRCErasureCode:
    """LRCErasureCode.kt:5-9 -- RS(R,1) local parity (coefficients [1,1,1]: XOR)."""

    def __init__(self):
        self.rs = ReedSolomon.create(LRCErasureUtil.R, 1)

    def encodeParitySingle(self, shard, output, index, blockSize):
        self.rs.encodeParitySingle(shard, output, index, 0, 0, blockSize)

    @staticmethod
    def map(blockPresent=None) -> GfMap:
        """The composed LRC map over the 16 blocks: encode (None) or decode (ecx_lrc_map)."""
        h = ctypes.c_void_p()
        pres = None if blockPresent is None else np.array([1 if p else 0 for p in blockPresent], np.uint8)
        check(lib().ecx_lrc_map(None if pres is None else pres.ctypes.data, ctypes.byref(h)))
        return GfMap(h)

    @staticmethod
    def encodeBatch(stripes, stripe_stride, block_stride, nstripes, blockSize, stream=None) -> None:
        """All group parities of device-resident [S][16][B] stripes, in place (ecx_lrc_encode_batch)."""
        LRCErasureCode.map()._check(stripes, stripe_stride, block_stride, stripes, stripe_stride, block_stride,
                                    nstripes, blockSize)
        check(lib().ecx_lrc_encode_batch(_dev_ptr(stripes), stripe_stride, block_stride, nstripes, blockSize,
                                         _stream(stream)))

    @staticmethod
    def decodeBatch(stripes, stripe_stride, block_stride, blockPresent, nstripes, blockSize, stream=None) -> None:
        """Rebuild the non-present blocks of device-resident stripes in place (ecx_lrc_decode_batch)."""
        pres = np.array([1 if p else 0 for p in blockPresent], np.uint8)
        if pres.all():
            return
        LRCErasureCode.map(blockPresent)._check(stripes, stripe_stride, block_stride, stripes, stripe_stride,
                                                block_stride, nstripes, blockSize)
        check(lib().ecx_lrc_decode_batch(_dev_ptr(stripes), stripe_stride, block_stride, pres.ctypes.data, nstripes,
                                         blockSize, _stream(stream)))


def lrc_encode(data: np.ndarray):
    """LRCErasureCodeExample.encode (:30-57): K blocks -> N blocks (group g: 3 data + parity)."""
    U = LRCErasureUtil
    block = len(data) // U.K
    rs = ReedSolomon.create(U.R, 1)
    out, pos = [], 0
    for _ in range(U.K // U.R):
        shards = []
        for _ in range(U.R):
            shards.append(np.ascontiguousarray(data[pos:pos + block], np.uint8).copy())
            pos += block
        shards.append(np.zeros(block, np.uint8))
        rs.encodeParity(shards, 0, block)
        out.extend(shards)
    return out


def lrc_encode_using_single(data: np.ndarray):
    """LRCErasureCodeExample.encodeUsingSingle (:59-90)."""
    U = LRCErasureUtil
    block = len(data) // U.K
    code = LRCErasureCode()
    out, pos = [], 0
    for _ in range(U.K // U.R):
        shards = []
        for _ in range(U.R):
            shards.append(np.ascontiguousarray(data[pos:pos + block], np.uint8).copy())
            pos += block
        acc = np.zeros(block, np.uint8)
        for idx in range(U.R):
            code.rs.encodeParitySingle(shards[idx], acc, idx, 0, 0, block)
        shards.append(acc)
        out.extend(shards)
    return out


def lrc_decode(blocks, missingIndices: Iterable[int], blockSize: int):
    """LRCErasureCodeExample.decode (:92-131): returns (file bytes, repaired blocks)."""
    U = LRCErasureUtil
    missing = set(missingIndices)
    rs = ReedSolomon.create(U.R, 1)
    shards = [np.array(blocks[i], np.uint8) if (i not in missing and blocks[i] is not None)
              else np.zeros(blockSize, np.uint8) for i in range(U.N)]
    for g in range(U.K // U.R):
        lo = g * (U.R + 1)
        present = [(lo + j) not in missing for j in range(U.R + 1)]
        rs.decodeMissing(shards[lo:lo + U.R + 1], present, 0, blockSize)
    data = [shards[i] for i in range(U.N) if i == 0 or (i + 1) % (U.R + 1) != 0]
    return np.concatenate(data), shards


# ---------------------------------------------------------------- SampleEncoder / SampleDecoder
def sample_encode(file_bytes: np.ndarray, data_shards: int = 4, parity_shards: int = 2):
    """SampleEncoder.java:54-83: [int32 BE length][file][zero pad] -> data shards + RS parity."""
    size = len(file_bytes)
    shard = (size + 4 + data_shards - 1) // data_shards
    allb = np.zeros(shard * data_shards, np.uint8)
    allb[:4] = np.frombuffer(int(size).to_bytes(4, "big"), np.uint8)
    allb[4:4 + size] = file_bytes
    shards = [allb[i * shard:(i + 1) * shard].copy() for i in range(data_shards)]
    shards += [np.zeros(shard, np.uint8) for _ in range(parity_shards)]
    ReedSolomon.create(data_shards, parity_shards).encodeParity(shards, 0, shard)
    return shards


def sample_decode(shards: Sequence[Optional[np.ndarray]], data_shards: int = 4, parity_shards: int = 2):
    """SampleDecoder.java:34-98: decodeMissing, then strip the length header."""
    present = [s is not None for s in shards]
    if sum(present) < data_shards:
        raise EcxError(-2, "Not enough shards present")
    size = next(len(s) for s in shards if s is not None)
    work = [np.array(s, np.uint8) if s is not None else np.zeros(size, np.uint8) for s in shards]
    ReedSolomon.create(data_shards, parity_shards).decodeMissing(work, present, 0, size)
    allb = np.concatenate(work[:data_shards])
    n = int.from_bytes(allb[:4].tobytes(), "big")
    return allb[4:4 + n].copy(), work
