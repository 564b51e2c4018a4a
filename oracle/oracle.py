"""TEST INFRASTRUCTURE ONLY -- ctypes front end of the C restatement of the
reference's JVM CPU path (oracle/ecx_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline -- never
as the thing measured or shipped.  The product library
(repair-pipelining_amd/) does not import it.

Mirrors the reference entry points:
  * Galois.java          -> gf_multiply / gf_divide / gf_exp / log_table / exp_table / mul_table
  * Matrix.java          -> matrix_times / matrix_invert
  * ReedSolomon.java     -> ReedSolomon (encode_parity, encode_parity_single,
                            is_parity_correct, decode_missing, decode_missing_single)
  * ClayCodeErasureDecodingStep.java / ClayCode.java / ClayCodeHelper.kt -> Clay
  * LRCErasureCodeExample.kt -> lrc_encode / lrc_encode_using_single / lrc_decode
  * SampleEncoder.java / SampleDecoder.java -> sample_encode / sample_decode
  * java.util.Random     -> JavaRandom
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "liborc.so"

ORC_ERRORS = {
    -1: "IllegalArgumentException",
    -2: "IllegalArgumentException: Not enough shards present",
    -3: "IllegalArgumentException: Matrix is singular",
    -4: "IllegalArgumentException: too many shards - max is 256",
    -5: "ArrayIndexOutOfBoundsException",
    -6: "NullPointerException",
    -7: "OutOfMemoryError",
}


class OracleError(Exception):
    def __init__(self, code: int):
        self.code = code
        super().__init__(f"oracle status {code}: {ORC_ERRORS.get(code, '?')}")


def build() -> Path:
    """Compile liborc.so with gcc (oracle/Makefile)."""
    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
    return _LIB_PATH


def _load():
    if not _LIB_PATH.exists():
        build()
    lib = ctypes.CDLL(str(_LIB_PATH))
    P = ctypes.c_void_p
    I = ctypes.c_int
    PP = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "orc_jrandom_init": (None, [P, ctypes.c_int64]),
        "orc_jrandom_next_int": (ctypes.c_int32, [P]),
        "orc_jrandom_next_int_bound": (ctypes.c_int32, [P, ctypes.c_int32]),
        "orc_jrandom_next_bytes": (None, [P, P, I]),
        "orc_gen_log_table": (I, [I, P]),
        "orc_gen_exp_table": (None, [P, P]),
        "orc_log_table": (P, []),
        "orc_exp_table": (P, []),
        "orc_mul_table": (P, []),
        "orc_gf_multiply": (ctypes.c_uint8, [ctypes.c_uint8, ctypes.c_uint8]),
        "orc_gf_divide": (I, [ctypes.c_uint8, ctypes.c_uint8]),
        "orc_gf_exp": (ctypes.c_uint8, [ctypes.c_uint8, I]),
        "orc_all_possible_polynomials": (I, [P]),
        "orc_matrix_times": (I, [P, I, I, P, I, I, P]),
        "orc_matrix_invert": (I, [P, I, P]),
        "orc_code_some_shards": (None, [PP, PP, I, PP, I, I, I]),
        "orc_check_some_shards": (I, [PP, PP, I, PP, I, I, I, P]),
        "orc_code_single": (None, [PP, P, I, P, I, I, I, I]),
        "orc_rs_create": (I, [I, I, ctypes.POINTER(P)]),
        "orc_rs_free": (None, [P]),
        "orc_rs_matrix": (None, [P, P]),
        "orc_rs_encode_parity": (I, [P, PP, I, I, I, I]),
        "orc_rs_encode_parity_single": (I, [P, P, P, I, I, I, I]),
        "orc_rs_is_parity_correct": (I, [P, PP, I, I, I, I, P, I]),
        "orc_rs_decode_missing": (I, [P, PP, P, I, I, I, I]),
        "orc_rs_decode_missing_single": (I, [P, P, I, I, P, PP, I, I, I, I]),
        "orc_clay_create": (I, [I, I, P, I, ctypes.POINTER(P)]),
        "orc_clay_create_ex": (I, [I, I, P, I, I, ctypes.POINTER(P)]),
        "orc_clay_free": (None, [P]),
        "orc_clay_alpha": (I, [P]),
        "orc_clay_q": (I, [P]),
        "orc_clay_t": (I, [P]),
        "orc_clay_helper_planes": (I, [P, I, P]),
        "orc_clay_perform_coding": (I, [P, PP, PP, I]),
        "orc_clay_decode_single_helper": (I, [P, PP, I, PP, I, I]),
        "orc_clay_get_inputs": (I, [I, I, I, P, P]),
        "orc_bench_clay_repair": (I, [I, I, I, I, PP, I, I, ctypes.c_double,
                                      ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double)]),
        "orc_bench_run": (I, [I, I, I, P, I, I, P, I, I, I, ctypes.c_double,
                              ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def _ptrs(arrays):
    arr = (ctypes.c_void_p * max(1, len(arrays)))()
    for i, a in enumerate(arrays):
        arr[i] = None if a is None else a.ctypes.data
    return arr


def _check(st: int) -> int:
    if st < 0:
        raise OracleError(st)
    return st


# ---------------------------------------------------------------- Random
class JavaRandom:
    """java.util.Random restated (JDK spec)."""

    class _S(ctypes.Structure):
        _fields_ = [("seed", ctypes.c_uint64)]

    def __init__(self, seed: int):
        self._s = JavaRandom._S()
        lib().orc_jrandom_init(ctypes.byref(self._s), seed)

    def next_int(self, bound: int | None = None) -> int:
        if bound is None:
            return lib().orc_jrandom_next_int(ctypes.byref(self._s))
        return _check(lib().orc_jrandom_next_int_bound(ctypes.byref(self._s), bound))

    def next_bytes(self, n: int) -> np.ndarray:
        out = np.zeros(n, dtype=np.uint8)
        lib().orc_jrandom_next_bytes(ctypes.byref(self._s), _ptr(out), n)
        return out


# ---------------------------------------------------------------- Galois
def log_table() -> np.ndarray:
    p = lib().orc_log_table()
    return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_int16)), (256,)).copy()


def exp_table() -> np.ndarray:
    p = lib().orc_exp_table()
    return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), (510,)).copy()


def mul_table() -> np.ndarray:
    p = lib().orc_mul_table()
    return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), (256, 256)).copy()


def gen_log_table(poly: int):
    out = np.zeros(256, dtype=np.int16)
    st = lib().orc_gen_log_table(poly, _ptr(out))
    return None if st else out


def gen_exp_table(log: np.ndarray) -> np.ndarray:
    log = np.ascontiguousarray(log, dtype=np.int16)
    out = np.zeros(510, dtype=np.uint8)
    lib().orc_gen_exp_table(_ptr(log), _ptr(out))
    return out


def all_possible_polynomials():
    out = np.zeros(256, dtype=np.int32)
    n = lib().orc_all_possible_polynomials(_ptr(out))
    return [int(x) for x in out[:n]]


def gf_multiply(a: int, b: int) -> int:
    return int(lib().orc_gf_multiply(a & 0xFF, b & 0xFF))


def gf_divide(a: int, b: int) -> int:
    return _check(lib().orc_gf_divide(a & 0xFF, b & 0xFF))


def gf_exp(a: int, n: int) -> int:
    return int(lib().orc_gf_exp(a & 0xFF, n))


# ---------------------------------------------------------------- Matrix
def matrix_times(a, b) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint8)
    b = np.ascontiguousarray(b, dtype=np.uint8)
    out = np.zeros((a.shape[0], b.shape[1]), dtype=np.uint8)
    _check(lib().orc_matrix_times(_ptr(a), a.shape[0], a.shape[1], _ptr(b), b.shape[0], b.shape[1], _ptr(out)))
    return out


def matrix_invert(m) -> np.ndarray:
    m = np.ascontiguousarray(m, dtype=np.uint8)
    out = np.zeros_like(m)
    _check(lib().orc_matrix_invert(_ptr(m), m.shape[0], _ptr(out)))
    return out


# ---------------------------------------------------------------- coding loop
def code_some_shards(matrix_rows, inputs, outputs, offset, byte_count):
    rows = [np.ascontiguousarray(r, dtype=np.uint8) for r in matrix_rows]
    lib().orc_code_some_shards(_ptrs(rows), _ptrs(inputs), len(inputs), _ptrs(outputs), len(outputs), offset,
                               byte_count)


# ---------------------------------------------------------------- ReedSolomon
class ReedSolomon:
    """ReedSolomon.java restated (default InputOutputByteTableCodingLoop)."""

    def __init__(self, data_shards: int, parity_shards: int):
        h = ctypes.c_void_p()
        _check(lib().orc_rs_create(data_shards, parity_shards, ctypes.byref(h)))
        self._h = h
        self.data_shard_count = data_shards
        self.parity_shard_count = parity_shards
        self.total_shard_count = data_shards + parity_shards

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.orc_rs_free(self._h)
            self._h = None

    @property
    def matrix(self) -> np.ndarray:
        out = np.zeros((self.total_shard_count, self.data_shard_count), dtype=np.uint8)
        lib().orc_rs_matrix(self._h, _ptr(out))
        return out

    @property
    def parity_rows(self) -> np.ndarray:
        return self.matrix[self.data_shard_count:]

    @staticmethod
    def _len(shards):
        return len(shards[0]) if len(shards) else 0

    def encode_parity(self, shards, offset, byte_count):
        _check(lib().orc_rs_encode_parity(self._h, _ptrs(shards), len(shards), self._len(shards), offset, byte_count))

    def encode_parity_single(self, shard, output, input_index, output_index, offset, byte_count):
        _check(lib().orc_rs_encode_parity_single(self._h, _ptr(shard), _ptr(output), input_index, output_index,
                                                 offset, byte_count))

    def is_parity_correct(self, shards, first_byte, byte_count, temp_buffer=None) -> bool:
        t = None if temp_buffer is None else _ptr(temp_buffer)
        tl = 0 if temp_buffer is None else len(temp_buffer)
        return bool(_check(lib().orc_rs_is_parity_correct(self._h, _ptrs(shards), len(shards), self._len(shards),
                                                          first_byte, byte_count, t, tl)))

    def decode_missing(self, shards, shard_present, offset, byte_count):
        pres = np.array([1 if p else 0 for p in shard_present], dtype=np.uint8)
        _check(lib().orc_rs_decode_missing(self._h, _ptrs(shards), _ptr(pres), len(shards), self._len(shards),
                                           offset, byte_count))

    def decode_missing_single(self, shard, shard_index, index, shard_present, outputs, offset, byte_count,
                              is_first):
        pres = np.array([1 if p else 0 for p in shard_present], dtype=np.uint8)
        _check(lib().orc_rs_decode_missing_single(self._h, _ptr(shard), shard_index, index, _ptr(pres),
                                                  _ptrs(outputs), len(outputs), offset, byte_count,
                                                  1 if is_first else 0))


# ---------------------------------------------------------------- Clay
class Clay:
    """ClayCodeErasureDecodingStep + ClayCode restated."""

    def __init__(self, data_units: int, parity_units: int, erased_indexes, is_test: bool = False):
        """is_test: the reference run with -DisTest=true (decodeDecoupledPlane :571-581)."""
        er = np.ascontiguousarray(list(erased_indexes), dtype=np.int32)
        h = ctypes.c_void_p()
        _check(lib().orc_clay_create_ex(data_units, parity_units, _ptr(er), len(er), 1 if is_test else 0,
                                        ctypes.byref(h)))
        self._h = h
        self.k, self.m = data_units, parity_units
        self.n = data_units + parity_units
        self.erased = list(erased_indexes)
        self.alpha = lib().orc_clay_alpha(h)
        self.q = lib().orc_clay_q(h)
        self.t = lib().orc_clay_t(h)

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.orc_clay_free(self._h)
            self._h = None

    def helper_planes(self, erased_index: int):
        out = np.zeros(self.alpha, dtype=np.int32)
        n = _check(lib().orc_clay_helper_planes(self._h, erased_index, _ptr(out)))
        return [int(x) for x in out[:n]]

    def perform_coding(self, inputs, outputs, buf_size: int):
        """inputs: n*alpha list (plane-major, None = absent); outputs: |E|*alpha arrays."""
        _check(lib().orc_clay_perform_coding(self._h, _ptrs(inputs), _ptrs(outputs), buf_size))

    def decode_single_helper(self, helper_coupled, helper_i, outputs, erased_index, buf_size):
        _check(lib().orc_clay_decode_single_helper(self._h, _ptrs(helper_coupled), helper_i, _ptrs(outputs),
                                                   erased_index, buf_size))


def bench_clay_repair(data_units, parity_units, erased, block_size, stripes, threads, seconds):
    """Timing harness (orc_bench.c): `stripes` is a list of threads*per_thread stripes, each a
    list of n*alpha sub-chunk arrays (None = absent).  Returns (repairs, max elapsed seconds)."""
    per = len(stripes) // threads
    flat = [sc for st in stripes[:per * threads] for sc in st]
    reps, el = ctypes.c_longlong(0), ctypes.c_double(0.0)
    _check(lib().orc_bench_clay_repair(data_units, parity_units, erased, block_size, _ptrs(flat), per, threads,
                                       float(seconds), ctypes.byref(reps), ctypes.byref(el)))
    return int(reps.value), float(el.value)


def shortened_clay_perform_coding(k, m, v, erased_real, inputs_real, B):
    """A shortened Clay code: the reference Clay(k+v, m)
    (ClayCodeErasureDecodingStep.java:53-107) run with the v virtual data nodes
    zero-filled.  inputs_real / the result use the REAL node numbering of the shortened
    code (slot z*(k+m) + node; output z*|E| + j)."""
    n_r, n_u = k + m, k + v + m
    und = lambda r: r if r < k else r + v  # noqa: E731
    c = Clay(k + v, m, [und(e) for e in erased_real])
    a = c.alpha
    zero = np.zeros(B, np.uint8)
    inputs = [None] * (n_u * a)
    for z in range(a):
        for r in range(n_r):
            inputs[z * n_u + und(r)] = inputs_real[z * n_r + r]
        for u in range(k, k + v):
            inputs[z * n_u + u] = zero
    outs = [np.zeros(B, np.uint8) for _ in range(len(erased_real) * a)]
    c.perform_coding(inputs, outs, B)
    return outs


BENCH_CLAY, BENCH_RS_DECODE, BENCH_RS_ENCODE, BENCH_RS_CHECK = 0, 1, 2, 3


def bench_run(op, data, parity, erased, buf_size, addrs, threads, seconds):
    """Timing harness (orc_bench.c orc_bench_run): `addrs` is an int64 array [units][slots]
    of host addresses (0 = absent) -- Clay: n*alpha sub-chunks per unit; RS: n shards --
    split evenly over `threads` workers.  Returns (operations, max elapsed seconds)."""
    addrs = np.ascontiguousarray(addrs, dtype=np.int64)
    units, slots = addrs.shape
    per = units // threads
    er = np.ascontiguousarray(list(erased) or [0], dtype=np.int32)
    reps, el = ctypes.c_longlong(0), ctypes.c_double(0.0)
    _check(lib().orc_bench_run(op, data, parity, _ptr(er), len(erased), buf_size, _ptr(addrs), slots, per, threads,
                               float(seconds), ctypes.byref(reps), ctypes.byref(el)))
    return int(reps.value), float(el.value)


def clay_get_inputs(data_units: int, parity_units: int, block_size: int):
    """ClayCode.getInputs (ClayCode.java:47-77): returns (list of n*alpha arrays or None)."""
    n = data_units + parity_units
    t = n // parity_units
    alpha = parity_units ** t
    flat = np.zeros(n * alpha * block_size, dtype=np.uint8)
    present = np.zeros(n * alpha, dtype=np.uint8)
    _check(lib().orc_clay_get_inputs(data_units, parity_units, block_size, _ptr(flat), _ptr(present)))
    flat = flat.reshape(n * alpha, block_size)
    return [flat[i].copy() if present[i] else None for i in range(n * alpha)]


def clay_encode(data_units, parity_units, inputs, block_size):
    """ClayCode.encode (ClayCode.java:89-99): parity column decoded by doDecodeMulti.
    Returns outputs: m*alpha arrays, outputs[z*m + j] = parity node k+j, plane z."""
    erased = list(range(data_units, data_units + parity_units))
    c = Clay(data_units, parity_units, erased)
    outs = [np.zeros(block_size, dtype=np.uint8) for _ in range(len(erased) * c.alpha)]
    c.perform_coding(inputs, outs, block_size)
    return outs


# ---------------------------------------------------------------- LRC (LRCErasureCodeExample.kt)
LRC_N, LRC_K, LRC_R = 16, 12, 3  # LRCErasureUtil.kt:4-6


def lrc_encode(data: np.ndarray):
    """LRCErasureCodeExample.encode (:30-57): K blocks of len/K bytes -> N blocks."""
    block = len(data) // LRC_K
    rs = ReedSolomon(LRC_R, 1)
    blocks = []
    pos = 0
    for _ in range(LRC_K // LRC_R):
        shards = []
        for _ in range(LRC_R):
            shards.append(np.ascontiguousarray(data[pos:pos + block], dtype=np.uint8).copy())
            pos += block
        shards.append(np.zeros(block, dtype=np.uint8))
        rs.encode_parity(shards, 0, block)
        blocks.extend(shards)
    return blocks


def lrc_encode_using_single(data: np.ndarray):
    """LRCErasureCodeExample.encodeUsingSingle (:59-90) via encodeParitySingle."""
    block = len(data) // LRC_K
    rs = ReedSolomon(LRC_R, 1)
    blocks = []
    pos = 0
    for _ in range(LRC_K // LRC_R):
        shards = []
        for _ in range(LRC_R):
            shards.append(np.ascontiguousarray(data[pos:pos + block], dtype=np.uint8).copy())
            pos += block
        out = np.zeros(block, dtype=np.uint8)
        for idx in range(LRC_R):
            rs.encode_parity_single(shards[idx], out, idx, 0, 0, block)
        shards.append(out)
        blocks.extend(shards)
    return blocks


def lrc_decode(blocks, missing, block_size):
    """LRCErasureCodeExample.decode (:92-131): group-wise RS(3,1).decodeMissing; returns file bytes."""
    rs = ReedSolomon(LRC_R, 1)
    shards = [None if i in missing else np.array(blocks[i], dtype=np.uint8) for i in range(LRC_N)]
    for i in range(LRC_N):
        if shards[i] is None:
            shards[i] = np.zeros(block_size, dtype=np.uint8)
    for g in range(LRC_K // LRC_R):
        lo = g * (LRC_R + 1)
        present = [(lo + j) not in missing for j in range(LRC_R + 1)]
        rs.decode_missing(shards[lo:lo + LRC_R + 1], present, 0, block_size)
    out = [shards[i] for i in range(LRC_N) if i == 0 or (i + 1) % (LRC_R + 1) != 0]
    return np.concatenate(out), shards


# ---------------------------------------------------------------- Sample{En,De}coder
def sample_encode(file_bytes: np.ndarray, data_shards=4, parity_shards=2):
    """SampleEncoder.java:54-83: [int32 BE len][file][0-pad] split into data shards + RS parity."""
    file_size = len(file_bytes)
    stored = file_size + 4
    shard_size = (stored + data_shards - 1) // data_shards
    allb = np.zeros(shard_size * data_shards, dtype=np.uint8)
    allb[:4] = np.frombuffer(int(file_size).to_bytes(4, "big"), dtype=np.uint8)
    allb[4:4 + file_size] = file_bytes
    shards = [allb[i * shard_size:(i + 1) * shard_size].copy() for i in range(data_shards)]
    shards += [np.zeros(shard_size, dtype=np.uint8) for _ in range(parity_shards)]
    ReedSolomon(data_shards, parity_shards).encode_parity(shards, 0, shard_size)
    return shards


def sample_decode(shards, data_shards=4, parity_shards=2):
    """SampleDecoder.java:34-98: decodeMissing over the present shards, strip the length header."""
    total = data_shards + parity_shards
    shard_size = next(len(s) for s in shards if s is not None)
    present = [s is not None for s in shards]
    if sum(present) < data_shards:
        raise OracleError(-2)
    work = [np.array(s, dtype=np.uint8) if s is not None else np.zeros(shard_size, dtype=np.uint8) for s in shards]
    ReedSolomon(data_shards, parity_shards).decode_missing(work, present, 0, shard_size)
    allb = np.concatenate(work[:data_shards])
    size = int.from_bytes(allb[:4].tobytes(), "big")
    return allb[4:4 + size].copy(), work
