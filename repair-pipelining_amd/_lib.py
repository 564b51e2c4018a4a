"""ctypes binding of libecx.so (include/ecx.h).

The shared library is built in-tree by ``make -C repair-pipelining_amd`` (or
``__graft_entry__.build()``).  There is deliberately no CPU fallback: if the
library or a HIP device is missing, calls raise.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
# ECX_LIB_PATH: load another build of the same ABI (A/B runs of two kernel builds,
# scripts/ab_configs.sh); the default is the in-tree build.
LIB_PATH = Path(os.environ["ECX_LIB_PATH"]) if os.environ.get("ECX_LIB_PATH") else PKG_DIR / "libecx.so"
HEADER = PKG_DIR.parent / "include" / "ecx.h"

STATUS = {
    0: "ok",
    -1: "IllegalArgumentException",
    -2: "IllegalArgumentException: Not enough shards present",
    -3: "IllegalArgumentException: Matrix is singular",
    -4: "IllegalArgumentException: too many shards - max is 256",
    -5: "ArrayIndexOutOfBoundsException",
    -6: "NullPointerException",
    -7: "OutOfMemoryError",
    -10: "HIP device error",
}


class EcxError(Exception):
    """Raised for a negative ecx_status; ``code`` is the status, the message
    names the Java exception the reference throws in the same situation."""

    def __init__(self, code: int, detail: str = ""):
        self.code = code
        super().__init__(f"{STATUS.get(code, 'status')} ({code}){': ' + detail if detail else ''}")


BUILD_LOCK = PKG_DIR / ".build.lock"


def build(verbose: bool = False, only_if_missing: bool = False) -> Path:
    """Compile libecx.so for gfx950 with hipcc (repair-pipelining_amd/Makefile).

    Serialised across processes by an exclusive flock on PKG_DIR/.build.lock, so the N
    ranks of `bench.py --gpus N` (or parallel test workers) on a checkout without a
    build never run `make` in the same directory at once; with ``only_if_missing`` the
    existence check runs under the lock too, so only the first rank builds."""
    import fcntl
    with open(BUILD_LOCK, "a") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if only_if_missing and LIB_PATH.exists():
                return LIB_PATH
            jobs = str(min(8, os.cpu_count() or 1))
            subprocess.run(["make", "-C", str(PKG_DIR), "-j", jobs] + ([] if verbose else ["-s"]), check=True)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    return LIB_PATH


P = ctypes.c_void_p
I = ctypes.c_int
I64 = ctypes.c_int64
U64 = ctypes.c_uint64
PP = ctypes.POINTER(ctypes.c_void_p)
PI = ctypes.POINTER(ctypes.c_int)

# name -> (restype, argtypes); kept in the order of include/ecx.h
SIGNATURES = {
    "ecx_status_string": (ctypes.c_char_p, [I]),
    "ecx_last_error": (ctypes.c_char_p, []),
    "ecx_version": (I, []),
    "ecx_device_count": (I, [PI]),
    "ecx_set_device": (I, [I]),
    "ecx_synchronize": (I, [P]),
    "ecx_gf_multiply": (I, [I, I]),
    "ecx_gf_divide": (I, [I, I]),
    "ecx_gf_exp": (I, [I, I]),
    "ecx_gf_tables": (I, [P, P, P]),
    "ecx_matrix_times": (I, [P, I, I, P, I, I, P]),
    "ecx_matrix_invert": (I, [P, I, P]),
    "ecx_code_some_shards": (I, [P, PP, I, PP, I, I, I]),
    "ecx_check_some_shards": (I, [P, PP, I, PP, I, I, I, P]),
    "ecx_code_single": (I, [P, I, P, I, P, I, I, I, I]),
    "ecx_rs_create": (I, [I, I, ctypes.POINTER(P)]),
    "ecx_rs_destroy": (None, [P]),
    "ecx_rs_matrix": (I, [P, P]),
    "ecx_rs_shape": (I, [P, PI, PI]),
    "ecx_rs_encode_parity": (I, [P, PP, I, I, I, I]),
    "ecx_rs_encode_parity_single": (I, [P, P, P, I, I, I, I]),
    "ecx_rs_is_parity_correct": (I, [P, PP, I, I, I, I, P, I]),
    "ecx_rs_decode_missing": (I, [P, PP, P, I, I, I, I]),
    "ecx_rs_decode_missing_single": (I, [P, P, I, I, P, PP, I, I, I, I]),
    "ecx_map_create": (I, [P, I, I, P, P, ctypes.POINTER(P)]),
    "ecx_map_destroy": (None, [P]),
    "ecx_map_info": (I, [P, PI, PI, PI]),
    "ecx_map_matrix": (I, [P, P, P, P]),
    "ecx_map_slot_extent": (I, [P, PI, PI]),
    "ecx_map_apply_batch": (I, [P, P, I64, I64, P, I64, I64, I64, I64, P]),
    "ecx_rs_blocked_layout": (I, [I, I, I64, P]),
    "ecx_rs_recommended_pitch": (I, [I, I, I64, P]),
    "ecx_rs_encode_parity_blocked_batch": (I, [P, P, I64, I64, I64, P]),
    "ecx_rs_decode_missing_blocked_batch": (I, [P, P, P, I64, I64, I64, P]),
    "ecx_rs_encode_parity_blocked_batch_host": (I, [P, P, I64, I64, I64]),
    "ecx_rs_decode_missing_blocked_batch_host": (I, [P, P, P, I64, I64, I64]),
    "ecx_rs_encode_parity_blocked_batch_host_devices": (I, [P, P, I64, I64, I64, P, I]),
    "ecx_rs_decode_missing_blocked_batch_host_devices": (I, [P, P, P, I64, I64, I64, P, I]),
    "ecx_map_accumulate_batch": (I, [P, P, I64, I64, P, I64, I64, I64, I64, P]),
    "ecx_rs_encode_map": (I, [P, ctypes.POINTER(P)]),
    "ecx_rs_decode_map": (I, [P, P, ctypes.POINTER(P)]),
    "ecx_rs_encode_parity_batch": (I, [P, P, I64, I64, I64, I64, I64, P]),
    "ecx_rs_is_parity_correct_batch": (I, [P, P, I64, I64, I64, I64, I64, P, P]),
    "ecx_rs_decode_missing_batch": (I, [P, P, P, I64, I64, I64, I64, I64, P]),
    "ecx_rs_decode_partial_batch": (I, [P, P, I, P, I64, P, I64, I64, I64, I64, I, P]),
    "ecx_rs_encode_partial_batch": (I, [P, I, P, I64, P, I64, I64, I64, I64, I, P]),
    "ecx_clay_create": (I, [I, I, P, I, ctypes.POINTER(P)]),
    "ecx_clay_create_shortened": (I, [I, I, I, P, I, ctypes.POINTER(P)]),
    "ecx_clay_create_ex": (I, [I, I, I, P, I, I, ctypes.POINTER(P)]),
    "ecx_clay_destroy": (None, [P]),
    "ecx_clay_geometry": (I, [P, PI, PI, PI]),
    "ecx_clay_helper_planes": (I, [P, I, P]),
    "ecx_clay_shape": (I, [P, PI, PI, PI]),
    "ecx_clay_perform_coding": (I, [P, PP, PP, I]),
    "ecx_clay_decode_single_helper": (I, [P, PP, I, PP, I, I]),
    "ecx_clay_map": (I, [P, ctypes.POINTER(P)]),
    "ecx_clay_perform_coding_batch": (I, [P, P, I64, I64, P, I64, I64, I64, I64, P]),
    "ecx_lrc_map": (I, [P, ctypes.POINTER(P)]),
    "ecx_lrc_encode_batch": (I, [P, I64, I64, I64, I64, P]),
    "ecx_lrc_decode_batch": (I, [P, I64, I64, P, I64, I64, P]),
    "ecx_map_apply_batch_host": (I, [P, P, I64, I64, P, I64, I64, I64, I64]),
    "ecx_clay_perform_coding_batch_host": (I, [P, P, I64, I64, P, I64, I64, I64, I64]),
    "ecx_map_apply_batch_host_devices": (I, [P, P, I64, I64, P, I64, I64, I64, I64, P, I]),
    "ecx_clay_perform_coding_batch_host_devices": (I, [P, P, I64, I64, P, I64, I64, I64, I64, P, I]),
    "ecx_rs_is_parity_correct_batch_host": (I, [P, P, I64, I64, I64, I64, I64, P]),
    "ecx_rs_is_parity_correct_batch_host_devices": (I, [P, P, I64, I64, I64, I64, I64, P, P, I]),
    "ecx_host_alloc": (I, [I64, ctypes.POINTER(P)]),
    "ecx_host_free": (I, [P]),
    "ecx_host_register": (I, [P, I64]),
    "ecx_host_unregister": (I, [P]),
    "ecx_fill_random": (I, [P, I64, U64, P]),
    "ecx_count_mismatch": (I, [P, I64, P, I64, I64, I64, P, P]),
}

_lib = None


def _share_torch_hip_runtime():
    """PyTorch-ROCm wheels bundle their own libamdhip64 (SONAME libamdhip64.so.7,
    but requested by the unversioned name).  If libecx were loaded first, the
    dynamic loader would map /opt/rocm's runtime for libecx and then a second
    copy for torch -- two HIP runtimes in one process.  Importing torch first
    makes libecx bind to the runtime torch already mapped (matching SONAME), so
    torch tensors / streams and libecx launches share one runtime."""
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    """Load libecx.so (building it first if this checkout has no build)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build(only_if_missing=True)
        _share_torch_hip_runtime()
        l = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def check(status: int) -> int:
    if status < 0:
        detail = lib().ecx_last_error()
        raise EcxError(status, detail.decode() if detail else "")
    return status
