"""ctypes driver of the generated JNI forwarders (jni/ecx_jni.c) over the fake JNIEnv of
tests/native/jni_fake_env.c (no JDK in this image): Java arrays are fakes
wrapping numpy memory, so a forwarder's writes land in the numpy arrays, and the fake
counts pins, releases and JNI-rule violations.  Used by tests/test_jni_runtime.py."""
import ctypes
import re
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
NATIVE = ROOT / "tests" / "native"
LIB = NATIVE / "_build" / "libjnitest.so"
JCLASS = "Java_com_backblaze_erasure_ecx_EcxNative_"

_CTYPE = {"jint": ctypes.c_int, "jlong": ctypes.c_int64}


def build():
    subprocess.run(["make", "-s", "-C", str(NATIVE)], check=True)
    return LIB


def _signatures():
    """forwarder name -> (restype, argtypes) parsed from the generated C."""
    src = (ROOT / "jni" / "ecx_jni.c").read_text()
    out = {}
    for m in re.finditer(r"JNIEXPORT (\w+) JNICALL %s(\w+)\(([^)]*)\)" % JCLASS, src):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        args = []
        for p in params.split(","):
            t = p.strip().rsplit(" ", 1)[0].replace(" *", "*")
            args.append(_CTYPE.get(t, ctypes.c_void_p))
        res = {"jint": ctypes.c_int, "void": None}.get(ret, ctypes.c_void_p)
        out[name] = (res, args)
    return out


class Jni:
    def __init__(self):
        # libecx.so is mapped through the product package first (torch's HIP runtime), so
        # the forwarders bind to that same library instance
        import rpamd
        rpamd.load()
        build()  # make is incremental: rebuilds when the forwarders or the fakes changed
        self.lib = ctypes.CDLL(str(LIB))
        L = self.lib
        L.fake_env.restype = ctypes.c_void_p
        L.fake_array.restype = ctypes.c_void_p
        L.fake_array.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
        L.fake_direct_buffer.restype = ctypes.c_void_p
        L.fake_direct_buffer.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.fake_object_array.restype = ctypes.c_void_p
        L.fake_object_array.argtypes = [ctypes.c_int32]
        L.fake_set_element.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
        L.fake_string.restype = ctypes.c_char_p
        L.fake_string.argtypes = [ctypes.c_void_p]
        L.fake_free.argtypes = [ctypes.c_void_p]
        L.fake_counters.argtypes = [ctypes.POINTER(ctypes.c_int64)]
        self.env = L.fake_env()
        self.sigs = _signatures()
        self._keep = []   # numpy arrays wrapped by live fakes
        self._fakes = []

    # ---------------------------------------------------------------- Java-side objects
    def array(self, a):
        """A Java primitive array (byte[] / int[] / short[] / long[] / boolean[] as bytes)
        over the numpy array `a` (no copy); None stays a null reference."""
        if a is None:
            return None
        a = np.ascontiguousarray(a)
        self._keep.append(a)
        o = self.lib.fake_array(a.ctypes.data, int(a.size), int(a.itemsize))  # non-null even when empty
        self._fakes.append(o)
        return o

    def direct(self, a, capacity=None):
        """A direct java.nio.ByteBuffer over the numpy array `a` (no copy), of `capacity`
        bytes (default: all of `a`)."""
        a = np.ascontiguousarray(a)
        self._keep.append(a)
        o = self.lib.fake_direct_buffer(a.ctypes.data, int(a.nbytes if capacity is None else capacity))
        self._fakes.append(o)
        return o

    def array2d(self, rows):
        """A Java byte[][] (element None = null)."""
        o = self.lib.fake_object_array(len(rows))
        self._fakes.append(o)
        for i, r in enumerate(rows):
            self.lib.fake_set_element(o, i, self.array(r))
        return o

    def ints(self, v):
        return self.array(np.asarray(v, np.int32))

    def counters(self):
        c = (ctypes.c_int64 * 7)()
        self.lib.fake_counters(c)
        keys = ("pins_now", "pins", "unpins", "violations", "deleted", "calls_while_pinned", "last_mode")
        return dict(zip(keys, list(c)))

    def reset(self):
        self.lib.fake_reset()

    def free_all(self):
        for o in self._fakes:
            self.lib.fake_free(o)
        self._fakes, self._keep = [], []

    # ---------------------------------------------------------------- forwarders
    def call(self, name, *args):
        """EcxNative.<name>(args) through its generated forwarder; returns the status."""
        res, argtypes = self.sigs[name]
        f = getattr(self.lib, JCLASS + name)
        f.restype, f.argtypes = res, argtypes
        assert len(args) == len(argtypes) - 2, (name, len(args), len(argtypes) - 2)
        return f(self.env, None, *args)

    def string(self, jstr):
        return self.lib.fake_string(jstr).decode()
