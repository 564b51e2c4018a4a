"""The JNI binding (jni/): generated from include/ecx.h by jni/gen_jni.py, one
forwarder per export.  No JDK exists in this container, so the binding
is checked structurally: the committed files are what the generator produces, every
export has exactly one forwarder that calls it with exactly its parameters, every
Java native has its C forwarder with the matching parameter count, and the C compiles
(gcc -fsyntax-only against tests/native/jni_syntax_stub.h, the JNI spec's shapes)."""
import re
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "jni"))
import gen_jni  # noqa: E402

C_SRC = (ROOT / "jni" / "ecx_jni.c").read_text()
JAVA_SRC = (ROOT / "jni" / "com" / "backblaze" / "erasure" / "ecx" / "EcxNative.java").read_text()


def forwarders():
    """JNI function name -> (parameter count, body)."""
    out = {}
    for m in re.finditer(r"JNIEXPORT \w+ JNICALL (Java_\w+)\(([^)]*)\) \{(.*?)\n\}", C_SRC, flags=re.S):
        out[m.group(1)] = (len([p for p in m.group(2).split(",") if p.strip()]), m.group(3))
    return out


def call_args(body, name):
    """Argument count of the (single) call to `name` in a forwarder body."""
    calls = [m.start() for m in re.finditer(r"\b%s\(" % name, body)]
    assert len(calls) == 1, (name, len(calls))
    i, depth, n, seen = calls[0] + len(name) + 1, 1, 1, False
    while depth:
        ch = body[i]
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        elif ch == "," and depth == 1:
            n += 1
        elif not ch.isspace() and depth == 1:
            seen = True
        i += 1
    return n if seen else 0


def test_generated_files_are_fresh():
    assert gen_jni.main(check=True), "jni/ecx_jni.c or EcxNative.java is stale: run python jni/gen_jni.py"


def test_one_forwarder_per_export_with_matching_arguments():
    fw = forwarders()
    exports = gen_jni.exports()
    assert len(exports) >= 50
    for ret, name, params in exports:
        jname = "Java_%s_%s" % (gen_jni.JCLASS, gen_jni.camel(name))
        assert jname in fw, name
        nparams, body = fw[jname]
        assert call_args(body, name) == len(params), name
    called = set(re.findall(r"\b(ecx_[a-z0-9_]+)\(", C_SRC)) - {"ecx_jni_buflist"}
    assert called == {name for _, name, _ in exports}


def test_java_natives_match_forwarders():
    fw = forwarders()
    natives = re.findall(r"(?:public )?static native [\w\[\]]+ (\w+)\(([^)]*)\);", JAVA_SRC)
    assert len(natives) == len(fw)
    for jname, params in natives:
        key = "Java_%s_%s" % (gen_jni.JCLASS, jname)
        assert key in fw, jname
        n_java = len([p for p in params.split(",") if p.strip()])
        assert fw[key][0] == n_java + 2, jname  # + JNIEnv*, jclass


def test_java_classes_use_existing_natives():
    """EcxCodingLoop / EcxPartialSums / EcxClayCodeErasureDecodingStep call only
    natives that EcxNative declares."""
    public = set(re.findall(r"public static native [\w\[\]]+ (\w+)\(", JAVA_SRC))
    private = set(re.findall(r"\n    static native [\w\[\]]+ (\w+)\(", JAVA_SRC))
    for f in (ROOT / "jni").rglob("*.java"):
        if f.name == "EcxNative.java":
            continue
        same_package = "package com.backblaze.erasure.ecx;" in f.read_text()
        for used in re.findall(r"EcxNative\.(\w+)\(", f.read_text()):
            assert used in public or (same_package and used in private), (f.name, used)
    loop = (ROOT / "jni" / "com" / "backblaze" / "erasure" / "EcxCodingLoop.java").read_text()
    assert "extends CodingLoopBase" in loop and "codeSomeShards" in loop and "checkSomeShards" in loop


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_forwarders_compile():
    stub_dir = ROOT / "tests" / "native"
    include = ROOT / "tests" / "native" / "_jni_include"
    include.mkdir(exist_ok=True)
    (include / "jni.h").write_text('#include "%s"\n' % (stub_dir / "jni_syntax_stub.h"))
    try:
        r = subprocess.run(["gcc", "-fsyntax-only", "-std=c11", "-Wall", "-Werror", "-I", str(include),
                            "-I", str(ROOT / "include"), str(ROOT / "jni" / "ecx_jni.c")],
                           capture_output=True, text=True)
    finally:
        shutil.rmtree(include, ignore_errors=True)
    assert r.returncode == 0, r.stderr[-3000:]


def test_no_public_native_takes_a_raw_host_address():
    """Round-4 verdict item: a Java caller must not bypass the ByteBuffer capacity checks.
    Every host-batch native that takes raw host addresses (long in / long out), and
    directAddress / wrapAddress, are package-private; the public host-batch natives take
    direct ByteBuffers whose capacity the forwarder reads itself (ClayCoordinator.kt:378-390)."""
    public = dict(re.findall(r"public static native [\w\[\]]+ (\w+)\(([^)]*)\);", JAVA_SRC))
    for name in ("directAddress", "wrapAddress", "mapApplyBatchHost", "clayPerformCodingBatchHost",
                 "mapApplyBatchHostDevices", "clayPerformCodingBatchHostDevices", "rsIsParityCorrectBatchHost",
                 "rsIsParityCorrectBatchHostDevices", "rsEncodeParityBlockedBatchHost",
                 "rsDecodeMissingBlockedBatchHost", "rsEncodeParityBlockedBatchHostDevices",
                 "rsDecodeMissingBlockedBatchHostDevices"):
        assert name not in public, name
        assert re.search(r"\n    static native [\w\[\]]+ %s\(" % name, JAVA_SRC), name
    host_batch = {n: p for n, p in public.items() if "BatchHost" in n}
    assert set(host_batch) == {"mapApplyBatchHostBuffer", "clayPerformCodingBatchHostBuffer",
                               "mapApplyBatchHostDevicesBuffer", "clayPerformCodingBatchHostDevicesBuffer",
                               "rsIsParityCorrectBatchHostBuffer", "rsIsParityCorrectBatchHostDevicesBuffer",
                               "rsEncodeParityBlockedBatchHostBuffer", "rsDecodeMissingBlockedBatchHostBuffer",
                               "rsEncodeParityBlockedBatchHostDevicesBuffer",
                               "rsDecodeMissingBlockedBatchHostDevicesBuffer"}
    blocked = {n for n in host_batch if "Blocked" in n}  # one buffer of whole blocked stripes, in place
    for n, params in host_batch.items():
        if n in blocked:
            assert "ByteBuffer base" in params and "long base," not in params, n
            continue
        if n.startswith("rsIsParityCorrect"):  # the stripes and one verdict byte per stripe
            assert "ByteBuffer base" in params and "ByteBuffer verdict" in params, n
            assert "long base," not in params and "long verdict," not in params, n
            continue
        assert "ByteBuffer in" in params and "ByteBuffer out" in params, n
        assert "long in," not in params and "long out," not in params, n
    # the generated C forwarder reads the capacity of every ByteBuffer it is given
    for n in host_batch:
        body = re.search(r"JNICALL Java_%s_%s\(.*?\n\}" % (gen_jni.JCLASS, n), C_SRC, flags=re.S).group(0)
        assert body.count("direct_check(") == (1 if n in blocked else 2), n


def test_no_read_only_int_array_is_pinned():
    """a critical pin stalls the JVM's GC for as long as it is held, and
    the multi-GPU host batches run for seconds.  Every read-only int[] (the device lists,
    slot lists, erased indices) is copied with GetIntArrayRegion before any pin opens, and no
    host-batch forwarder pins anything across its export call (its buffers are raw addresses
    or direct ByteBuffers)."""
    const_ints = {(name, p) for _ret, name, params in gen_jni.exports() for t, p in params
                  if t.replace(" ", "") == "constint*"}
    assert ("ecx_map_apply_batch_host_devices", "devices") in const_ints and len(const_ints) >= 7
    fw = forwarders()
    for name, p in const_ints:
        body = fw["Java_%s_%s" % (gen_jni.JCLASS, gen_jni.camel(name))][1]
        assert "PIN(%s)" % p not in body, (name, p)
        copy = body.index("GetIntArrayRegion(env, %s, " % p)
        first_pin = min([body.index(x) for x in ("PIN(", "buflist_pin(") if x in body] or [len(body)])
        assert copy < first_pin < len(body) or first_pin == len(body), (name, p)
        assert "free(%s_p);" % p in body
    for jname, (_n, body) in fw.items():
        if "BatchHost" in jname:
            assert "PIN(" not in body and "buflist_pin(" not in body and "Critical" not in body, jname
