"""Generate the JNI binding of libecx.so from include/ecx.h:

  jni/ecx_jni.c                        one JNI forwarder per ecx.h export
  jni/com/backblaze/erasure/ecx/EcxNative.java   the matching `static native` declarations

Each forwarder converts its Java arguments and calls the export with exactly the
export's parameters (the checks in tests/test_jni.py parse both files).  Java-side
types:

  int / int64_t / uint64_t          int / long / long
  handle (ecx_rs*, ecx_clay*, ecx_map*), void* stream / host or device address
                                    long
  ecx_X **out, void **out           long[] (element 0 receives the handle / address)
  host byte buffer (uint8_t *)      byte[] (pinned with GetPrimitiveArrayCritical; may be null
                                    where the C side accepts NULL)
  int* / int16_t*                   int[] / short[] (pinned)
  uint8_t *const * (buffer list)    byte[][] plus an int[] of per-buffer start positions (null =
                                    all 0); null elements stay NULL (absent Clay sub-chunks)
  const char * result               String

In the device-batch and host-batch entry points (*_batch, *_batch_host, fill_random,
count_mismatch) byte pointers are addresses (long): device pointers, or pinned /
direct-buffer host addresses; only the *_present flag arrays there are byte[].

JNI rules kept by every forwarder: all non-critical JNI calls (array elements,
positions, lengths) happen before the first GetPrimitiveArrayCritical and after the last
release, so no JNI call runs inside a critical region.

Argument checks (RULES below): the C ABI takes plain pointers and cannot know a Java
array's length, so before anything is pinned every forwarder checks what the export
will touch, and returns the status of the exception the reference would throw instead
of reading or writing past a Java array:
  * a handle of 0, or a null array the export dereferences     -> ECX_E_NULL
    (NullPointerException)
  * a negative count / size / offset                           -> ECX_E_ILLEGAL_ARGUMENT
  * a byte[][] shorter than the count the export reads (Clay: not exactly n*alpha /
    |E|*alpha, ClayCodeErasureDecodingStep.java:76-82; RS shard lists: "wrong number of
    shards", ReedSolomon.java:341-343)                         -> ECX_E_ILLEGAL_ARGUMENT
    or ECX_E_INDEX (ArrayIndexOutOfBoundsException, CodingLoop lists)
  * an element (or array) with fewer than position + offset + byteCount bytes, or a
    negative position                                          -> ECX_E_INDEX, or
    ECX_E_ILLEGAL_ARGUMENT where the reference's checkBuffersAndSizes throws
    ("buffers to small", ReedSolomon.java:360-362)
Every pointer parameter of every export must have a rule: the generator stops otherwise.

Run:  python jni/gen_jni.py   (tests/test_jni.py fails if the committed files are stale)
"""
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "ecx.h"
OUT_C = ROOT / "jni" / "ecx_jni.c"
OUT_JAVA = ROOT / "jni" / "com" / "backblaze" / "erasure" / "ecx" / "EcxNative.java"
JCLASS = "com_backblaze_erasure_ecx_EcxNative"
HANDLES = ("ecx_rs", "ecx_clay", "ecx_map")
# byte pointers of these functions may be NULL (C side: "NULL = ..." or unused)
NULLABLE = {("ecx_check_some_shards", "temp_buffer"), ("ecx_rs_is_parity_correct", "temp_buffer"),
            ("ecx_lrc_map", "block_present"), ("ecx_map_create", "in_slot"), ("ecx_map_create", "out_slot"),
            ("ecx_map_info", "n_out"), ("ecx_map_info", "n_in"), ("ecx_map_info", "nnz"),
            ("ecx_map_matrix", "matrix"), ("ecx_map_matrix", "in_slot"), ("ecx_map_matrix", "out_slot"),
            ("ecx_map_slot_extent", "max_in_slot"), ("ecx_map_slot_extent", "max_out_slot"),
            ("ecx_clay_geometry", "q"), ("ecx_clay_geometry", "t"), ("ecx_clay_geometry", "alpha"),
            ("ecx_clay_shape", "nodes"), ("ecx_clay_shape", "n_erased"), ("ecx_clay_shape", "alpha"),
            ("ecx_rs_shape", "data_shards"), ("ecx_rs_shape", "parity_shards"),
            ("ecx_gf_tables", "log_table"), ("ecx_gf_tables", "exp_table"), ("ecx_gf_tables", "mul_table")}

ILL, IDX = "ECX_E_ILLEGAL_ARGUMENT", "ECX_E_INDEX"
OFF_BC = "(int64_t)offset + byte_count"
RS_N = "(int64_t)rs_k + rs_m"
# Queries a forwarder runs (after its handle checks) to size its argument checks.
QUERIES = {
    "rs": "    int rs_k = 0, rs_m = 0;\n    if (st == ECX_OK) st = ecx_rs_shape((const ecx_rs *)(intptr_t)rs, &rs_k, &rs_m);",
    "clay": "    int cl_n = 0, cl_ne = 0, cl_a = 0, cl_q = 1;\n"
            "    if (st == ECX_OK) st = ecx_clay_shape((const ecx_clay *)(intptr_t)clay, &cl_n, &cl_ne, &cl_a);\n"
            "    if (st == ECX_OK) st = ecx_clay_geometry((const ecx_clay *)(intptr_t)clay, &cl_q, NULL, NULL);",
    "map": "    int mp_out = 0, mp_in = 0;\n    if (st == ECX_OK) st = ecx_map_info((const ecx_map *)(intptr_t)map, &mp_out, &mp_in, NULL);",
}


def A(param, need, err=IDX):
    """A primitive array (byte[] / int[] / short[] / boolean flags) of >= need elements."""
    return ("array", param, need, err)


def L(param, count, need, count_err=IDX, len_err=IDX, exact=False, nulls=False, when=None):
    """A byte[][]: >= count entries (== with exact); entry i < count non-null (unless
    nulls) with pos[i] >= 0 and pos[i] + need bytes; only checked when `when` holds."""
    return ("list", param, count, need, count_err, len_err, exact, nulls, when)


def NN(*params, err=ILL):
    return ("nonneg", params, err)


# export -> (queries, rules); exports without pointer parameters need no entry.
RULES = {
    "ecx_device_count": ((), [A("count", "1")]),
    "ecx_gf_tables": ((), [A("log_table", "256"), A("exp_table", "510"), A("mul_table", "65536")]),
    "ecx_matrix_times": ((), [NN("a_rows", "a_cols", "b_rows", "b_cols"), A("a", "(int64_t)a_rows * a_cols"),
                              A("b", "(int64_t)b_rows * b_cols"), A("out", "(int64_t)a_rows * b_cols")]),
    "ecx_matrix_invert": ((), [NN("n"), A("m", "(int64_t)n * n"), A("out", "(int64_t)n * n")]),
    "ecx_code_some_shards": ((), [NN("input_count", "output_count", "offset", "byte_count"),
                                  A("matrix_rows", "(int64_t)output_count * input_count"),
                                  L("inputs", "input_count", OFF_BC), L("outputs", "output_count", OFF_BC)]),
    "ecx_check_some_shards": ((), [NN("input_count", "check_count", "offset", "byte_count"),
                                   A("matrix_rows", "(int64_t)check_count * input_count"),
                                   L("inputs", "input_count", OFF_BC), L("to_check", "check_count", OFF_BC),
                                   A("temp_buffer", "0")]),
    "ecx_code_single": ((), [NN("row_length", "offset", "byte_count"), NN("index", "output_index", err=IDX),
                             A("matrix_rows", "((int64_t)output_index + 1) * row_length"),
                             A("input", OFF_BC), A("output", OFF_BC)]),
    "ecx_rs_create": ((), []),
    "ecx_rs_matrix": (("rs",), [A("out", "(%s) * rs_k" % RS_N)]),
    "ecx_rs_shape": ((), [A("data_shards", "1"), A("parity_shards", "1")]),
    "ecx_rs_encode_parity": ((), [NN("shard_count", "shard_length", "offset", "byte_count"),
                                  L("shards", "shard_count", "shard_length", count_err=ILL, len_err=ILL)]),
    "ecx_rs_encode_parity_single": ((), [NN("offset", "byte_count"), A("shard", OFF_BC), A("output", OFF_BC)]),
    "ecx_rs_is_parity_correct": ((), [NN("shard_count", "shard_length", "first_byte", "byte_count", "temp_length"),
                                      L("shards", "shard_count", "shard_length", count_err=ILL, len_err=ILL),
                                      A("temp_buffer", "temp_length", err=ILL)]),
    "ecx_rs_decode_missing": (("rs",), [NN("shard_count", "shard_length", "offset", "byte_count"),
                                        L("shards", "shard_count", "shard_length", count_err=ILL, len_err=ILL),
                                        A("shard_present", RS_N)]),
    "ecx_rs_decode_missing_single": (("rs",), [NN("output_count", "offset", "byte_count"), A("shard", OFF_BC),
                                               A("shard_present", RS_N), L("outputs", "output_count", OFF_BC)]),
    "ecx_map_create": ((), [NN("n_out", "n_in"), A("matrix", "(int64_t)n_out * n_in"), A("in_slot", "n_in"),
                            A("out_slot", "n_out")]),
    "ecx_map_info": ((), [A("n_out", "1"), A("n_in", "1"), A("nnz", "1")]),
    "ecx_map_matrix": (("map",), [A("matrix", "(int64_t)mp_out * mp_in"), A("in_slot", "mp_in"),
                                  A("out_slot", "mp_out")]),
    "ecx_map_slot_extent": ((), [A("max_in_slot", "1"), A("max_out_slot", "1")]),
    "ecx_rs_decode_map": (("rs",), [A("shard_present", RS_N)]),
    "ecx_rs_decode_missing_batch": (("rs",), [A("shard_present", RS_N)]),
    "ecx_rs_blocked_layout": ((), [A("layout", "3")]),
    "ecx_rs_recommended_pitch": ((), [A("pitch", "1")]),
    "ecx_rs_decode_missing_blocked_batch": (("rs",), [A("shard_present", RS_N)]),
    "ecx_rs_decode_partial_batch": (("rs",), [A("shard_present", RS_N)]),
    "ecx_clay_create": ((), [NN("n_erased"), A("erased", "n_erased")]),
    "ecx_clay_create_shortened": ((), [NN("n_erased"), A("erased", "n_erased")]),
    "ecx_clay_create_ex": ((), [NN("n_erased"), A("erased", "n_erased")]),
    "ecx_clay_geometry": ((), [A("q", "1"), A("t", "1"), A("alpha", "1")]),
    "ecx_clay_shape": ((), [A("nodes", "1"), A("n_erased", "1"), A("alpha", "1")]),
    "ecx_clay_helper_planes": (("clay",), [A("out", "cl_a / (cl_q > 0 ? cl_q : 1)")]),
    # performCoding returns before its length checks when nothing is erased (:54-56)
    "ecx_clay_perform_coding": (("clay",), [NN("buf_size"),
                                            L("inputs", "(int64_t)cl_n * cl_a", "buf_size", count_err=ILL,
                                              exact=True, nulls=True, when="cl_ne > 0"),
                                            L("outputs", "(int64_t)cl_ne * cl_a", "buf_size", count_err=ILL,
                                              exact=True, when="cl_ne > 0")]),
    "ecx_clay_decode_single_helper": (("clay",), [NN("buf_size"),
                                                  L("helper_coupled", "(int64_t)(cl_a / (cl_q > 0 ? cl_q : 1)) * cl_n",
                                                    "buf_size", nulls=True),
                                                  L("outputs", "cl_a", "buf_size", nulls=True)]),
    "ecx_lrc_map": ((), [A("block_present", "16")]),
    "ecx_lrc_decode_batch": ((), [A("block_present", "16")]),
    "ecx_map_apply_batch_host_devices": ((), [NN("ndev"), A("devices", "ndev", err=ILL)]),
    "ecx_clay_perform_coding_batch_host_devices": ((), [NN("ndev"), A("devices", "ndev", err=ILL)]),
    "ecx_rs_is_parity_correct_batch_host_devices": ((), [NN("ndev"), A("devices", "ndev", err=ILL)]),
    "ecx_rs_decode_missing_blocked_batch_host": (("rs",), [A("shard_present", RS_N)]),
    "ecx_rs_encode_parity_blocked_batch_host_devices": ((), [NN("ndev"), A("devices", "ndev", err=ILL)]),
    "ecx_rs_decode_missing_blocked_batch_host_devices": (("rs",), [A("shard_present", RS_N), NN("ndev"),
                                                                   A("devices", "ndev", err=ILL)]),
}


# Host-batch exports that also get a ByteBuffer forwarder, <camel>Buffer: the buffers are
# direct ByteBuffers whose address AND capacity the forwarder reads itself, so the extent
# check cannot be skipped from Java.  export -> (handle query, extent source, condition
# under which the export touches the buffers at all).
BUFFER_VARIANTS = {
    "ecx_map_apply_batch_host": ("map", "    if (st == ECX_OK) st = ecx_map_slot_extent((const ecx_map *)(intptr_t)map, &max_in, &max_out);",
                                 None),
    # performCoding returns before its checks when nothing is erased (ClayCodeErasureDecodingStep.java:54-56)
    "ecx_clay_perform_coding_batch_host": ("clay", "    if (st == ECX_OK && cl_ne > 0) {\n"
                                           "        const ecx_map *cm = NULL;\n"
                                           "        st = ecx_clay_map((ecx_clay *)(intptr_t)clay, &cm);\n"
                                           "        if (st == ECX_OK) st = ecx_map_slot_extent(cm, &max_in, &max_out);\n"
                                           "    }", "cl_ne > 0"),
}
# The host check batch: the stripes (every shard read, max slot n - 1, bytes up to offset +
# byte_count) and a verdict buffer of one byte per stripe.
BUFFER_VARIANTS["ecx_rs_is_parity_correct_batch_host"] = ("rs", "    max_in = rs_k + rs_m - 1;", None)
# the multi-GPU forms take the same buffers, extents and conditions
BUFFER_VARIANTS["ecx_map_apply_batch_host_devices"] = BUFFER_VARIANTS["ecx_map_apply_batch_host"]
BUFFER_VARIANTS["ecx_clay_perform_coding_batch_host_devices"] = BUFFER_VARIANTS["ecx_clay_perform_coding_batch_host"]
BUFFER_VARIANTS["ecx_rs_is_parity_correct_batch_host_devices"] = BUFFER_VARIANTS["ecx_rs_is_parity_correct_batch_host"]
# The blocked RS batches from host memory: one buffer of nstripes whole stripes (n * byte_count
# bytes each, the body and the tails together), the stripe size overflow-checked first.
BLOCKED_EXTENT = ("    int64_t stripe_bytes = 0;\n"
                  "    if (st == ECX_OK && __builtin_mul_overflow((int64_t)rs_k + rs_m, byte_count, &stripe_bytes))\n"
                  "        st = ECX_E_ILLEGAL_ARGUMENT;\n"
                  "    max_in = 0;")
BUFFER_VARIANTS["ecx_rs_encode_parity_blocked_batch_host"] = ("rs", BLOCKED_EXTENT, None)
BUFFER_VARIANTS["ecx_rs_decode_missing_blocked_batch_host"] = ("rs", BLOCKED_EXTENT, None)
BUFFER_VARIANTS["ecx_rs_encode_parity_blocked_batch_host_devices"] = ("rs", BLOCKED_EXTENT, None)
BUFFER_VARIANTS["ecx_rs_decode_missing_blocked_batch_host_devices"] = ("rs", BLOCKED_EXTENT, None)
# buffers laid out other than (stripe stride, slot stride) after the address: param (or (export,
# param)) -> (stripe stride, slot stride, max slot, bytes per slot), as C expressions
BUFFER_SHAPES = {"verdict": ("1", "0", "0", "1"),
                 ("ecx_rs_encode_parity_blocked_batch_host", "base"): ("stripe_bytes", "0", "0", "stripe_bytes"),
                 ("ecx_rs_decode_missing_blocked_batch_host", "base"): ("stripe_bytes", "0", "0", "stripe_bytes"),
                 ("ecx_rs_encode_parity_blocked_batch_host_devices", "base"): ("stripe_bytes", "0", "0", "stripe_bytes"),
                 ("ecx_rs_decode_missing_blocked_batch_host_devices", "base"): ("stripe_bytes", "0", "0",
                                                                                "stripe_bytes")}


def host_address_native(name):
    """Host-batch exports whose buffers are raw host addresses (longs): their natives are
    package-private, so Java callers outside com.backblaze.erasure.ecx reach them only
    through the capacity-checked <camel>Buffer forwarders (ClayCoordinator.kt:378-390)."""
    return "_batch_host" in name


def copied(name, kind, ctype):
    """A read-only array argument the forwarder copies instead of pinning: every const int[], and
    the const byte[] flags of a host batch (which runs for as long as its PCIe transfers)."""
    if not ctype.startswith("const"):
        return False
    return kind == "ints" or (kind == "bytes" and host_address_native(name))


def buffer_variant(ret, name, params):
    """The <camel>Buffer forwarder of a host-batch export (BUFFER_VARIANTS)."""
    query, extent, when = BUFFER_VARIANTS[name]
    names = [p for _, p in params]
    handle = names[0]
    length = next(p for p in reversed(names) if p in ("byte_count", "buf_size"))
    negative = "nstripes < 0 || %s < 0" % length
    if "offset" in names:  # a window [offset, offset + byte_count) of every slot
        negative += " || offset < 0"
        length = "(int64_t)offset + %s" % length
    jparams, cparams, args, bufs, ints, flags = [], ["JNIEnv *env", "jclass cls"], [], [], [], []
    for i, (t, p) in enumerate(params):
        kind = classify(name, t, p)[0]
        if kind == "int":
            jparams.append("int %s" % camel("ecx_" + p))
            cparams.append("jint %s" % p)
            args.append("(int)%s" % p)
        elif kind == "ints":  # copied out of the Java array (no critical region), length-checked
            jparams.append("int[] %s" % camel("ecx_" + p))
            cparams.append("jintArray %s" % p)
            ints.append((p, names[i + 1]))
            args.append("%s_c" % p)
        elif kind == "bytes":  # a *_present flag array: copied out (no critical region), length-checked
            jparams.append("byte[] %s" % camel("ecx_" + p))
            cparams.append("jbyteArray %s" % p)
            flags.append((p, dict((r[1], r[2]) for r in RULES[name][1] if r[0] == "array")[p]))
            args.append("%s_c" % p)
        elif kind == "addr":
            jparams.append("ByteBuffer %s" % camel("ecx_" + p))
            cparams.append("jobject %s" % p)
            if (name, p) in BUFFER_SHAPES:
                bufs.append((p,) + BUFFER_SHAPES[(name, p)])
            elif p in BUFFER_SHAPES:
                bufs.append((p,) + BUFFER_SHAPES[p])
            else:  # (stripe stride, slot stride) follow; the map's slots; the batch's bytes per slot
                bufs.append((p, names[i + 1], names[i + 2], "max_in" if p in ("in", "base") else "max_out", length))
            args.append("(%s)%s_p" % (t.strip(), p))
        elif kind == "handle":
            jparams.append("long %s" % camel("ecx_" + p))
            cparams.append("jlong %s" % p)
            args.append("(%s)(intptr_t)%s" % (t.strip(), p))
        else:
            jparams.append("long %s" % camel("ecx_" + p))
            cparams.append("jlong %s" % p)
            args.append("(int64_t)%s" % p)
    body = ["    (void)cls;", "    jint st = ECX_OK;", "    if (!%s) st = ECX_E_NULL;" % handle,
            "    if (st == ECX_OK && (%s)) st = ECX_E_ILLEGAL_ARGUMENT;" % negative,
            QUERIES[query], "    int max_in = -1, max_out = -1;", extent, "    (void)max_in;", "    (void)max_out;"]
    for b in bufs:
        body.append("    uint8_t *%s_p = NULL;" % b[0])
    cond = "st == ECX_OK" + (" && (%s)" % when if when else "")
    for p, ss, sl, ms, nb in bufs:
        body.append("    if (%s) st = direct_check(env, %s, %s, %s, %s, nstripes, %s, &%s_p);"
                    % (cond, p, ss, sl, ms, nb, p))
    for p, cnt in ints:
        body.append("    int *%s_c = NULL;" % p)
        body.append("    if (st == ECX_OK && %s < 0) st = ECX_E_ILLEGAL_ARGUMENT;" % cnt)
        body.append("    if (st == ECX_OK) st = array_check(env, %s, %s, 0, ECX_E_ILLEGAL_ARGUMENT);" % (p, cnt))
        body.append("    if (st == ECX_OK && !(%s_c = (int *)malloc(sizeof(int) * ((size_t)%s + 1)))) st = ECX_E_NOMEM;"
                    % (p, cnt))
        body.append("    if (st == ECX_OK) (*env)->GetIntArrayRegion(env, %s, 0, %s, (jint *)%s_c);" % (p, cnt, p))
    for p, need in flags:
        body.append("    uint8_t *%s_c = NULL;" % p)
        body.append("    if (st == ECX_OK) st = array_check(env, %s, %s, 0, ECX_E_INDEX);" % (p, need))
        body.append("    if (st == ECX_OK && !(%s_c = (uint8_t *)malloc((size_t)(%s) + 1))) st = ECX_E_NOMEM;"
                    % (p, need))
        body.append("    if (st == ECX_OK) (*env)->GetByteArrayRegion(env, %s, 0, (jsize)(%s), (jbyte *)%s_c);"
                    % (p, need, p))
    body.append("    if (st == ECX_OK) st = %s(%s);" % (name, ", ".join(args)))
    for p, _ in ints + flags:
        body.append("    free(%s_c);" % p)
    body.append("    return st;")
    jname = camel(name) + "Buffer"
    c = ("\n/* %s over direct ByteBuffers, extent-checked from their capacity */\n"
         "JNIEXPORT jint JNICALL Java_%s_%s(%s) {\n%s\n}\n"
         % (name, JCLASS, jname, ", ".join(cparams), "\n".join(body)))
    java = ("\n    /** %s over direct ByteBuffers: the forwarder checks each buffer's capacity against the\n"
            "     *  batch extent and refuses heap buffers (NullPointerException). */\n"
            "    public static native int %s(%s);\n" % (name, jname, ", ".join(jparams)))
    return c, java


def exports():
    src = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    out = []
    for m in re.finditer(r"^\s*((?:const\s+)?[a-z_0-9]+\s*\**)\s*(ecx_[a-z0-9_]+)\s*\(([^;]*?)\);", src,
                         flags=re.M | re.S):
        ret, name, args = m.group(1).replace(" ", ""), m.group(2), " ".join(m.group(3).split())
        params = []
        if args != "void":
            for a in args.split(","):
                a = a.strip()
                pm = re.match(r"(.*?)([A-Za-z_][A-Za-z_0-9]*)$", a)
                params.append((" ".join(pm.group(1).split()), pm.group(2)))
        out.append((ret, name, params))
    return out


def camel(name):
    parts = name[len("ecx_"):].split("_")
    return parts[0] + "".join(p.capitalize() for p in parts[1:])


def is_address_fn(name):
    return "batch" in name or name in ("ecx_fill_random", "ecx_count_mismatch")


def classify(fn, ctype, pname):
    """(kind, java type, jni type) of one C parameter."""
    t = ctype.replace(" ", "")
    base = t.replace("const", "")
    if base in ("int",):
        return "int", "int", "jint"
    if base in ("int64_t",):
        return "i64", "long", "jlong"
    if base in ("uint64_t",):
        return "u64", "long", "jlong"
    if any(base == h + "*" for h in HANDLES):
        return "handle", "long", "jlong"
    if any(base == h + "**" for h in HANDLES) or base == "void**":
        return "outhandle", "long[]", "jlongArray"
    if base == "void*":
        return "addr", "long", "jlong"
    if base == "uint64_t*":
        return "addr", "long", "jlong"
    if base in ("uint8_t*const*", "uint8_t**"):
        return "buflist", "byte[][]", "jobjectArray"
    if base == "uint8_t*":
        if is_address_fn(fn) and not pname.endswith("_present"):
            return "addr", "long", "jlong"
        return "bytes", "byte[]", "jbyteArray"
    if base == "int*":
        return "ints", "int[]", "jintArray"
    if base == "int64_t*":
        return "longs", "long[]", "jlongArray"
    if base == "int16_t*":
        return "shorts", "short[]", "jshortArray"
    raise SystemExit("unmapped parameter type %r of %s" % (ctype, fn))


def gen():
    c, java = [], []
    c.append("""/*
 * ecx_jni.c -- JNI binding of libecx.so (include/ecx.h) for the reference's JVM code.
 * GENERATED by jni/gen_jni.py from include/ecx.h: one forwarder per export, each
 * calling the export with exactly its parameters.  Java side:
 * com.backblaze.erasure.ecx.EcxNative (same generator); the Java classes built on it
 * (EcxCodingLoop, EcxClayCodeErasureDecodingStep, EcxPartialSums) are in jni/.
 * Build: make -C jni (needs JAVA_HOME for jni.h; links -lecx).
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "ecx.h"

/* byte[][] + per-buffer start positions -> pinned host pointers (NULL for null
 * elements).  Phase 1 (refs) runs JNI calls; phase 2 (pin) only critical pins. */
typedef struct {
    jsize n;
    jbyteArray *refs;
    jint *pos;
    jsize *lens;
    uint8_t **ptrs;
} ecx_jni_buflist;

static int buflist_refs(JNIEnv *env, jobjectArray arr, jintArray positions, ecx_jni_buflist *b) {
    b->n = arr ? (*env)->GetArrayLength(env, arr) : 0;
    b->refs = (jbyteArray *)calloc((size_t)b->n + 1, sizeof(jbyteArray));
    b->pos = (jint *)calloc((size_t)b->n + 1, sizeof(jint));
    b->lens = (jsize *)calloc((size_t)b->n + 1, sizeof(jsize));
    b->ptrs = (uint8_t **)calloc((size_t)b->n + 1, sizeof(uint8_t *));
    if (!b->refs || !b->pos || !b->lens || !b->ptrs) return ECX_E_NOMEM;
    for (jsize i = 0; i < b->n; ++i) {
        b->refs[i] = (jbyteArray)(*env)->GetObjectArrayElement(env, arr, i);
        b->lens[i] = b->refs[i] ? (*env)->GetArrayLength(env, b->refs[i]) : 0;
    }
    if (positions) {
        if ((*env)->GetArrayLength(env, positions) < b->n) return ECX_E_ILLEGAL_ARGUMENT;
        (*env)->GetIntArrayRegion(env, positions, 0, b->n, b->pos);
    }
    return ECX_OK;
}

/* A byte[][] the export reads `count` entries of: at least `count` entries (exactly,
 * with `exact`), entry i < count non-null unless `nulls`, pos[i] >= 0 and
 * pos[i] + need <= its length.  Runs before anything is pinned. */
static int buflist_check(const ecx_jni_buflist *b, jobjectArray arr, int64_t count, int64_t need, int exact,
                         int nulls, int count_err, int len_err) {
    if (count < 0) return ECX_E_ILLEGAL_ARGUMENT;
    if (!arr) return count > 0 ? ECX_E_NULL : ECX_OK;
    if (exact ? (int64_t)b->n != count : (int64_t)b->n < count) return count_err;
    if (need < 0) need = 0;
    for (int64_t i = 0; i < count; ++i) {
        if (!b->refs[i]) {
            if (nulls) continue;
            return ECX_E_NULL;
        }
        if (b->pos[i] < 0 || (int64_t)b->pos[i] + need > (int64_t)b->lens[i]) return len_err;
    }
    return ECX_OK;
}

/* A primitive array the export touches `need` elements of (null: NullPointerException
 * unless the export accepts NULL). */
static int array_check(JNIEnv *env, jarray arr, int64_t need, int nullable, int err) {
    if (!arr) return nullable ? ECX_OK : ECX_E_NULL;
    if (need < 0) return ECX_E_ILLEGAL_ARGUMENT;
    return (int64_t)(*env)->GetArrayLength(env, arr) < need ? err : ECX_OK;
}

static int buflist_pin(JNIEnv *env, ecx_jni_buflist *b) {
    for (jsize i = 0; i < b->n; ++i) {
        if (!b->refs[i]) continue;
        uint8_t *p = (uint8_t *)(*env)->GetPrimitiveArrayCritical(env, b->refs[i], NULL);
        if (!p) return ECX_E_NOMEM;
        b->ptrs[i] = p + b->pos[i];
    }
    return ECX_OK;
}

static void buflist_unpin(JNIEnv *env, ecx_jni_buflist *b, jint mode) {
    for (jsize i = b->n; i-- > 0;)
        if (b->refs[i] && b->ptrs[i]) (*env)->ReleasePrimitiveArrayCritical(env, b->refs[i], b->ptrs[i] - b->pos[i], mode);
}

static void buflist_free(JNIEnv *env, ecx_jni_buflist *b) {
    for (jsize i = 0; i < b->n; ++i)
        if (b->refs && b->refs[i]) (*env)->DeleteLocalRef(env, b->refs[i]);
    free(b->refs);
    free(b->pos);
    free(b->lens);
    free(b->ptrs);
}

#define PIN(arr) ((arr) ? (*env)->GetPrimitiveArrayCritical(env, (arr), NULL) : NULL)
#define UNPIN(arr, p, mode) do { if ((arr) && (p)) (*env)->ReleasePrimitiveArrayCritical(env, (arr), (p), (mode)); } while (0)

/* A direct ByteBuffer a host-batch call reads or writes (nstripes-1)*stripe_stride +
 * max_slot*slot_stride + nbytes bytes of, from its address (ecx_map_slot_extent): null or a
 * heap buffer (no address, capacity -1) -> NullPointerException; negative strides ->
 * IllegalArgumentException; shorter than that -> ArrayIndexOutOfBoundsException, as the
 * reference's ByteBuffer get/put would throw (ClayCoordinator.kt:378-390). */
static int direct_check(JNIEnv *env, jobject buf, int64_t stripe_stride, int64_t slot_stride, int max_slot,
                        int64_t nstripes, int64_t nbytes, uint8_t **addr) {
    *addr = NULL;
    if (!buf) return ECX_E_NULL;
    uint8_t *p = (uint8_t *)(*env)->GetDirectBufferAddress(env, buf);
    const jlong cap = (*env)->GetDirectBufferCapacity(env, buf);
    if (!p || cap < 0) return ECX_E_NULL;
    *addr = p;
    if (nstripes <= 0 || nbytes <= 0 || max_slot < 0) return ECX_OK;
    if (stripe_stride < 0 || slot_stride < 0) return ECX_E_ILLEGAL_ARGUMENT;
    int64_t a = 0, b = 0, need = 0;
    if (__builtin_mul_overflow(nstripes - 1, stripe_stride, &a) ||
        __builtin_mul_overflow((int64_t)max_slot, slot_stride, &b) || __builtin_add_overflow(a, b, &need) ||
        __builtin_add_overflow(need, nbytes, &need))
        return ECX_E_INDEX;
    return need > (int64_t)cap ? ECX_E_INDEX : ECX_OK;
}

/* Address of a direct ByteBuffer (package-private on the Java side: host-batch callers use
 * the capacity-checked ByteBuffer forwarders). */
JNIEXPORT jlong JNICALL Java_%(J)s_directAddress(JNIEnv *env, jclass cls, jobject buffer) {
    (void)cls;
    return (jlong)(intptr_t)(*env)->GetDirectBufferAddress(env, buffer);
}

/* A direct ByteBuffer over host memory, e.g. pinned memory from ecx_host_alloc. */
JNIEXPORT jobject JNICALL Java_%(J)s_wrapAddress(JNIEnv *env, jclass cls, jlong address, jlong nbytes) {
    (void)cls;
    return (*env)->NewDirectByteBuffer(env, (void *)(intptr_t)address, nbytes);
}
""" % {"J": JCLASS})
    java.append("""package com.backblaze.erasure.ecx;

import java.nio.ByteBuffer;

/**
 * JNI declarations of libecx.so (include/ecx.h), GENERATED by jni/gen_jni.py: one
 * native per export, same parameters in the same order (types per gen_jni.py).
 * Status codes are the return values; {@link Ecx#check} turns them into the Java
 * exceptions the reference throws.
 */
public final class EcxNative {
    static {
        System.loadLibrary("ecxjni");
    }

    private EcxNative() {
    }

    /** Address of a direct ByteBuffer.  Package-private: outside this package host batches
     *  go through the capacity-checked ByteBuffer forwarders. */
    static native long directAddress(ByteBuffer buffer);

    /** A direct ByteBuffer over host memory.  Package-private (a caller-chosen capacity would
     *  defeat the forwarders' extent checks): use {@link Ecx#allocatePinned}. */
    static native ByteBuffer wrapAddress(long address, long nbytes);
""")
    for ret, name, params in exports():
        jname = camel(name)
        kinds = [(classify(name, t, p), t, p) for t, p in params]
        jparams, cparams = [], ["JNIEnv *env", "jclass cls"]
        for (kind, jt, jnt), t, p in kinds:
            jparams.append("%s %s" % (jt, camel("ecx_" + p)))
            cparams.append("%s %s" % (jnt, p))
            if kind == "buflist":
                jparams.append("int[] %sPositions" % camel("ecx_" + p))
                cparams.append("jintArray %s_positions" % p)
        jret = {"constchar*": "String", "int": "int", "void": "void"}[ret]
        cret = {"constchar*": "jstring", "int": "jint", "void": "void"}[ret]
        vis = "" if host_address_native(name) else "public "
        if vis == "":
            java.append("\n    /** Raw host addresses: package-private (use %sBuffer). */" % jname)
        java.append("\n    %sstatic native %s %s(%s);\n" % (vis, jret, jname, ", ".join(jparams)))
        body = []
        pre, copies, pin, unpin, post, args = [], [], [], [], [], []
        pnames = {p: kind for (kind, _, _), t, p in kinds}
        needs_rule = [p for p, k in pnames.items() if k in ("bytes", "ints", "shorts", "longs", "buflist")]
        if needs_rule and name not in RULES:
            raise SystemExit("no argument rule for %s (pointer parameters %s)" % (name, needs_rule))
        queries, rules = RULES.get(name, ((), []))
        covered = {r[1] for r in rules if r[0] in ("array", "list")}
        if set(needs_rule) - covered:
            raise SystemExit("%s: no rule for %s" % (name, sorted(set(needs_rule) - covered)))
        checks = []
        if not name.endswith("_destroy"):
            for p, k in pnames.items():
                if k == "handle":
                    checks.append("    if (st == ECX_OK && !%s) st = ECX_E_NULL;" % p)
        for r in rules:
            if r[0] == "nonneg":
                for p in r[1]:
                    checks.append("    if (st == ECX_OK && %s < 0) st = %s;" % (p, r[2]))
        for q in queries:
            checks.append(QUERIES[q])
        late = []  # after the buffer lists' references are taken, before pinning
        for r in rules:
            if r[0] == "array":
                _, p, need, err = r
                late.append("    if (st == ECX_OK) st = array_check(env, %s, %s, %d, %s);"
                            % (p, need, 1 if (name, p) in NULLABLE else 0, err))
            elif r[0] == "list":
                _, p, count, need, cerr, lerr, exact, nulls, when = r
                cond = "st == ECX_OK" + (" && (%s)" % when if when else "")
                late.append("    if (%s) st = buflist_check(&%s_b, %s, %s, %s, %d, %d, %s, %s);"
                            % (cond, p, p, count, need, int(exact), int(nulls), cerr, lerr))
        for (kind, _, _), t, p in kinds:
            if kind == "outhandle":
                late.append("    if (st == ECX_OK) st = array_check(env, %s, 1, 0, ECX_E_INDEX);" % p)
        for (kind, jt, jnt), t, p in kinds:
            ct = t.replace("const ", "const ").strip()
            if kind == "int":
                args.append("(int)%s" % p)
            elif kind == "i64":
                args.append("(int64_t)%s" % p)
            elif kind == "u64":
                args.append("(uint64_t)%s" % p)
            elif kind in ("handle", "addr"):
                args.append("(%s)(intptr_t)%s" % (ct, p))
            elif kind == "outhandle":
                hb = ct.replace("**", "*").strip()
                pre.append("    %s %s_h = NULL;" % (hb, p))
                args.append("&%s_h" % p)
                post.append("    if (st >= 0 && %s) { jlong v = (jlong)(intptr_t)%s_h; (*env)->SetLongArrayRegion(env, %s, 0, 1, &v); }"
                            % (p, p, p))
            elif copied(name, kind, t):
                # read-only int[] (device lists, slots, erased indices) and the flag byte[] of a
                # host batch: copied out of the Java array before any critical region opens, never
                # pinned, so a long export (a host batch) holds no GC-blocking pin
                # ("pinning")
                need = next(r[2] for r in rules if r[0] == "array" and r[1] == p)
                cty, jty, get = (("int", "jint", "GetIntArrayRegion") if kind == "ints" else
                                 ("uint8_t", "jbyte", "GetByteArrayRegion"))
                pre.append("    %s *%s_p = NULL;" % (cty, p))
                copies.append("    if (st == ECX_OK && %s && !(%s_p = (%s *)malloc(sizeof(%s) * ((size_t)(%s) + 1))))"
                              " st = ECX_E_NOMEM;" % (p, p, cty, cty, need))
                copies.append("    if (st == ECX_OK && %s) (*env)->%s(env, %s, 0, (jsize)(%s), (%s *)%s_p);"
                              % (p, get, p, need, jty, p))
                post.append("    free(%s_p);" % p)
                args.append("%s_p" % p)
            elif kind in ("bytes", "ints", "shorts", "longs"):
                cty = {"bytes": "uint8_t", "ints": "int", "shorts": "int16_t", "longs": "int64_t"}[kind]
                mode = "JNI_ABORT" if t.startswith("const") else "0"
                pre.append("    %s *%s_p = NULL;" % (cty, p))
                pin.append("    if (st == ECX_OK) %s_p = (%s *)PIN(%s);" % (p, cty, p))
                unpin.insert(0, "    UNPIN(%s, %s_p, %s);" % (p, p, mode))
                args.append("%s_p" % p)
            elif kind == "buflist":
                mode = "JNI_ABORT" if t.startswith("const") else "0"
                pre.append("    ecx_jni_buflist %s_b = {0, NULL, NULL, NULL, NULL};" % p)
                pre.append("    if (st == ECX_OK) st = buflist_refs(env, %s, %s_positions, &%s_b);" % (p, p, p))
                pin.append("    if (st == ECX_OK) st = buflist_pin(env, &%s_b);" % p)
                unpin.insert(0, "    buflist_unpin(env, &%s_b, %s);" % (p, mode))
                post.append("    buflist_free(env, &%s_b);" % p)
                cast = "(const uint8_t *const *)" if t.startswith("const") else "(uint8_t *const *)"
                args.append("%s%s_b.ptrs" % (cast, p))
        call = "%s(%s)" % (name, ", ".join(args))
        if ret == "constchar*":
            body.append("    (void)cls;")
            body.append("    const char *s = %s;" % call)
            body.append("    return s ? (*env)->NewStringUTF(env, s) : NULL;")
        elif ret == "void":
            body.append("    (void)env;")
            body.append("    (void)cls;")
            body.append("    %s;" % call)
        else:
            body.append("    (void)cls;")
            body.append("    jint st = ECX_OK;")
            body.extend(checks)
            body.extend(pre)
            body.extend(late)
            body.extend(copies)
            body.extend(pin)
            pinned = [ln for ln in pin]
            if pinned:
                # every PIN that returned NULL for a non-null array is an allocation failure
                checks = ["(%s && !%s_p)" % (p, p) for (kind, _, _), t, p in kinds
                          if kind in ("bytes", "ints", "shorts", "longs") and not copied(name, kind, t)]
                if checks:
                    body.append("    if (st == ECX_OK && (%s)) st = ECX_E_NOMEM;" % " || ".join(checks))
            body.append("    if (st == ECX_OK) st = %s;" % call)
            body.extend(unpin)
            body.extend(post)
            body.append("    return st;")
        c.append("\n/* %s */\nJNIEXPORT %s JNICALL Java_%s_%s(%s) {\n%s\n}\n"
                 % (name, cret, JCLASS, jname, ", ".join(cparams), "\n".join(body)))
        if name in BUFFER_VARIANTS:
            bc, bj = buffer_variant(ret, name, params)
            c.append(bc)
            java.append(bj)
    java.append("}\n")
    return "".join(c), "".join(java)


def main(check=False):
    c, java = gen()
    if check:
        return OUT_C.read_text() == c and OUT_JAVA.read_text() == java
    OUT_JAVA.parent.mkdir(parents=True, exist_ok=True)
    OUT_C.write_text(c)
    OUT_JAVA.write_text(java)
    return True


if __name__ == "__main__":
    sys.exit(0 if main("--check" in sys.argv) else 1)
