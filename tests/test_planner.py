"""Host-planner parity on CPU: the composed GF(256) maps that the HIP kernels
apply, applied here in numpy, must reproduce the oracle's stage-by-stage
restatement of the reference on the same (random, non-codeword) inputs.
This pins the planner independently of the GPU; tests/test_gpu_parity.py then
pins the kernels against the same oracle."""
from pathlib import Path

import numpy as np
import pytest

import oracle as O
from conftest import gf_apply_numpy, shortened_clay_oracle as _shortened_oracle

ROOT = Path(__file__).resolve().parents[1]


def test_field_tables_match_reference(ecx, kats):
    log, exp, mul = ecx.Galois.tables()
    g = kats["galois"]
    assert log.tolist() == g["log_table"]
    assert exp.tolist() == g["exp_table"]
    assert (mul == O.mul_table()).all()
    for a, b, r in g["multiply"]:
        assert ecx.Galois.multiply(a, b) == r
    for a, n, r in g["exp"]:
        assert ecx.Galois.exp(a, n) == r


def test_matrix_kats(ecx, kats):
    t = kats["matrix"]["times"]
    assert ecx.Matrix.times(t["a"], t["b"]).tolist() == t["out"]
    for case in kats["matrix"]["invert"]:
        assert ecx.Matrix.invert(case["m"]).tolist() == case["inv"]


def test_rs_generator_matrix(ecx, kats):
    for key, rows in kats["rs_parity_rows"].items():
        if key == "17,3_row0":
            assert ecx.ReedSolomon.create(17, 3).parityRows[0].tolist() == rows
        else:
            k, m = map(int, key.split(","))
            assert ecx.ReedSolomon.create(k, m).parityRows.tolist() == rows
    for k, m in [(5, 5), (64, 64), (10, 4)]:
        assert (ecx.ReedSolomon.create(k, m).matrix == O.ReedSolomon(k, m).matrix).all()


@pytest.mark.parametrize("k,m,present", [
    (4, 2, [1, 0, 1, 1, 1, 1]), (4, 2, [0, 1, 1, 0, 1, 1]), (4, 2, [1, 1, 1, 1, 0, 0]),
    (4, 2, [1, 1, 0, 1, 0, 1]), (12, 4, [0, 0] + [1] * 14), (5, 5, [0, 1, 0, 1, 0, 1, 1, 1, 1, 1]),
    (3, 1, [1, 1, 0, 1]),
])
def test_rs_decode_map_vs_oracle(ecx, k, m, present):
    """decodeMissing's composed map on NON-codeword shards == the oracle (first-k-present rule)."""
    rng = np.random.default_rng(k * 31 + m)
    L = 64
    shards = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k + m)]
    ref = [s.copy() for s in shards]
    O.ReedSolomon(k, m).decode_missing(ref, [bool(p) for p in present], 0, L)
    mat, ins, outs = ecx.ReedSolomon.create(k, m).decode_map([bool(p) for p in present]).matrix()
    got = gf_apply_numpy(mat, [shards[j] for j in ins])
    for o, slot in enumerate(outs):
        assert (got[o] == ref[slot]).all()
    assert sorted(outs.tolist()) == [i for i in range(k + m) if not present[i]]


def _oracle_perform(k, m, erased, inputs, B):
    c = O.Clay(k, m, erased)
    outs = [np.zeros(B, np.uint8) for _ in range(len(erased) * c.alpha)]
    c.perform_coding(inputs, outs, B)
    return outs


CLAY_CASES = [(2, 2, [0]), (2, 2, [3]), (4, 2, [0]), (4, 2, [1]), (4, 2, [2]), (4, 2, [3]), (4, 2, [4]),
              (4, 2, [5]), (4, 2, [4, 5]), (4, 2, [0, 1]), (4, 2, [1, 4]), (6, 3, [2]), (6, 3, [6, 7, 8]),
              (6, 3, [0, 4]), (12, 4, [5]), (12, 4, [12, 13, 14, 15]), (12, 4, [0, 15])]


@pytest.mark.parametrize("k,m,erased", CLAY_CASES)
def test_clay_map_vs_oracle_random_inputs(ecx, k, m, erased):
    """The composed Clay map equals the reference stage sequence on random (non-codeword) inputs."""
    n = k + m
    step = ecx.ClayCodeErasureDecodingStep(erased, k, m)
    a = step.subPacketSize
    B = 8 if a >= 64 else 24
    rng = np.random.default_rng(sum(erased) + 7 * k)
    inputs = [None if (i % n) in erased else rng.integers(0, 256, B, dtype=np.uint8) for i in range(n * a)]
    ref = _oracle_perform(k, m, erased, inputs, B)
    mat, ins, outs = step.map().matrix()
    got = gf_apply_numpy(mat, [inputs[j] for j in ins])
    assert outs.tolist() == list(range(len(erased) * a))
    for o in range(len(outs)):
        assert (got[o] == ref[o]).all(), o


def test_clay42_map_shape(ecx):
    """Clay(4,2) single repair is an 8 x 20 map with 52 non-zeros
    for every erased node; the encode map is 16 x 32 with 144 non-zeros."""
    for e in range(6):
        inf = ecx.ClayCodeErasureDecodingStep([e], 4, 2).map().info()
        assert (inf["n_out"], inf["n_in"], inf["nnz"]) == (8, 20, 52)
    inf = ecx.ClayCodeErasureDecodingStep([4, 5], 4, 2).map().info()
    assert (inf["n_out"], inf["n_in"], inf["nnz"]) == (16, 32, 144)


A3_E1_COEFFS = {143, 104, 208, 52, 187, 210, 107, 92, 105, 184, 109, 189, 185, 214}


def _probe_oracle_repair_map(k, m, e, ins):
    """The oracle's single-repair map, read off by unit vectors: byte position j of
    input slot ins[j] is 1, every other helper byte 0 (GF linearity per byte
    position), so output byte j of row o is the coefficient M[o][j]."""
    n, nin = k + m, len(ins)
    c = O.Clay(k, m, [e])
    inputs = [None if (i % n) == e else np.zeros(nin, np.uint8) for i in range(n * c.alpha)]
    for j, slot in enumerate(ins):
        inputs[slot][j] = 1
    outs = [np.zeros(nin, np.uint8) for _ in range(c.alpha)]
    c.perform_coding(inputs, outs, nin)
    return np.stack(outs)


def test_clay42_repair_map_pinned_to_survey_a3(ecx):
    """SURVEY.md A.3, the survey's independent scratch restatement of
    ClayCodeErasureDecodingStep.java:435-492,630-666 (the non-codeword repair map, H2):
    the e=1 Clay(4,2) single repair has exactly the 14 distinct coefficients
    {143,104,208,52,187,210,107,92,105,184,109,189,185,214}, and every e has 52
    non-zeros with 6-7 per row.  Asserted on the planner's composed map
    (ecx_clay_map) and on the oracle probed with unit vectors; the two must also be
    the same matrix."""
    for e in range(6):
        mat, ins, outs = ecx.ClayCodeErasureDecodingStep([e], 4, 2).map().matrix()
        probed = _probe_oracle_repair_map(4, 2, e, ins.tolist())
        assert (probed == mat).all(), e
        for mm in (mat, probed):
            nnz = (mm != 0).sum(1)
            assert mm.shape == (8, 20) and int(nnz.sum()) == 52 and set(nnz.tolist()) <= {6, 7}, e
        if e == 1:
            assert set(mat[mat != 0].tolist()) == A3_E1_COEFFS
            assert set(probed[probed != 0].tolist()) == A3_E1_COEFFS


def _probe_oracle_map(k, m, erased, ins):
    """The oracle's performCoding map for the standard null pattern, read off by unit
    vectors (byte j of input slot ins[j] is 1, every other byte 0)."""
    n, nin = k + m, len(ins)
    c = O.Clay(k, m, list(erased))
    inputs = [None if (i % n) in erased else np.zeros(nin, np.uint8) for i in range(n * c.alpha)]
    for j, slot in enumerate(ins):
        inputs[slot][j] = 1
    outs = [np.zeros(nin, np.uint8) for _ in range(len(erased) * c.alpha)]
    c.perform_coding(inputs, outs, nin)
    return np.stack(outs)


@pytest.mark.parametrize("name,erased", [("repair_e1", [1]), ("repair_e4", [4]), ("encode_45", [4, 5])])
def test_clay42_maps_equal_closed_form(ecx, name, erased):
    """An independent pin against a shared misreading of ClayCodeErasureDecodingStep.java
    by the planner and the oracle (both restate its stage sequence): the full Clay(4,2)
    repair maps of nodes 1 and 4 (8 x 20) and the encode map (16 x 32), derived in closed
    form from the pair-transform equations, the helper-plane set and the RS(4,2)
    generator alone (tests/golden/gen_clay42_maps.py, committed as
    tests/golden/clay42_closed_form.json), equal entry for entry the planner's composed map
    (ecx_clay_map) and the oracle's, read off by unit vectors."""
    import json
    d = json.loads((ROOT / "tests" / "golden" / "clay42_closed_form.json").read_text())[name]
    want = {(o, i): c for o, i, c in zip(d["out"], d["in"], d["coef"])}
    mat, ins, outs = ecx.ClayCodeErasureDecodingStep(erased, 4, 2).map().matrix()
    probed = _probe_oracle_map(4, 2, erased, ins.tolist())
    for mm in (mat, probed):
        got = {(int(outs[o]), int(ins[i])): int(mm[o, i]) for o in range(mm.shape[0]) for i in range(mm.shape[1])
               if mm[o, i]}
        assert got == want
    assert d["nnz"] == (144 if name == "encode_45" else 52)


@pytest.mark.parametrize("k,m,v,e", [(12, 4, 0, 5), (12, 4, 0, 14), (10, 4, 2, 3), (10, 4, 2, 13)])
def test_clay_q4_repair_maps_equal_closed_form(ecx, k, m, v, e):
    """The same independent pin for the q = 4 codes of BASELINE config 4: the Clay(12,4)
    single repair (256 x 960) and the shortened Clay(10,4) one -- the Clay(12,4) repair with
    the two virtual data nodes' columns dropped (they read zeros) and real node
    r >= 10 standing for Clay(12,4) node r + 2 -- derived in closed form by
    tests/golden/gen_clay42_maps.py's equations equal the planner's composed map."""
    import sys
    sys.path.insert(0, str(ROOT / "tests" / "golden"))
    import gen_clay42_maps as cf
    kk = k + v
    gf, g, rs = cf.field_and_code(kk, m)
    real_to_full = (lambda r: r if r < k else r + v)
    want_full = cf.repair_map(gf, g, rs, real_to_full(e))
    full_to_real = {real_to_full(r): r for r in range(k + m)}
    n_real = k + m
    want = {}
    for o, form in want_full.items():
        for slot, c in form.items():
            z, node = divmod(slot, g.n)
            if node in full_to_real:  # a virtual node's column multiplies zeros
                want[(o, z * n_real + full_to_real[node])] = c
    mat, ins, outs = ecx.ClayCodeErasureDecodingStep([e], k, m, virtualUnits=v).map().matrix()
    nz = np.nonzero(mat)
    got = {(int(outs[o]), int(ins[i])): int(mat[o, i]) for o, i in zip(*nz)}
    assert got == want


@pytest.mark.parametrize("k,m,v,erased", [(4, 2, 0, E) for E in ([0, 3], [1, 5], [0, 1], [2, 3], [4, 5], [0, 5])] +
                         [(6, 3, 0, [0, 4, 8]), (6, 3, 0, [1, 2, 3]), (8, 4, 0, [0, 5, 10, 11]),
                          (12, 4, 0, [0, 5, 10, 15]), (10, 4, 2, [0, 5, 11, 13]), (10, 4, 2, [10, 11, 12, 13])])
def test_clay_multi_erasure_maps_equal_parity_check_solution(ecx, k, m, v, erased):
    """Multi-node repair (doDecodeMulti's composition in the planner and the oracle)
    against the code's definition alone: gen_clay42_maps.solve_map solves every plane's RS
    parity checks on the pair-transformed symbols for the m erased nodes' sub-chunks by
    Gaussian elimination -- no decoding order, helper choice or stage sequence.  With
    |E| = m the linear map is unique, so the planner's composed map must equal it entry
    for entry, and so must the oracle's (read off by unit vectors, k + m <= 12).
    Shortened codes: the Clay(k + v, m) solution with the virtual nodes' columns dropped."""
    import sys
    sys.path.insert(0, str(ROOT / "tests" / "golden"))
    import gen_clay42_maps as cf
    gf, g, rs = cf.field_and_code(k + v, m)
    real_to_full = (lambda r: r if r < k else r + v)
    full_to_real = {real_to_full(r): r for r in range(k + m)}
    want = {}
    for o, form in cf.solve_map(gf, g, rs, [real_to_full(e) for e in erased]).items():
        for slot, c in form.items():
            z, node = divmod(slot, g.n)
            if node in full_to_real:  # a virtual node's column multiplies zeros
                want[(o, z * (k + m) + full_to_real[node])] = c
    kw = {"virtualUnits": v} if v else {}
    mat, ins, outs = ecx.ClayCodeErasureDecodingStep(erased, k, m, **kw).map().matrix()
    mats = [mat]
    if v == 0 and k + m <= 12:
        mats.append(_probe_oracle_map(k, m, erased, ins.tolist()))
    for mm in mats:
        nz = np.nonzero(mm)
        got = {(int(outs[o]), int(ins[i])): int(mm[o, i]) for o, i in zip(*nz)}
        assert got == want


def test_clay124_map_shape(ecx):
    inf = ecx.ClayCodeErasureDecodingStep([5], 12, 4).map().info()
    assert (inf["n_out"], inf["n_in"], inf["nnz"]) == (256, 960, 5568)


def test_helper_overload_maps(ecx):
    """ClayCodeHelper drives doDecodeSingle overload 2 per helper plane; the union of
    the per-plane maps reproduces the oracle's overload-2 outputs."""
    import ctypes
    k, m, B = 4, 2, 16
    n = 6
    rng = np.random.default_rng(5)
    for e in range(n):
        oc = O.Clay(k, m, [e])
        hidx = oc.helper_planes(e)
        helper = [rng.integers(0, 256, B, dtype=np.uint8) for _ in range(len(hidx) * n)]
        ref = [np.zeros(B, np.uint8) for _ in range(oc.alpha)]
        for i in range(len(hidx)):
            oc.decode_single_helper(helper, i, ref, e, B)
        step = ecx.ClayCodeErasureDecodingStep([e], k, m)
        assert step.getHelperPlanesIndexes(e) == hidx


@pytest.mark.parametrize("k,m,v,erased", [(10, 4, 2, [3]), (10, 4, 2, [13]), (10, 4, 2, [10, 11, 12, 13]),
                                          (3, 2, 1, [1]), (3, 2, 1, [3, 4])])
def test_shortened_clay_map_vs_oracle(ecx, k, m, v, erased):
    step = ecx.ClayCodeErasureDecodingStep(erased, k, m, virtualUnits=v)
    n = k + m
    a = step.subPacketSize
    B = 8
    rng = np.random.default_rng(3 + sum(erased))
    inputs = [None if (i % n) in erased else rng.integers(0, 256, B, dtype=np.uint8) for i in range(n * a)]
    ref = _shortened_oracle(k, m, v, erased, inputs, B)
    mat, ins, outs = step.map().matrix()
    assert ins.max() < n * a
    got = gf_apply_numpy(mat, [inputs[j] for j in ins])
    for o in range(len(outs)):
        assert (got[o] == ref[o]).all(), o


def test_clay104_shortened_shape(ecx):
    """BASELINE config 4: Clay(10,4) repair reads 13 real helper nodes x 64 planes."""
    inf = ecx.ClayCodeErasureDecodingStep([3], 10, 4, virtualUnits=2).map().info()
    assert inf["n_out"] == 256 and inf["n_in"] == 13 * 64


@pytest.mark.parametrize("k,m,v,erased", [(4, 2, 0, [1]), (4, 2, 0, [4, 5]), (4, 2, 0, [0, 3]), (6, 3, 0, [6, 7, 8]),
                                          (6, 3, 0, [1, 7]), (10, 4, 2, [3]), (10, 4, 2, [10, 11, 12, 13]),
                                          (12, 4, 0, [2, 9])])
def test_compiled_plan_selftest_clay(ecx, k, m, v, erased):
    """The compiled plan -- split tables, row tiles, tile groups and the LDS unions of
    k_gf_apply_lds -- interpreted on the host reproduces the composed map."""
    step = ecx.ClayCodeErasureDecodingStep(erased, k, m, virtualUnits=v)
    step.map().selftest(seed=len(erased) + k)


def test_compiled_plan_selftest_rs_lrc(ecx):
    import numpy as np
    rs = ecx.ReedSolomon.create(12, 4)
    rs.encode_map().selftest()
    rs.decode_map([False, True, True, False] + [True] * 11 + [False]).selftest()
    m = np.zeros((4, 12), np.uint8)
    for g in range(4):
        m[g, 3 * g:3 * g + 3] = 1
    ecx.GfMap.from_matrix(m, in_slot=[g * 4 + r for g in range(4) for r in range(3)],
                          out_slot=[g * 4 + 3 for g in range(4)]).selftest()
    rng = np.random.default_rng(0)
    big = rng.integers(0, 256, (40, 30), dtype=np.uint8)
    big[big < 100] = 0
    ecx.GfMap.from_matrix(big).selftest(7)  # 5 tiles with arbitrary sharing


def test_lrc_maps_match_reference_groups(ecx):
    """LRC maps (ecx_lrc_map): encode = XOR of each group's 3 data blocks into its parity
    (RS(3,1), LRCErasureCode.kt); decode rebuilds one block per group from the other 3
    and refuses two missing blocks in a group (RS(3,1).decodeMissing's exception)."""
    import numpy as np
    m, ins, outs = ecx.LRCErasureCode.map().matrix()
    assert list(outs) == [3, 7, 11, 15] and list(ins) == [g * 4 + r for g in range(4) for r in range(3)]
    assert (m == np.kron(np.eye(4, dtype=np.uint8), np.ones((1, 3), np.uint8))).all()
    pres = [True] * 16
    pres[2] = pres[7] = pres[12] = False
    dm = ecx.LRCErasureCode.map(pres)
    dm.selftest()
    m, ins, outs = dm.matrix()
    assert list(outs) == [2, 7, 12]
    rng = np.random.default_rng(4)
    blocks = [rng.integers(0, 256, 64, dtype=np.uint8) for _ in range(16)]
    for g in range(4):
        blocks[4 * g + 3] = blocks[4 * g] ^ blocks[4 * g + 1] ^ blocks[4 * g + 2]
    from conftest import gf_apply_numpy
    got = gf_apply_numpy(m, [blocks[s] for s in ins])
    for o, slot in enumerate(outs):
        assert (got[o] == blocks[slot]).all()
    pres[13] = False
    with pytest.raises(ecx.EcxError) as e:
        ecx.LRCErasureCode.map(pres)
    assert e.value.code == -2


def test_compiled_plan_selftest_random_maps(ecx):
    """Property test over random GF(256) maps: any shape (1..48 outputs, 1..48 inputs),
    any sparsity, coefficient-1 entries, all-zero rows and columns, and scattered
    (non-contiguous) slot numbers.  The compiled plan -- row tiles, entry tables, the
    padded arrays uploaded for ring depths 4 and 8 (with and without the LDS table
    copy), tile groups and their unions -- interpreted on the host reproduces the map."""
    import numpy as np
    hyp = pytest.importorskip("hypothesis")
    st = hyp.strategies

    @hyp.settings(max_examples=60, deadline=None, derandomize=True)
    @hyp.given(st.integers(1, 48), st.integers(1, 48), st.floats(0.0, 1.0), st.floats(0.0, 0.5),
               st.integers(0, 2**32 - 1))
    def check(n_out, n_in, density, ones, seed):
        rng = np.random.default_rng(seed)
        m = rng.integers(2, 256, (n_out, n_in)).astype(np.uint8)
        m[rng.random((n_out, n_in)) < ones] = 1
        m[rng.random((n_out, n_in)) >= density] = 0
        in_slot = sorted(rng.choice(4 * n_in, n_in, replace=False).tolist())
        out_slot = rng.permutation(rng.choice(4 * n_out, n_out, replace=False)).tolist()
        ecx.GfMap.from_matrix(m, in_slot=in_slot, out_slot=out_slot).selftest(seed & 0xFFFF)

    check()


@pytest.mark.parametrize("k,m,v,e", [(4, 2, 0, 1), (4, 2, 0, 5), (10, 4, 2, 3), (10, 4, 2, 13), (10, 4, 2, 9),
                                     (12, 4, 0, 0), (8, 4, 0, 11), (6, 3, 0, 7), (2, 2, 0, 0)])
def test_clay_repair_program_and_rtc_compile(ecx, k, m, v, e):
    """The single-node repair as a per-helper-plane program (ClayPlanner::repair_program:
    decouple with the dot identity pair_a ^ pair_b = 1, plane decode, re-couple) composes
    to exactly the reference stage sequence's map (checked inside the builder), and both
    generated kernels compile with hiprtc for gfx950 without a device: the plane-group
    kernel for q = 4 codes (the default, ecx_tune "rtc_group" 1), the one-plane-per-
    workgroup kernel for every code."""
    step = ecx.ClayCodeErasureDecodingStep([e], k, m, virtualUnits=v)
    try:
        for grp, persist, nt in ((1, 0, 0), (1, 2, 0), (0, 0, 0), (1, 0, 7), (1, 0, 1), (0, 0, 8), (0, 0, 5), (1, 0, 5)):
            if persist and not ecx.is_diag():
                continue  # the persistent grid: diagnostic library only (make DIAG=1)
            ecx.tune("rtc_group", grp)
            if ecx.is_diag():
                ecx.tune("rtc_persist", persist)
            ecx.tune("rtc_nt", nt)
            assert step.rtcCompileCheck() > 0
            src = step.rtcSource()
            name = "k_clay_repair_grp(" if grp and m == 4 else "k_clay_repair("
            assert name in src and "__launch_bounds__" in src
            if name == "k_clay_repair_grp(":
                assert ("for (u32 b = blockIdx.x; b < n_units" in src) == (persist > 0)
                # rtc_nt: the non-temporal loader is called only when some bit asks for it
                assert ("    ldv2(" in src) == (nt & 7 > 0)
                if nt & 1 == 0:
                    assert "    ldv0(" in src
            else:
                assert ("(int)so, 2);" in src) == (nt & 8 > 0)
    finally:
        ecx.tune("rtc_group", 1)
        if ecx.is_diag():
            ecx.tune("rtc_persist", 0)
        ecx.tune("rtc_nt", 5)


def test_clay_rtc_refuses_multi_erasure(ecx):
    step = ecx.ClayCodeErasureDecodingStep([0, 3], 4, 2)
    with pytest.raises(ecx.EcxError):
        step.rtcCompileCheck()


@pytest.mark.parametrize("case", ["clay42_03", "clay42_encode", "random16", "one_row", "accumulate"])
def test_map_planes_source_compiles(ecx, case):
    """The bit-plane kernel generated for one composed map (k_map_planes, map_rtc.cpp)
    compiles with hiprtc for gfx950 without a device, for the Clay(4,2) two-node repair
    and encode maps, a dense random 16-row map with coefficient-1 entries and zero rows,
    a one-row map, and in accumulate mode; every used input is loaded exactly once and
    every row stored exactly once."""
    rng = np.random.default_rng(5)
    acc = case == "accumulate"
    if case == "clay42_03":
        gm = ecx.ClayCodeErasureDecodingStep([0, 3], 4, 2).map()
    elif case == "clay42_encode":
        gm = ecx.ClayCodeErasureDecodingStep([4, 5], 4, 2).map()
    else:
        n_out = 1 if case == "one_row" else 16
        m = rng.integers(2, 256, (n_out, 40)).astype(np.uint8)
        m[rng.random(m.shape) < 0.2] = 1
        m[rng.random(m.shape) < 0.3] = 0
        if n_out > 1:
            m[3] = 0  # a row no input reaches
            m[:, 7] = 0  # an input no row reads
        gm = ecx.GfMap.from_matrix(m, in_slot=list(range(0, 80, 2)), out_slot=list(range(n_out)))
    mat, ins, outs = gm.matrix()
    src = gm.planes_source(acc)
    assert "k_map_planes(" in src
    used = [j for j in range(mat.shape[1]) if mat[:, j].any()]
    assert src.count("    ld(") == len(used)
    assert all(("    ld(%du * sl" % ins[j]) in src for j in used)
    stored = [r for r in range(mat.shape[0]) if mat[r].any() or not acc]
    assert src.count("    st(") == len(stored)
    assert gm.planes_compile_check(acc) > 0


def test_map_planes_refuses_wide_maps(ecx):
    """More than 16 rows do not fit the kernel's registers: refused, not truncated."""
    gm = ecx.ClayCodeErasureDecodingStep([3], 10, 4, virtualUnits=2).map()
    with pytest.raises(ecx.EcxError):
        gm.planes_source()


def test_lab_knobs_refused_by_the_product_library(ecx, monkeypatch):
    """The product library (libecx.so) does not contain the measured-and-rejected kernels
    and builds: ecx_tune refuses their keys, at any value, even with
    ECX_DIAGNOSTIC=1 (which only opens the diagnostic library's output-changing builds)."""
    if ecx.is_diag():
        pytest.skip("the diagnostic library accepts these keys")
    monkeypatch.setenv("ECX_DIAGNOSTIC", "1")
    for key in ("bitslice", "lds_lut", "wave_groups", "rtc_units", "rtc_persist", "rtc_diag", "occ_lds"):
        for val in (0, 1, 2):
            with pytest.raises(ecx.EcxError) as e:
                ecx.tune(key, val)
            assert e.value.code == -1, key
    with pytest.raises(ecx.EcxError):
        ecx.tune("rtc_lookahead", 17)  # the data-movement-only Clay build
    with pytest.raises(ecx.EcxError):
        ecx.tune("skew_trial", 1)  # replaced by layout_select


@pytest.mark.diag
def test_clay_grp_movement_only_build_is_isolated(ecx, monkeypatch):
    """rtc_lookahead bit 4 (16) generates the plane-group kernel's data-movement-only
    diagnostic build (coefficients as 1, no transposes), marked as such; the next
    default generation is byte-identical to one made before it.  Its outputs are not
    the repair, so ecx_tune refuses the bit unless the process set ECX_DIAGNOSTIC=1."""
    step = ecx.ClayCodeErasureDecodingStep([3], 10, 4, virtualUnits=2)
    monkeypatch.delenv("ECX_DIAGNOSTIC", raising=False)
    with pytest.raises(ecx.EcxError) as e:
        ecx.tune("rtc_lookahead", 17)
    assert e.value.code == -1
    monkeypatch.setenv("ECX_DIAGNOSTIC", "1")
    try:
        before = step.rtcSource()
        ecx.tune("rtc_lookahead", 17)
        diag = step.rtcSource()
        assert diag.startswith("// DIAGNOSTIC BUILD") and "    tr(" not in diag and "untr(" not in diag.split("DEV void untr")[1].split("\n", 1)[1]
        assert step.rtcCompileCheck() > 0
        ecx.tune("rtc_lookahead", 1)
        assert step.rtcSource() == before and "DIAGNOSTIC" not in before
    finally:
        ecx.tune("rtc_lookahead", 1)


def test_generated_kernels_without_hiprtc(tmp_path):
    """With no usable libhiprtc (ECX_HIPRTC_LIB names a missing file) the generated-kernel
    compile reports ECX_E_DEVICE with the reason, instead of crashing; run in a child
    process because the library is bound once per process."""
    import os
    import subprocess
    import sys
    code = (
        "import rpamd\n"
        "ecx = rpamd.load()\n"
        "step = ecx.ClayCodeErasureDecodingStep([3], 10, 4, virtualUnits=2)\n"
        "try:\n"
        "    step.rtcCompileCheck()\n"
        "except ecx.EcxError as e:\n"
        "    print('code', e.code, 'hiprtc' in str(e))\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ECX_HIPRTC_LIB=str(tmp_path / "no-libhiprtc.so"), PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "code -10 True" in r.stdout, r.stdout


def test_plane_group_kernel_wide_addresses_compile(ecx):
    """The plane-group kernel's 64-bit-address form (RtcShape::wide, ecx_tune "rtc_wide"), used
    where a stripe's slot offsets exceed 31 bits (Clay(10,4) with 1 MiB sub-chunks: 3.5 GiB per
    stripe): flat global loads with 64-bit offsets replace the buffer-resource loads, the rest
    of the generated source is the same, and it compiles with hiprtc for gfx950."""
    step = ecx.ClayCodeErasureDecodingStep([3], 10, 4, virtualUnits=2)
    narrow = step.rtcSource()
    ecx.tune("rtc_wide", 1)
    try:
        wide = step.rtcSource()
        assert "make_buffer_rsrc" in narrow and "make_buffer_rsrc" not in wide
        assert "const long long vz" in wide and "ibp + " in wide and "zero_page + voff" in wide
        assert wide.count("tr(") == narrow.count("tr(")  # same arithmetic
        assert step.rtcCompileCheck() > 0
    finally:
        ecx.tune("rtc_wide", 0)
    assert step.rtcSource() == narrow


@pytest.mark.parametrize("k,m,e", [(4, 2, 0), (4, 2, 1), (4, 2, 2), (4, 2, 3), (12, 4, 2), (12, 4, 5), (12, 4, 10),
                                   (2, 2, 1)])
def test_clay_is_test_branch_vs_oracle(ecx, k, m, e):
    """decodeDecoupledPlane's -DisTest=true branch (ClayCodeErasureDecodingStep
    .java:571-581; ecx_clay_create_ex ECX_CLAY_IS_TEST) -- decodeMissingSingle per helper, shard
    i + |E| taken as the i-th present one (bug B2).  The planner's map equals the oracle's
    restatement of that branch on random non-codeword inputs; for a repair whose erased row is
    nodes 0..q-1 it equals the default branch (B2 does not bite), for the other rows it differs,
    as the reference's does."""
    import oracle as O
    n = k + m
    step = ecx.ClayCodeErasureDecodingStep([e], k, m, isTest=True)
    a, q = step.subPacketSize, step.q
    B = 8 if a >= 64 else 24
    rng = np.random.default_rng(100 * k + e)
    inputs = [None if (i % n) == e else rng.integers(0, 256, B, dtype=np.uint8) for i in range(n * a)]
    ref = [np.zeros(B, np.uint8) for _ in range(a)]
    O.Clay(k, m, [e], is_test=True).perform_coding([x if x is None else x.copy() for x in inputs], ref, B)
    mat, ins, outs = step.map().matrix()
    got = gf_apply_numpy(mat, [inputs[j] for j in ins])
    assert all((got[o] == ref[o]).all() for o in range(a))
    std = _oracle_perform(k, m, [e], inputs, B)
    same = all((std[o] == ref[o]).all() for o in range(a))
    assert same == (e // q == 0), (e, same)  # row y = 0 holds nodes 0..q-1
    assert step.isTest and not ecx.ClayCodeErasureDecodingStep([e], k, m).isTest


@pytest.mark.parametrize("k,m,e", [(4, 2, 4), (4, 2, 5), (12, 4, 13)])
def test_clay_is_test_branch_parity_row_throws(ecx, k, m, e):
    """The isTest branch on a repair whose erased row holds a parity node: decodeMissingSingle has
    no matrix row for it and the reference throws NullPointerException (bug B3) -- the oracle's
    restatement returns ORC_E_NULL, libecx's map build ECX_E_NULL (-6); the default branch repairs."""
    import oracle as O
    n = k + m
    step = ecx.ClayCodeErasureDecodingStep([e], k, m, isTest=True)
    with pytest.raises(ecx.EcxError) as ei:
        step.map()
    assert ei.value.code == -6
    a = step.subPacketSize
    inputs = [None if (i % n) == e else np.zeros(8, np.uint8) for i in range(n * a)]
    with pytest.raises(Exception) as eo:
        O.Clay(k, m, [e], is_test=True).perform_coding(inputs, [np.zeros(8, np.uint8) for _ in range(a)], 8)
    assert "-6" in str(eo.value) or "Null" in str(eo.value)
    assert ecx.ClayCodeErasureDecodingStep([e], k, m).map() is not None
