"""Pin the oracle (CPU restatement of the reference JVM path) to the reference's
own known-answer tests and fixtures before trusting it as the parity checker.

Mirrors GaloisTest.java, MatrixTest.java and ReedSolomonTest.java; the Clay and
LRC layers (which the reference never tests) are pinned by the
survey's independent digests and by repair self-consistency.
"""
import hashlib
import itertools
from pathlib import Path

import numpy as np
import pytest

import oracle as O

GOLDEN = Path(__file__).resolve().parent / "golden"


def h16(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


# ---------------------------------------------------------------- GaloisTest.java
def test_tables_match_reference_literals(kats):
    g = kats["galois"]
    assert O.log_table().tolist() == g["log_table"]          # GaloisTest.java:116-117
    assert O.exp_table().tolist() == g["exp_table"]          # GaloisTest.java:119-120
    assert O.all_possible_polynomials() == g["polynomials"]  # GaloisTest.java:122-126


def test_galois_python_answers(kats):
    for a, b, r in kats["galois"]["multiply"]:
        assert O.gf_multiply(a, b) == r
    for a, n, r in kats["galois"]["exp"]:
        assert O.gf_exp(a, n) == r


def test_field_axioms_and_mul_table():
    mt = O.mul_table()
    # commutativity / identity / zero (GaloisTest.java:50-83), table == multiply (:129-137)
    assert (mt == mt.T).all()
    assert (mt[1] == np.arange(256)).all() and (mt[0] == 0).all()
    for a in range(1, 256):  # inverse: a * (1/a) == 1
        assert mt[a, O.gf_divide(1, a)] == 1
    # associativity (GaloisTest.java:28-47) and distributivity (:85-100) over all 256^3 triples
    a = np.arange(256).reshape(256, 1, 1)
    b = np.arange(256).reshape(1, 256, 1)
    c = np.arange(256).reshape(1, 1, 256)
    assert (mt[a, mt[b, c]] == mt[mt[a, b], c]).all()
    assert (mt[a, b ^ c] == (mt[a, b] ^ mt[a, c])).all()
    for x in (0, 1, 2, 3, 77, 255):                            # exp == repeated multiply (:102-112)
        p = 1
        for n in range(256):
            assert O.gf_exp(x, n) == p
            p = int(mt[p, x])
    with pytest.raises(O.OracleError):
        O.gf_divide(5, 0)


# ---------------------------------------------------------------- MatrixTest.java
def test_matrix_kats(kats):
    t = kats["matrix"]["times"]
    assert O.matrix_times(t["a"], t["b"]).tolist() == t["out"]
    for case in kats["matrix"]["invert"]:
        inv = O.matrix_invert(case["m"])
        assert inv.tolist() == case["inv"]
        ident = O.matrix_times(case["m"], inv)
        assert (ident == np.eye(len(inv), dtype=np.uint8)).all()
    with pytest.raises(O.OracleError):
        O.matrix_invert([[1, 1], [1, 1]])


# ---------------------------------------------------------------- ReedSolomonTest.java
def test_rs_one_encode_kat(kats):
    r = kats["reed_solomon"]
    rs = O.ReedSolomon(5, 5)
    shards = [np.array(x, np.uint8) for x in r["rs55_data"]] + [np.zeros(2, np.uint8) for _ in range(5)]
    rs.encode_parity(shards, 0, 2)
    assert [s.tolist() for s in shards[5:]] == r["rs55_parity"]
    assert rs.is_parity_correct(shards, 0, 2)
    shards[8][0] += 1
    assert not rs.is_parity_correct(shards, 0, 2)
    assert not rs.is_parity_correct(shards, 0, 2, np.zeros(2, np.uint8))


def test_rs_parity_rows(kats):
    for key, rows in kats["rs_parity_rows"].items():
        if key == "17,3_row0":
            assert O.ReedSolomon(17, 3).parity_rows[0].tolist() == rows
        else:
            k, m = map(int, key.split(","))
            assert O.ReedSolomon(k, m).parity_rows.tolist() == rows


def test_zero_size_encode():
    rs = O.ReedSolomon(2, 1)  # ReedSolomonTest.java:32-37
    rs.encode_parity([np.zeros(0, np.uint8) for _ in range(3)], 0, 0)


def test_java_random(kats):
    assert O.JavaRandom(0).next_int() == kats["reed_solomon"]["java_random_0_first_int"]


def _encode_decode_all_subsets(k, m, data):
    rs = O.ReedSolomon(k, m)
    n = k + m
    L = len(data[0])
    allsh = [np.array(d, np.uint8) for d in data] + [np.zeros(L, np.uint8) for _ in range(m)]
    rs.encode_parity(allsh, 0, L)
    test = [s.copy() for s in allsh]
    for nmiss in range(m + 1):  # ReedSolomonTest.java:140-169, allSubsets(n, 0, 10)
        for subset in itertools.combinations(range(min(10, n)), nmiss):
            present = [True] * n
            for s in subset:
                test[s][:] = 0
                present[s] = False
            rs.decode_missing(test, present, 0, L)
            for a, b in zip(allsh, test):
                assert (a == b).all()


def test_simple_encode_decode(kats):
    _encode_decode_all_subsets(5, 5, kats["reed_solomon"]["simple_data"])


def test_big_encode_decode():
    r = O.JavaRandom(0)  # ReedSolomonTest.java:90-103
    data = [[r.next_int(256) for _ in range(200)] for _ in range(64)]
    rs = O.ReedSolomon(64, 64)
    allsh = [np.array(d, np.uint8) for d in data] + [np.zeros(200, np.uint8) for _ in range(64)]
    rs.encode_parity(allsh, 0, 200)
    # runEncodeDecode / tryAllSubsetsMissing (:111-169): numberMissing 0..64, every subset of
    # that size among shards [0, 10) -- sizes 0..10, 1,024 subsets -- on one set of test
    # shards that each decode must restore for the next subset
    test = [s.copy() for s in allsh]
    n_subsets = 0
    for nmiss in range(64 + 1):
        for subset in itertools.combinations(range(10), nmiss):
            present = [True] * 128
            for s in subset:
                test[s][:] = 0
                present[s] = False
            rs.decode_missing(test, present, 0, 200)
            assert all((a == b).all() for a, b in zip(allsh, test)), subset
            n_subsets += 1
    assert n_subsets == 1024


def test_not_enough_shards():
    rs = O.ReedSolomon(4, 2)
    sh = [np.zeros(8, np.uint8) for _ in range(6)]
    with pytest.raises(O.OracleError) as e:
        rs.decode_missing(sh, [True, False, False, False, True, True], 0, 8)
    assert e.value.code == -2
    with pytest.raises(O.OracleError):
        O.ReedSolomon(200, 57)


def test_decode_missing_single_matches_decode_missing():
    """decodeMissingSingle summed along a chain == decodeMissing (the pipelined RS path)."""
    rs = O.ReedSolomon(4, 2)
    rng = np.random.default_rng(3)
    data = [rng.integers(0, 256, 100, dtype=np.uint8) for _ in range(4)]
    sh = data + [np.zeros(100, np.uint8) for _ in range(2)]
    rs.encode_parity(sh, 0, 100)
    present = [True, False, True, True, True, False]
    outs = [np.zeros(100, np.uint8)]
    chain = [i for i in range(6) if present[i]][:4]
    for c, idx in enumerate(chain):
        rs.decode_missing_single(sh[idx], idx, c, present, outs, 0, 100, c == 0)
    assert (outs[0] == data[1]).all()
    with pytest.raises(O.OracleError) as e:  # bug B3: no missing data shard -> NPE
        rs.decode_missing_single(sh[0], 0, 0, [True] * 4 + [False, True], outs, 0, 100, True)
    assert e.value.code == -6


# ---------------------------------------------------------------- files / LRC / Clay digests
def test_sample_encoder_lp_block(kats):
    lp = np.fromfile(GOLDEN / "LP-block.jpg", dtype=np.uint8)
    shards = O.sample_encode(lp)
    assert len(shards[0]) == 104449
    assert [h16(s) for s in shards] == kats["survey_digests"]["sample_encoder_lp_block"]
    for missing in range(6):
        partial = [None if i == missing else s for i, s in enumerate(shards)]
        out, _ = O.sample_decode(partial)
        assert (out == lp).all()


def test_lrc_lp_block(kats):
    lp = np.fromfile(GOLDEN / "LP-block.jpg", dtype=np.uint8)
    blocks = O.lrc_encode(lp)
    assert [h16(blocks[i]) for i in (3, 7, 11, 15)] == kats["survey_digests"]["lrc_local_parities_3_7_11_15"]
    single = O.lrc_encode_using_single(lp)
    assert all((a == b).all() for a, b in zip(blocks, single))
    out, shards = O.lrc_decode(blocks, [2], len(blocks[0]))
    assert (out == lp[:len(out)]).all() and (shards[2] == blocks[2]).all()


def test_clay42_getinputs_and_encode(kats):
    d = kats["survey_digests"]
    inp = O.clay_get_inputs(4, 2, 32768)
    assert bytes(inp[0][:8]).hex() == d["clay42_first_bytes"]
    outs = O.clay_encode(4, 2, inp, 32768)
    assert [h16(outs[z * 2]) for z in range(8)] == d["clay42_parity_node4"]
    assert [h16(outs[z * 2 + 1]) for z in range(8)] == d["clay42_parity_node5"]


def clay_stripe(k, m, B):
    inp = O.clay_get_inputs(k, m, B)
    outs = O.clay_encode(k, m, inp, B)
    n = k + m
    a = len(inp) // n
    return [inp[z * n + i] if i < k else outs[z * m + i - k] for z in range(a) for i in range(n)]


@pytest.mark.parametrize("k,m,B", [(2, 2, 32), (4, 2, 40), (6, 3, 16), (12, 4, 8)])
def test_clay_repair_self_consistent(k, m, B):
    full = clay_stripe(k, m, B)
    n = k + m
    a = len(full) // n
    for e in range(n):
        c = O.Clay(k, m, [e])
        ins = [None if (i % n) == e else full[i] for i in range(n * a)]
        outs = [np.zeros(B, np.uint8) for _ in range(a)]
        c.perform_coding(ins, outs, B)
        assert all((outs[z] == full[z * n + e]).all() for z in range(a))


def test_clay_helper_overload_matches_overload1():
    """ClayCodeHelper.getHelperPlanesAndDecode drives doDecodeSingle overload 2 per helper plane."""
    k, m, B = 4, 2, 24
    full = clay_stripe(k, m, B)
    n = 6
    for e in range(n):
        c = O.Clay(k, m, [e])
        hidx = c.helper_planes(e)
        helper = [full[z * n + j] for z in hidx for j in range(n)]
        outs = [np.zeros(B, np.uint8) for _ in range(c.alpha)]
        for i in range(len(hidx)):
            c.decode_single_helper(helper, i, outs, e, B)
        assert all((outs[z] == full[z * n + e]).all() for z in range(c.alpha))


def test_clay_unsupported_geometry():
    # Clay(10,4): t = 14 // 4 = 3, nodes 12,13 have y = 3 >= t (bug B7) -> index error
    c = O.Clay(10, 4, [13])
    with pytest.raises(O.OracleError):
        c.helper_planes(13)


def test_cpu_baseline_harness_runs_threads():
    """orc_bench.c (bench.py's cpu_baseline) runs the oracle repair on several threads."""
    import numpy as np
    import oracle as O
    rng = np.random.default_rng(3)
    k, m, e, b = 4, 2, 1, 512
    stripes = []
    for _ in range(4):
        data = [rng.integers(0, 256, b, dtype=np.uint8) if i % 6 < k else None for i in range(48)]
        par = O.clay_encode(k, m, data, b)
        full = [data[i] if i % 6 < k else par[(i // 6) * m + i % 6 - k] for i in range(48)]
        stripes.append([None if i % 6 == e else full[i] for i in range(48)])
    reps, el = O.bench_clay_repair(k, m, e, b, stripes, 2, 0.05)
    assert reps >= 2 and el >= 0.05
