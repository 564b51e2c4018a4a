"""GPU parity: every entry point of the C ABI, executed by the HIP kernels on
the MI355X, is bit-exact against the oracle (the CPU restatement of the
reference JVM path) on the same seeded inputs; at BASELINE sizes through
size-independent properties (encode -> erase -> repair round trips)."""
import hashlib
from pathlib import Path

import numpy as np
import pytest

import oracle as O
from conftest import diag_build, gf_apply_numpy, shortened_clay_oracle

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"


def h16(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


# ---------------------------------------------------------------- CodingLoop
@pytest.mark.parametrize("nin,nout,L,offset", [(1, 1, 1, 0), (3, 2, 15, 0), (5, 5, 17, 3), (17, 3, 4095, 0),
                                               (17, 3, 4097, 5), (4, 8, 10000, 100), (20, 8, 65536, 0),
                                               (2, 9, 333, 7)])
def test_code_some_shards(ecx, nin, nout, L, offset):
    rng = np.random.default_rng(nin * 100 + nout)
    rows = rng.integers(0, 256, (nout, nin), dtype=np.uint8)
    rows[0, 0] = 1
    if nin > 1:
        rows[-1, 1] = 0
    ins = [rng.integers(0, 256, L + offset, dtype=np.uint8) for _ in range(nin)]
    outs = [rng.integers(0, 256, L + offset, dtype=np.uint8) for _ in range(nout)]
    ref = [o.copy() for o in outs]
    O.code_some_shards(list(rows), ins, ref, offset, L)
    ecx.CodingLoop().codeSomeShards(rows, ins, nin, outs, nout, offset, L)
    for a, b in zip(outs, ref):
        assert (a == b).all()


def test_check_some_shards(ecx):
    rng = np.random.default_rng(2)
    rows = rng.integers(0, 256, (3, 6), dtype=np.uint8)
    ins = [rng.integers(0, 256, 777, dtype=np.uint8) for _ in range(6)]
    outs = [np.zeros(777, np.uint8) for _ in range(3)]
    O.code_some_shards(list(rows), ins, outs, 0, 777)
    loop = ecx.CodingLoop()
    assert loop.checkSomeShards(rows, ins, 6, outs, 3, 0, 777)
    outs[2][776] ^= 1
    assert not loop.checkSomeShards(rows, ins, 6, outs, 3, 0, 777)
    assert loop.checkSomeShards(rows, ins, 6, outs, 3, 0, 776)


@pytest.mark.parametrize("first", [True, False])
def test_code_single(ecx, first):
    rng = np.random.default_rng(3)
    rows = rng.integers(0, 256, (4, 4), dtype=np.uint8)
    x = rng.integers(0, 256, 1000, dtype=np.uint8)
    out = rng.integers(0, 256, 1000, dtype=np.uint8)
    exp = out.copy()
    mt = O.mul_table()
    prod = mt[rows[2][3]][x[10:990]]
    exp[10:990] = prod if first else exp[10:990] ^ prod
    ecx.InputOutputByteTableCodingLoopSingle().codeSomeShards(rows, x, 3, out, 2, 10, 980, first)
    assert (out == exp).all()


# ---------------------------------------------------------------- ReedSolomon
def test_rs_one_encode_kat(ecx, kats):
    r = kats["reed_solomon"]
    rs = ecx.ReedSolomon.create(5, 5)
    shards = [np.array(x, np.uint8) for x in r["rs55_data"]] + [np.zeros(2, np.uint8) for _ in range(5)]
    rs.encodeParity(shards, 0, 2)
    assert [s.tolist() for s in shards[5:]] == r["rs55_parity"]
    assert rs.isParityCorrect(shards, 0, 2)
    shards[8][0] += 1
    assert not rs.isParityCorrect(shards, 0, 2)
    assert not rs.isParityCorrect(shards, 0, 2, np.zeros(2, np.uint8))


def test_rs_zero_size_encode(ecx):
    ecx.ReedSolomon.create(2, 1).encodeParity([np.zeros(0, np.uint8) for _ in range(3)], 0, 0)


@pytest.mark.parametrize("k,m,L", [(4, 2, 104449), (5, 5, 2000), (17, 3, 200000), (12, 4, 4096 + 13)])
def test_rs_encode_vs_oracle(ecx, k, m, L):
    rng = np.random.default_rng(k + m)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    a = [d.copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(m)]
    b = [d.copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(m)]
    ecx.ReedSolomon.create(k, m).encodeParity(a, 0, L)
    O.ReedSolomon(k, m).encode_parity(b, 0, L)
    assert all((x == y).all() for x, y in zip(a, b))


def test_rs_decode_all_subsets(ecx):
    """ReedSolomonTest.runEncodeDecode (:111-169) for RS(5,5) over every erasure subset."""
    import itertools
    k, m, L = 5, 5, 300
    rng = np.random.default_rng(9)
    allsh = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)] + [np.zeros(L, np.uint8) for _ in range(m)]
    rs = ecx.ReedSolomon.create(k, m)
    rs.encodeParity(allsh, 0, L)
    for nmiss in range(m + 1):
        for subset in itertools.combinations(range(10), nmiss):
            test = [s.copy() for s in allsh]
            present = [True] * 10
            for s in subset:
                test[s][:] = 0
                present[s] = False
            rs.decodeMissing(test, present, 0, L)
            assert all((x == y).all() for x, y in zip(allsh, test)), subset


def test_rs_big_encode_decode(ecx):
    """ReedSolomonTest.testBigEncodeDecode (:90-103) on the device: RS(64,64) with
    200-B shards of java.util.Random(0).nextInt(256) -- a multi-tile map (8 row tiles
    of 64 entries each).  The encode equals the oracle's; decoding every erasure subset
    the reference's runEncodeDecode / tryAllSubsetsMissing (:111-169) tries -- every
    subset of shards [0, 10), sizes 0..10, 1,024 subsets, on one set of test shards that
    each decode restores for the next -- restores the stripe, and so do random 64-shard
    erasures; on non-codeword shards decodeMissing equals the oracle's map."""
    import itertools
    r = O.JavaRandom(0)
    data = [np.array([r.next_int(256) for _ in range(200)], np.uint8) for _ in range(64)]
    allsh = [d.copy() for d in data] + [np.zeros(200, np.uint8) for _ in range(64)]
    ref = [d.copy() for d in data] + [np.zeros(200, np.uint8) for _ in range(64)]
    rs = ecx.ReedSolomon.create(64, 64)
    rs.encodeParity(allsh, 0, 200)
    O.ReedSolomon(64, 64).encode_parity(ref, 0, 200)
    assert all((a == b).all() for a, b in zip(allsh, ref))
    rng = np.random.default_rng(64)
    subsets = [s for n in range(64 + 1) for s in itertools.combinations(range(10), n)]
    assert len(subsets) == 1024
    subsets += [tuple(int(i) for i in rng.choice(128, 64, replace=False)) for _ in range(4)]
    test = [s.copy() for s in allsh]
    for subset in subsets:
        present = [True] * 128
        for s in subset:
            test[s][:] = 0
            present[s] = False
        rs.decodeMissing(test, present, 0, 200)
        assert all((a == b).all() for a, b in zip(allsh, test)), subset
    for subset in subsets[-2:]:
        junk = [rng.integers(0, 256, 200, dtype=np.uint8) for _ in range(128)]
        a, b = [x.copy() for x in junk], [x.copy() for x in junk]
        present = [i not in subset for i in range(128)]
        rs.decodeMissing(a, present, 0, 200)
        O.ReedSolomon(64, 64).decode_missing(b, present, 0, 200)
        assert all((x == y).all() for x, y in zip(a, b))


def test_rs_decode_noncodeword_vs_oracle(ecx):
    rng = np.random.default_rng(12)
    for present in ([1, 0, 1, 1, 0, 1], [0, 1, 1, 1, 1, 1], [1, 1, 1, 1, 0, 0], [0, 0, 1, 1, 1, 1]):
        shards = [rng.integers(0, 256, 5000, dtype=np.uint8) for _ in range(6)]
        a = [s.copy() for s in shards]
        b = [s.copy() for s in shards]
        pres = [bool(p) for p in present]
        ecx.ReedSolomon.create(4, 2).decodeMissing(a, pres, 7, 4000)
        O.ReedSolomon(4, 2).decode_missing(b, pres, 7, 4000)
        assert all((x == y).all() for x, y in zip(a, b))


def test_rs_not_enough_shards(ecx):
    rs = ecx.ReedSolomon.create(4, 2)
    with pytest.raises(ecx.EcxError) as e:
        rs.decodeMissing([np.zeros(8, np.uint8) for _ in range(6)], [1, 0, 0, 0, 1, 1], 0, 8)
    assert e.value.code == -2
    with pytest.raises(ecx.EcxError) as e:
        rs.encodeParity([np.zeros(8, np.uint8) for _ in range(5)], 0, 8)
    assert e.value.code == -1
    with pytest.raises(ecx.EcxError):
        rs.encodeParity([np.zeros(8, np.uint8) for _ in range(6)], 4, 8)


def test_rs_single_apis(ecx):
    """encodeParitySingle chains (LRC) and decodeMissingSingle chains (pipelined RS)."""
    rng = np.random.default_rng(4)
    k, m, L = 4, 2, 3000
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    rs, ors = ecx.ReedSolomon.create(k, m), O.ReedSolomon(k, m)
    for p in range(m):
        a = rng.integers(0, 256, L, dtype=np.uint8)
        b = a.copy()
        for i in range(k):
            rs.encodeParitySingle(data[i], a, i, p, 0, L)
            ors.encode_parity_single(data[i], b, i, p, 0, L)
        assert (a == b).all()
    shards = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k + m)]
    present = [True, False, True, False, True, True]
    a = [np.zeros(L, np.uint8) for _ in range(2)]
    b = [np.zeros(L, np.uint8) for _ in range(2)]
    chain = [0, 2, 4, 5]
    for c, idx in enumerate(chain):
        rs.decodeMissingSingle(shards[idx], idx, c, present, a, 0, L, c == 0)
        ors.decode_missing_single(shards[idx], idx, c, present, b, 0, L, c == 0)
    assert all((x == y).all() for x, y in zip(a, b))
    with pytest.raises(ecx.EcxError) as e:  # bug B3: parity-only erasure -> NPE
        rs.decodeMissingSingle(shards[0], 0, 0, [True] * 5 + [False], [np.zeros(L, np.uint8)], 0, L, True)
    assert e.value.code == -6


# ---------------------------------------------------------------- files / LRC
def test_sample_encoder_lp_block(ecx, kats):
    lp = np.fromfile(GOLDEN / "LP-block.jpg", dtype=np.uint8)
    shards = ecx.sample_encode(lp)
    assert [h16(s) for s in shards] == kats["survey_digests"]["sample_encoder_lp_block"]
    for missing in range(6):
        out, _ = ecx.sample_decode([None if i == missing else s for i, s in enumerate(shards)])
        assert (out == lp).all()


def test_lrc_lp_block(ecx, kats):
    lp = np.fromfile(GOLDEN / "LP-block.jpg", dtype=np.uint8)
    blocks = ecx.lrc_encode(lp)
    assert [h16(blocks[i]) for i in (3, 7, 11, 15)] == kats["survey_digests"]["lrc_local_parities_3_7_11_15"]
    single = ecx.lrc_encode_using_single(lp)
    assert all((a == b).all() for a, b in zip(blocks, single))
    for missing in (2, 7, 12):
        out, shards = ecx.lrc_decode(blocks, [missing], len(blocks[0]))
        assert (shards[missing] == blocks[missing]).all()


# ---------------------------------------------------------------- Clay (per call)
CLAY_CASES = [(2, 2, [0]), (4, 2, [0]), (4, 2, [1]), (4, 2, [2]), (4, 2, [3]), (4, 2, [4]), (4, 2, [5]),
              (4, 2, [4, 5]), (4, 2, [0, 1]), (4, 2, [1, 4]), (6, 3, [2]), (6, 3, [6, 7, 8]), (12, 4, [5]),
              (12, 4, [12, 13, 14, 15])]


@pytest.mark.parametrize("k,m,erased", CLAY_CASES)
def test_clay_perform_coding_vs_oracle(ecx, k, m, erased):
    n = k + m
    step = ecx.ClayCodeErasureDecodingStep(erased, k, m)
    a = step.subPacketSize
    B = 64 if a >= 64 else 2174  # 2174 = ClayCodeHelper.kt:90's CLAY_BLOCK_SIZE (ragged, not 16-aligned)
    rng = np.random.default_rng(len(erased) * 13 + k)
    inputs = [None if (i % n) in erased else rng.integers(0, 256, B, dtype=np.uint8) for i in range(n * a)]
    oc = O.Clay(k, m, erased)
    ref = [np.zeros(B, np.uint8) for _ in range(len(erased) * a)]
    oc.perform_coding(inputs, ref, B)
    got = [np.zeros(B, np.uint8) for _ in range(len(erased) * a)]
    step.performCoding(inputs, got, B)
    for o in range(len(got)):
        assert (got[o] == ref[o]).all(), o


@pytest.mark.parametrize("k,m,e", [(4, 2, 1), (4, 2, 2), (4, 2, 4), (12, 4, 5)])
def test_clay_is_test_branch_on_device(ecx, torch_dev, k, m, e):
    """The reference run with -DisTest=true (decodeDecoupledPlane :571-581, ecx_clay_create_ex):
    per call and as a device batch, the repair equals the oracle's restatement of that branch on
    random non-codeword inputs -- the default map for row 0 (e = 1), the branch's own map (bug B2)
    for another row (e = 2; Clay(12,4) e = 5, where the composed-map kernel runs: the generated
    plane-group kernel implements the default branch only) -- and a row holding a parity node
    (e = 4) fails with NullPointerException's status (-6, bug B3) on both paths."""
    torch = torch_dev
    n = k + m
    step = ecx.ClayCodeErasureDecodingStep([e], k, m, isTest=True)
    a = step.subPacketSize
    B = 4096
    rng = np.random.default_rng(500 + e)
    inputs = [None if (i % n) == e else rng.integers(0, 256, B, dtype=np.uint8) for i in range(n * a)]
    got = [np.zeros(B, np.uint8) for _ in range(a)]
    pool = torch.from_numpy(np.stack([x if x is not None else np.zeros(B, np.uint8) for x in inputs])).cuda()
    out = torch.zeros((a, B), dtype=torch.uint8, device="cuda")
    if e == 4:
        with pytest.raises(ecx.EcxError) as ei:
            step.performCoding(inputs, got, B)
        assert ei.value.code == -6
        with pytest.raises(ecx.EcxError) as ei:
            step.performCodingBatch(pool, n * a * B, B, out, a * B, B, 1, B)
        assert ei.value.code == -6
        return
    ref = [np.zeros(B, np.uint8) for _ in range(a)]
    O.Clay(k, m, [e], is_test=True).perform_coding([x if x is None else x.copy() for x in inputs], ref, B)
    step.performCoding(inputs, got, B)
    assert all((got[z] == ref[z]).all() for z in range(a))
    step.performCodingBatch(pool, n * a * B, B, out, a * B, B, 1, B)
    torch.cuda.synchronize()
    dev = out.cpu().numpy()
    assert all((dev[z] == ref[z]).all() for z in range(a))


def test_clay_multi_nonnull_erased_inputs(ecx):
    """doDecodeMulti with non-null buffers at erased slots (the reference reads them)."""
    k, m, erased, B = 4, 2, [0, 1], 100
    n, a = 6, 8
    rng = np.random.default_rng(21)
    inputs = [rng.integers(0, 256, B, dtype=np.uint8) for _ in range(n * a)]
    ref = [np.zeros(B, np.uint8) for _ in range(2 * a)]
    O.Clay(k, m, erased).perform_coding([x.copy() for x in inputs], ref, B)
    got = [np.zeros(B, np.uint8) for _ in range(2 * a)]
    ecx.ClayCodeErasureDecodingStep(erased, k, m).performCoding(inputs, got, B)
    assert all((x == y).all() for x, y in zip(got, ref))


def test_clay_getinputs_encode_digests(ecx, kats):
    """ClayCodeRunner.main's encode half (ClayCodeRunner.java:20-28) through the facade."""
    d = kats["survey_digests"]
    cc = ecx.ClayCode(4, 2, 32768, [4, 5])
    inp = cc.getInputs()
    assert bytes(inp[0].getChunk().getBuffer()[:8]).hex() == d["clay42_first_bytes"]
    ic, oc = cc.encode(inp, cc.getOutputs())
    outs = ecx.ECChunk.toBuffers(oc)
    assert [h16(outs[z * 2]) for z in range(8)] == d["clay42_parity_node4"]
    assert [h16(outs[z * 2 + 1]) for z in range(8)] == d["clay42_parity_node5"]


def test_clay_runner_flow_and_b1_quirk(ecx, tmp_path):
    """ClayCodeRunner.main (ClayCodeRunner.java:6-39) end to end: encode, getTestInputs,
    performCoding.  The reference's getTestInputs index quirk leaves
    the erased node's data in place for e in {1,2,3} (repair correct) and zeroes the
    wrong sub-chunks for e in {0,4,5} -- reproduced exactly, and checked vs the oracle."""
    k, m, B = 4, 2, 2174
    enc = ecx.ClayCode(k, m, B, [4, 5])
    ic, oc = enc.encode(enc.getInputs(), enc.getOutputs())
    ib, ob = ecx.ECChunk.toBuffers(ic), ecx.ECChunk.toBuffers(oc)
    full = [ib[i] if ib[i] is not None else ob[(i // 6) * 2 + (i % 6) - 4] for i in range(48)]
    for e in range(6):
        cc = ecx.ClayCode(k, m, B, [e])
        test = cc.getTestInputs(ic, oc, [e], write_dir=tmp_path if e == 1 else None)
        outs = cc.getTestOutputs(1)
        cc.performCoding(cc.getChunks(test), cc.getChunks(outs))
        got = [o.getChunk().getBuffer() for o in outs]
        ref = [np.zeros(B, np.uint8) for _ in range(8)]
        O.Clay(k, m, [e]).perform_coding([t.getChunk().getBuffer() for t in test], ref, B)
        assert all((g == r).all() for g, r in zip(got, ref))
        correct = all((got[z] == full[z * 6 + e]).all() for z in range(8))
        assert correct == (e in (1, 2, 3)), e
    assert (ecx.read_subchunk(tmp_path, "LP", 2, 5, B) == full[5 * 6 + 2]).all()
    assert (ecx.read_subchunk(tmp_path, "LP", 1, 3, B, original=True) == full[3 * 6 + 1]).all()


def test_clay_code_helper(ecx):
    """ClayCodeHelper.getHelperPlanesAndDecode (ClayCodeHelper.kt:19-56), main()'s shape
    (B = 2174, e = 1, ClayCodeHelper.kt:78-104)."""
    k, m, B, e = 4, 2, 2174, 1
    enc = ecx.ClayCode(k, m, B, [4, 5])
    ic, oc = enc.encode(enc.getInputs(), enc.getOutputs())
    ib, ob = ecx.ECChunk.toBuffers(ic), ecx.ECChunk.toBuffers(oc)
    full = [ib[i] if ib[i] is not None else ob[(i // 6) * 2 + (i % 6) - 4] for i in range(48)]
    blocks = [ecx.ECBlock(ecx.ECChunk(None if (i % 6) == e else full[i].copy())) for i in range(48)]
    outs = [[np.zeros(B, np.uint8)] for _ in range(8)]
    helper = ecx.ClayCodeHelper(k, m, 8, blocks)
    helper.getHelperPlanesAndDecode(ecx.ClayCodeUtil([e], k, m), "LP", outs, e, B)
    assert all((outs[z][0] == full[z * 6 + e]).all() for z in range(8))


def test_clay_helper_overload(ecx):
    """ClayCodeHelper.getHelperPlanesAndDecode: overload 2, one helper plane at a time."""
    k, m, B, n = 4, 2, 2174, 6
    rng = np.random.default_rng(8)
    for e in range(n):
        oc = O.Clay(k, m, [e])
        hidx = oc.helper_planes(e)
        helper = [rng.integers(0, 256, B, dtype=np.uint8) for _ in range(len(hidx) * n)]
        ref = [np.zeros(B, np.uint8) for _ in range(oc.alpha)]
        got = [np.zeros(B, np.uint8) for _ in range(oc.alpha)]
        step = ecx.ClayCodeErasureDecodingStep([e], k, m)
        rows = [helper[i * n:(i + 1) * n] for i in range(len(hidx))]
        for i in range(len(hidx)):
            oc.decode_single_helper(helper, i, ref, e, B)
            step.doDecodeSingleHelper(rows, i, got, e, B)
        assert all((x == y).all() for x, y in zip(got, ref))


# ---------------------------------------------------------------- batched, device-resident
def _clay_pool(ecx, torch, k, m, B, S, seed=1):
    """S valid Clay stripes [S][n*alpha][B] built on the device: random data + GPU encode."""
    n = k + m
    enc = ecx.ClayCodeErasureDecodingStep(list(range(k, n)), k, m)
    a = enc.subPacketSize
    pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), seed)
    par = torch.empty((S, m * a, B), dtype=torch.uint8, device="cuda")
    enc.performCodingBatch(pool, n * a * B, B, par, m * a * B, B, S, B)
    pv = pool.view(S, a, n, B)
    pv[:, :, k:, :] = par.view(S, a, m, B)
    torch.cuda.synchronize()
    return pool, a


def test_clay_batch_encode_vs_oracle(ecx, torch_dev):
    torch = torch_dev
    k, m, B, S = 4, 2, 4096 + 48, 3
    pool, a = _clay_pool(ecx, torch, k, m, B, S)
    host = pool.cpu().numpy()
    for s in range(S):
        inputs = [host[s, i].copy() if (i % 6) < k else None for i in range(6 * a)]
        ref = [np.zeros(B, np.uint8) for _ in range(2 * a)]
        O.Clay(k, m, [4, 5]).perform_coding(inputs, ref, B)
        for z in range(a):
            for j in range(2):
                assert (host[s, z * 6 + 4 + j] == ref[z * 2 + j]).all()


@pytest.mark.parametrize("e", range(6))
def test_clay42_batch_repair_headline_roundtrip(ecx, torch_dev, e):
    """BASELINE config 2 shape (B = 32 KiB): repair every stripe's node e and compare
    with the original sub-chunks on the device; sampled stripes also vs the oracle."""
    torch = torch_dev
    k, m, B, S = 4, 2, 32768, 64
    pool, a = _clay_pool(ecx, torch, k, m, B, S, seed=100 + e)
    out = torch.empty((S, a, B), dtype=torch.uint8, device="cuda")
    step = ecx.ClayCodeErasureDecodingStep([e], k, m)
    step.performCodingBatch(pool, 6 * a * B, B, out, a * B, B, S, B)
    torch.cuda.synchronize()
    orig = pool.view(S, a, 6, B)[:, :, e, :]
    assert torch.equal(out, orig)
    host = pool[0].cpu().numpy()
    inputs = [None if (i % 6) == e else host[i].copy() for i in range(6 * a)]
    ref = [np.zeros(B, np.uint8) for _ in range(a)]
    O.Clay(k, m, [e]).perform_coding(inputs, ref, B)
    got = out[0].cpu().numpy()
    assert all((got[z] == ref[z]).all() for z in range(a))


def test_clay_batch_noncodeword_vs_oracle(ecx, torch_dev):
    """Random (non-codeword) stripes: the batch kernel reproduces the reference's linear map."""
    torch = torch_dev
    k, m, B, S, e = 4, 2, 8192 + 16, 4, 1
    pool = torch.empty((S, 48, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 77)
    out = torch.empty((S, 8, B), dtype=torch.uint8, device="cuda")
    ecx.ClayCodeErasureDecodingStep([e], k, m).performCodingBatch(pool, 48 * B, B, out, 8 * B, B, S, B)
    torch.cuda.synchronize()
    host, got = pool.cpu().numpy(), out.cpu().numpy()
    for s in range(S):
        inputs = [None if (i % 6) == e else host[s, i].copy() for i in range(48)]
        ref = [np.zeros(B, np.uint8) for _ in range(8)]
        O.Clay(k, m, [e]).perform_coding(inputs, ref, B)
        assert all((got[s, z] == ref[z]).all() for z in range(8))


@pytest.mark.parametrize("k,m", [(2, 2), (4, 2), (3, 3), (6, 2), (6, 3)])
def test_clay_batch_erasure_patterns_vs_oracle(ecx, torch_dev, k, m):
    """Non-codeword stripes through the device batch path for many erasure patterns of
    every size 1..m (all of them for Clay(2,2) and Clay(4,2), 12 random ones per size
    otherwise): single repairs (doDecodeSingle) and doDecodeMulti's IS-ordered type
    0/1/2 solves, each equal to the oracle's stage-by-stage run on every stripe."""
    import itertools
    torch = torch_dev
    n = k + m
    rng = np.random.default_rng(k * 10 + m)
    pats = []
    for size in range(1, m + 1):
        allp = [list(p) for p in itertools.combinations(range(n), size)]
        if n <= 6:
            pats += allp
        else:
            pats += [allp[i] for i in rng.choice(len(allp), min(12, len(allp)), replace=False)]
    a = ecx.ClayCodeErasureDecodingStep([0], k, m).subPacketSize
    B, S = 4096 + 48, 2
    pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 31 + k + m)
    host = pool.cpu().numpy()
    for erased in pats:
        E = len(erased)
        out = torch.full((S, E * a, B), 0x5A, dtype=torch.uint8, device="cuda")
        ecx.ClayCodeErasureDecodingStep(erased, k, m).performCodingBatch(pool, n * a * B, B, out, E * a * B, B, S, B)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        for s in range(S):
            inputs = [None if (i % n) in erased else host[s, i].copy() for i in range(n * a)]
            ref = [np.zeros(B, np.uint8) for _ in range(E * a)]
            O.Clay(k, m, erased).perform_coding(inputs, ref, B)
            for o in range(E * a):
                assert (got[s, o] == ref[o]).all(), (erased, s, o)


def test_clay_batch_unaligned_layout(ecx, torch_dev):
    """Unaligned base/strides take the byte-safe kernel path; results unchanged."""
    torch = torch_dev
    k, m, B, S, e = 4, 2, 1001, 3, 3
    stride = 48 * B + 5
    raw = torch.empty((S * stride + 64,), dtype=torch.uint8, device="cuda")
    ecx.fill_random(raw, raw.numel(), 5)
    base = raw[3:]
    outraw = torch.zeros((S * 8 * B + 64,), dtype=torch.uint8, device="cuda")
    ecx.ClayCodeErasureDecodingStep([e], k, m).performCodingBatch(base, stride, B, outraw[1:], 8 * B, B, S, B)
    torch.cuda.synchronize()
    host, got = base.cpu().numpy(), outraw[1:].cpu().numpy()
    for s in range(S):
        inputs = [None if (i % 6) == e else host[s * stride + i * B: s * stride + (i + 1) * B].copy()
                  for i in range(48)]
        ref = [np.zeros(B, np.uint8) for _ in range(8)]
        O.Clay(k, m, [e]).perform_coding(inputs, ref, B)
        for z in range(8):
            assert (got[s * 8 * B + z * B: s * 8 * B + (z + 1) * B] == ref[z]).all()


def test_rs124_two_erasure_batch_roundtrip(ecx, torch_dev):
    """BASELINE config 5 shape: RS(12,4), 4 MiB shards, erasures {0,1}, in place."""
    torch = torch_dev
    k, m, L, S = 12, 4, 4 << 20, 2
    rs = ecx.ReedSolomon.create(k, m)
    pool = torch.empty((S, 16, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 9)
    rs.encode_map().apply_batch(pool, 16 * L, L, pool, 16 * L, L, S, L)
    orig = pool.clone()
    pool[:, 0:2, :] = 0
    present = [False, False] + [True] * 14
    rs.decode_map(present).apply_batch(pool, 16 * L, L, pool, 16 * L, L, S, L)
    torch.cuda.synchronize()
    assert torch.equal(pool, orig)
    # oracle parity on a 64 KiB window of stripe 0
    host = orig[0, :, :65536].cpu().numpy()
    b = [host[i].copy() for i in range(16)]
    O.ReedSolomon(k, m).encode_parity(b, 0, 65536)
    assert all((b[i] == host[i]).all() for i in range(12, 16))


def test_rs124_random_erasure_pairs(ecx, torch_dev):
    """BASELINE config 5's "plus random pairs" (SURVEY.md 8(d)): RS(12,4) decodeMissing of
    random erasure pairs -- data+data, data+parity, parity+parity -- in place on valid
    stripes restores every shard; on non-codeword stripes it equals the oracle's
    decodeMissing (first-k-present rule) on a window that includes the ragged tail."""
    torch = torch_dev
    k, m, S = 12, 4, 2
    L, P = (1 << 20) + 208, (1 << 20) + 4096
    rs = ecx.ReedSolomon.create(k, m)
    rng = np.random.default_rng(124)
    pairs = [(0, 5), (3, 14), (12, 15), (7, 11), (1, 13)]
    pairs += [tuple(sorted(rng.choice(16, 2, replace=False).tolist())) for _ in range(5)]
    pool = torch.empty((S, 16, P), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 41)
    rs.encode_map().apply_batch(pool, 16 * P, P, pool, 16 * P, P, S, L)
    noise = torch.empty_like(pool)
    ecx.fill_random(noise, noise.numel(), 42)
    torch.cuda.synchronize()
    for pair in pairs:
        present = [i not in pair for i in range(16)]
        work = pool.clone()
        for i in pair:
            work[:, i, :L] = 0
        rs.decode_map(present).apply_batch(work, 16 * P, P, work, 16 * P, P, S, L)
        torch.cuda.synchronize()
        assert torch.equal(work[:, :, :L], pool[:, :, :L]), pair
        nc = noise.clone()
        rs.decode_map(present).apply_batch(nc, 16 * P, P, nc, 16 * P, P, S, L)
        torch.cuda.synchronize()
        w0 = L - 3000
        b = [x.copy() for x in noise[1, :, w0:L].cpu().numpy()]
        O.ReedSolomon(k, m).decode_missing(b, present, 0, L - w0)
        got = nc[1, :, w0:L].cpu().numpy()
        assert all((b[i] == got[i]).all() for i in range(16)), pair


@pytest.mark.parametrize("L", [(1 << 20) + 1008, 4 << 20])
def test_rs124_padded_pitch_one_wave_auto(ecx, torch_dev, L):
    """RS(12,4) decode on a padded shard pitch (4 MiB + 4 KiB style) runs on one-wave
    workgroups under the auto workgroup size (ecx_tune "block_threads" 0): same bytes as
    the 256-thread kernel, ragged tail included, and the non-codeword decode equals the
    oracle's decodeMissing on a sampled window."""
    torch = torch_dev
    k, m, S = 12, 4, 3
    P = L + 4096
    rs = ecx.ReedSolomon.create(k, m)
    pool = torch.empty((S, 16, P), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 19)
    present = [False, False] + [True] * 14
    outs = []
    try:
        for bt in (0, 256):
            ecx.tune("block_threads", bt)
            o = pool.clone()
            rs.decode_map(present).apply_batch(o, 16 * P, P, o, 16 * P, P, S, L)
            torch.cuda.synchronize()
            outs.append((o, ecx.last_kernel()))
    finally:
        ecx.tune("block_threads", 0)
    assert ", 64, " in outs[0][1] and ", 256, " in outs[1][1], (outs[0][1], outs[1][1])
    assert torch.equal(outs[0][0], outs[1][0])
    w0 = L - 5000  # a window that ends in the ragged tail (16-B aligned pitch: the full chunks run the fast path)
    host = pool[1, :, w0:L].cpu().numpy()
    b = [host[i].copy() for i in range(16)]
    O.ReedSolomon(k, m).decode_missing(b, present, 0, L - w0)
    got = outs[0][0][1, :, w0:L].cpu().numpy()
    assert all((b[i] == got[i]).all() for i in range(16))


def test_lrc_batch_config3(ecx, torch_dev):
    """BASELINE config 3 shape: LRC (12 data, 4 XOR groups), 64 KiB blocks, repair block 2."""
    torch = torch_dev
    B, S = 65536, 16
    enc = np.zeros((4, 16), np.uint8)
    for g in range(4):
        enc[g, 4 * g:4 * g + 3] = 1
    encmap = ecx.GfMap.from_matrix(enc, in_slot=list(range(16)), out_slot=[3, 7, 11, 15])
    pool = torch.empty((S, 16, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 31)
    encmap.apply_batch(pool, 16 * B, B, pool, 16 * B, B, S, B)
    torch.cuda.synchronize()
    host = pool[0].cpu().numpy()
    ref = O.lrc_encode(np.concatenate([host[i] for i in range(16) if (i + 1) % 4 != 0]))
    assert all((ref[i] == host[i]).all() for i in range(16))
    rs = ecx.ReedSolomon.create(3, 1)
    dm = rs.decode_map([True, True, False, True])
    out = torch.empty((S, 1, B), dtype=torch.uint8, device="cuda")
    mat, ins, outs = dm.matrix()
    assert mat.tolist() == [[1, 1, 1]] and outs.tolist() == [2]
    repair = ecx.GfMap.from_matrix(mat, in_slot=[0, 1, 3], out_slot=[0])
    repair.apply_batch(pool, 16 * B, B, out, B, B, S, B)
    torch.cuda.synchronize()
    assert torch.equal(out[:, 0], pool[:, 2])


def test_clay104_shortened_batch_roundtrip(ecx, torch_dev):
    """BASELINE config 4 shape: shortened Clay(10,4) (= Clay(12,4) with 2 virtual zero
    data nodes), 1 MiB node blocks = 256 planes x 4 KiB; encode on the GPU, erase,
    repair, compare; one stripe against the oracle (reference Clay(12,4), zero-filled)."""
    torch = torch_dev
    k, m, v, B, S = 10, 4, 2, 4096, 4
    n = k + m
    enc = ecx.ClayCodeErasureDecodingStep(list(range(k, n)), k, m, virtualUnits=v)
    a = enc.subPacketSize
    assert a == 256
    pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 404)
    par = torch.empty((S, m * a, B), dtype=torch.uint8, device="cuda")
    enc.performCodingBatch(pool, n * a * B, B, par, m * a * B, B, S, B)
    pool.view(S, a, n, B)[:, :, k:, :] = par.view(S, a, m, B)
    for e in (0, 3, 9, 10, 13):
        out = torch.empty((S, a, B), dtype=torch.uint8, device="cuda")
        ecx.ClayCodeErasureDecodingStep([e], k, m, virtualUnits=v).performCodingBatch(
            pool, n * a * B, B, out, a * B, B, S, B)
        torch.cuda.synchronize()
        assert torch.equal(out, pool.view(S, a, n, B)[:, :, e, :]), e
    # oracle: reference Clay(12,4) with the virtual nodes zero-filled, stripe 0, parity of plane 0..255
    host = pool[0].cpu().numpy()
    und = lambda r: r if r < k else r + v
    inputs = [None] * (16 * a)
    for z in range(a):
        for r in range(k):
            inputs[z * 16 + und(r)] = host[z * n + r].copy()
        for u in range(k, k + v):
            inputs[z * 16 + u] = np.zeros(B, np.uint8)
    ref = [np.zeros(B, np.uint8) for _ in range(m * a)]
    O.Clay(12, 4, [12, 13, 14, 15]).perform_coding(inputs, ref, B)
    for z in range(0, a, 17):
        for j in range(m):
            assert (host[z * n + k + j] == ref[z * m + j]).all()


def test_partial_sum_batches(ecx, torch_dev):
    """Batched partial sums along a repair chain: summing the chain's
    decodeMissingSingle contributions reproduces decodeMissing for data AND parity shards
    (the reference can only do data, bug B3); per-stripe the oracle's decodeMissingSingle
    chain matches the data rows; encode partials reproduce encodeParity."""
    torch = torch_dev
    k, m, L, S = 4, 2, 8192 + 32, 6
    rs = ecx.ReedSolomon.create(k, m)
    pool = torch.empty((S, 6, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 17)
    rs.encode_map().apply_batch(pool, 6 * L, L, pool, 6 * L, L, S, L)
    present = [True, False, True, True, True, False]  # missing data 1 and parity 5
    chain = [0, 2, 3, 4]
    acc = torch.empty((S, 2, L), dtype=torch.uint8, device="cuda")
    for c, idx in enumerate(chain):
        rs.decodePartialBatch(present, idx, pool[:, idx], 6 * L, acc, 2 * L, L, S, L, c == 0)
    torch.cuda.synchronize()
    assert torch.equal(acc[:, 0], pool[:, 1]) and torch.equal(acc[:, 1], pool[:, 5])
    host = pool[0].cpu().numpy()
    ref = [np.zeros(L, np.uint8)]
    for c, idx in enumerate(chain):
        O.ReedSolomon(k, m).decode_missing_single(host[idx].copy(), idx, c, present, ref, 0, L, c == 0)
    assert (acc[0, 0].cpu().numpy() == ref[0]).all()
    par = torch.empty((S, 2, L), dtype=torch.uint8, device="cuda")
    for i in range(k):
        rs.encodePartialBatch(i, pool[:, i], 6 * L, par, 2 * L, L, S, L, i == 0)
    torch.cuda.synchronize()
    assert torch.equal(par, pool[:, 4:6])


# ---------------------------------------------------------------- host-memory batches
@pytest.fixture
def small_host_chunks(ecx):
    """Force many pipelined chunks and ring reuse (one stripe per chunk on these layouts, even with
    the many-run rule of host_pipe.cpp); restore the defaults afterwards."""
    ecx.tune("host_chunk_kib", 16)
    ecx.tune("host_buffers", 3)
    yield
    ecx.tune("host_chunk_kib", 65536)
    ecx.tune("host_buffers", 3)


@pytest.mark.parametrize("pinned", [False, True])
def test_clay_host_batch_vs_oracle(ecx, small_host_chunks, pinned):
    """performCodingBatchHost from the full 48-slot host layout (only the 20 helper
    slots cross PCIe) equals the oracle's performCoding on every stripe."""
    k, m, B, S, e = 4, 2, 2048 + 16, 23, 1
    rng = np.random.default_rng(41)
    if pinned:
        hb = ecx.HostBuffer(S * 48 * B)
        pool = hb.array.reshape(S, 48, B)
        pool[:] = rng.integers(0, 256, (S, 48, B), dtype=np.uint8)
    else:
        pool = rng.integers(0, 256, (S, 48, B), dtype=np.uint8)
    out = np.full((S, 8, B), 0xAB, np.uint8)
    ecx.ClayCodeErasureDecodingStep([e], k, m).performCodingBatchHost(pool, 48 * B, B, out, 8 * B, B, S, B)
    for s in range(S):
        inputs = [None if (i % 6) == e else pool[s, i].copy() for i in range(48)]
        ref = [np.zeros(B, np.uint8) for _ in range(8)]
        O.Clay(k, m, [e]).perform_coding(inputs, ref, B)
        assert all((out[s, z] == ref[z]).all() for z in range(8)), s


def test_rs_host_batch_in_place_unaligned(ecx, small_host_chunks):
    """RS(12,4) decodeMissing over host stripes, in place, with a ragged shard length and a
    padded shard stride (per-slot strided copies, byte-safe kernel)."""
    k, m, L, S = 12, 4, 10001, 9
    pitch = L + 37
    rs = ecx.ReedSolomon.create(k, m)
    rng = np.random.default_rng(8)
    pool = np.zeros((S, 16, pitch), np.uint8)
    pool[:, :k, :L] = rng.integers(0, 256, (S, k, L), dtype=np.uint8)
    rs.encode_map().apply_batch_host(pool, 16 * pitch, pitch, pool, 16 * pitch, pitch, S, L)
    for s in (0, S - 1):
        b = [pool[s, i, :L].copy() for i in range(16)]
        O.ReedSolomon(k, m).encode_parity(b, 0, L)
        assert all((b[i] == pool[s, i, :L]).all() for i in range(k, 16))
    orig = pool.copy()
    present = [True] * 16
    for i in (0, 5, 13):
        present[i] = False
        pool[:, i] = 0x5A
    rs.decode_map(present).apply_batch_host(pool, 16 * pitch, pitch, pool, 16 * pitch, pitch, S, L)
    assert (pool[:, :, :L] == orig[:, :, :L]).all()
    assert (pool[:, (0, 5, 13), L:] == 0x5A).all()  # bytes past the shard untouched


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_clay_host_batch_devices_vs_oracle(ecx, small_host_chunks, devices):
    """performCodingBatchHostDevices (ecx_clay_perform_coding_batch_host_devices): a ragged
    stripe count split into contiguous ranges over the device list -- here device 0 several
    times, each entry a worker thread of its own -- equals the oracle on every stripe."""
    k, m, B, S, e = 4, 2, 4096, 7, 2
    rng = np.random.default_rng(77)
    pool = rng.integers(0, 256, (S, 48, B), dtype=np.uint8)
    out = np.full((S, 8, B), 0xCD, np.uint8)
    ecx.ClayCodeErasureDecodingStep([e], k, m).performCodingBatchHostDevices(pool, 48 * B, B, out, 8 * B, B, S, B,
                                                                              devices)
    for s in range(S):
        inputs = [None if (i % 6) == e else pool[s, i].copy() for i in range(48)]
        ref = [np.zeros(B, np.uint8) for _ in range(8)]
        O.Clay(k, m, [e]).perform_coding(inputs, ref, B)
        assert all((out[s, z] == ref[z]).all() for z in range(8)), s


def test_map_host_batch_devices_and_refusals(ecx, small_host_chunks):
    """ecx_map_apply_batch_host_devices over [0, 0] with a ragged count equals the one-device
    host batch; an unknown device id, an empty list or a null list is refused before anything
    is copied (the output stays untouched)."""
    k, m, L, S = 12, 4, 5000, 5
    rs = ecx.ReedSolomon.create(k, m)
    rng = np.random.default_rng(78)
    pool = np.zeros((S, 16, L), np.uint8)
    pool[:, :k] = rng.integers(0, 256, (S, k, L), dtype=np.uint8)
    one = pool.copy()
    emap = rs.encode_map()
    emap.apply_batch_host(one, 16 * L, L, one, 16 * L, L, S, L)
    emap.apply_batch_host_devices(pool, 16 * L, L, pool, 16 * L, L, S, L, [0, 0])
    assert (pool == one).all()
    ref = [one[S - 1, i].copy() for i in range(16)]
    ref[k:] = [np.zeros(L, np.uint8) for _ in range(m)]
    O.ReedSolomon(k, m).encode_parity(ref, 0, L)
    assert all((ref[i] == pool[S - 1, i]).all() for i in range(16))
    fresh = np.zeros((S, 16, L), np.uint8)
    fresh[:, :k] = pool[:, :k]
    for bad in ([ecx.device_count()], [0, -1], []):
        with pytest.raises(ecx.EcxError) as ei:
            emap.apply_batch_host_devices(fresh, 16 * L, L, fresh, 16 * L, L, S, L, bad)
        assert ei.value.code == -1, bad
        assert (fresh[:, k:] == 0).all()


@pytest.mark.parametrize("k,m,L,off,S", [(17, 3, 200000, 0, 6), (4, 2, 104449, 0, 5), (4, 2, 4096 * 3, 16, 4),
                                         (10, 10, 8192 + 48, 0, 3), (5, 5, 1001, 3, 4), (17, 3, 4096, 0, 3),
                                         (2, 1, 16, 0, 2), (64, 64, 4096 + 16, 0, 2), (12, 4, 3 * 4096, 0, 9),
                                         (17, 3, 200000, 5, 4), (4, 2, 4096 * 2 + 7, 9, 3)])
def test_is_parity_correct_batch_vs_oracle(ecx, torch_dev, k, m, L, off, S):
    """isParityCorrectBatch (k_gf_check, read-only): valid stripes pass; one flipped byte --
    in a data shard at byte 0, in a parity shard inside the partial last chunk, at the last
    byte -- fails exactly that stripe, as the oracle's isParityCorrect says; the shards are
    not written; firstByte / byteCount windows follow ReedSolomon.java:129-178 (a flip
    outside the window passes).  Shapes: the published RS(17,3) 200,000 B (fused partial
    chunk), RS(4,2) on the LP-block shard size (ragged: byte-safe tail), an unaligned base
    (offset 3), RS(10,10) (two 8-row tiles), a shard of one chunk and one of 16 B; and a
    firstByte off a 16-B boundary on 16-B strides (5, 9: the head up to the boundary runs
    byte-safe, the rest vectorised; the flip at firstByte lies in the head)."""
    torch = torch_dev
    n = k + m
    pitch = off + L + 32
    if off % 16:  # the unaligned-start cases on 16-B strides (the (5,5,1001,3) case keeps odd strides)
        pitch = pitch if (k, m, L) == (5, 5, 1001) else -(-pitch // 16) * 16
    rng = np.random.default_rng(k * 1000 + L)
    host = np.zeros((S, n, pitch), np.uint8)
    host[:, :k] = rng.integers(0, 256, (S, k, pitch), dtype=np.uint8)
    rs = ecx.ReedSolomon.create(k, m)
    for s in range(S):
        sh = [host[s, i] for i in range(n)]
        O.ReedSolomon(k, m).encode_parity(sh, off, L)
    pool = torch.from_numpy(host).cuda()
    verdict = torch.full((S,), 7, dtype=torch.uint8, device="cuda")
    rs.isParityCorrectBatch(pool, n * pitch, pitch, S, off, L, verdict)
    torch.cuda.synchronize()
    assert verdict.cpu().tolist() == [1] * S
    flips = {0: (0, off), S - 1: (n - 1, off + L - 1)}
    if S > 2:
        flips[1] = (k, off + L - max(1, (L % 4096) // 2))  # a parity shard, in the partial last chunk
    for s, (i, b) in flips.items():
        host[s, i, b] ^= 0x81
    pool = torch.from_numpy(host).cuda()
    before = pool.clone()
    rs.isParityCorrectBatch(pool, n * pitch, pitch, S, off, L, verdict)
    torch.cuda.synchronize()
    want = [0 if s in flips else 1 for s in range(S)]
    assert verdict.cpu().tolist() == want
    assert torch.equal(pool, before)  # read-only
    for s in range(S):
        sh = [host[s, i].copy() for i in range(n)]
        assert O.ReedSolomon(k, m).is_parity_correct(sh, off, L) == bool(want[s])
    # the same stripes from host memory (isParityCorrectBatchHost: chunks pipelined H2D through
    # k_gf_check, only the verdict bytes D2H), one device and the list [0, 0], in 16 KiB chunks
    ecx.tune("host_chunk_kib", 16)
    try:
        for devs in (None, [0, 0]):
            for win in (L, L - 1, 0):
                # a stripe fails when one of its flipped bytes lies in [off, off + win)
                expect = [0 if s in flips and flips[s][1] < off + win else 1 for s in range(S)]
                hv = np.full(S, 7, np.uint8)
                if devs is None:
                    rs.isParityCorrectBatchHost(host, n * pitch, pitch, S, off, win, hv)
                else:
                    rs.isParityCorrectBatchHostDevices(host, n * pitch, pitch, S, off, win, hv, devs)
                assert hv.tolist() == expect, (devs, win, hv.tolist())
    finally:
        ecx.tune("host_chunk_kib", 65536)
    # the window: a check that ends before the last flipped byte passes that stripe
    if L > 1:
        rs.isParityCorrectBatch(pool, n * pitch, pitch, S, off, L - 1, verdict)
        torch.cuda.synchronize()
        assert verdict.cpu().tolist()[S - 1] == 1
    # empty: no stripes, or zero bytes (every verdict 1)
    rs.isParityCorrectBatch(pool, n * pitch, pitch, 0, off, L, verdict)
    rs.isParityCorrectBatch(pool, n * pitch, pitch, S, off, 0, verdict)
    torch.cuda.synchronize()
    assert verdict.cpu().tolist() == [1] * S


def test_is_parity_correct_batch_at_benchmark_scale(ecx, torch_dev):
    """ReedSolomonBenchmark's buffer sets at scale (4,096 RS(17,3) stripes of 200,000 B, 16 GB):
    GPU encode then GPU check -- every verdict 1 -- then one byte flipped per 512th stripe fails
    exactly those (the size-independent property at BASELINE size)."""
    torch = torch_dev
    S, L = 4096, 200000
    pool = torch.empty((S, 20, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 99)
    rs = ecx.ReedSolomon.create(17, 3)
    rs.encodeParityBatch(pool, 20 * L, L, S, 0, L)
    verdict = torch.zeros(S, dtype=torch.uint8, device="cuda")
    rs.isParityCorrectBatch(pool, 20 * L, L, S, 0, L, verdict)
    torch.cuda.synchronize()
    assert bool((verdict == 1).all())
    bad = list(range(0, S, 512))
    for j, s in enumerate(bad):
        pool[s, j % 20, (j * 7919) % L] ^= 1
    rs.isParityCorrectBatch(pool, 20 * L, L, S, 0, L, verdict)
    torch.cuda.synchronize()
    v = verdict.cpu().numpy()
    assert sorted(np.nonzero(v == 0)[0].tolist()) == bad
    del pool


def test_lrc_host_batch_matches_device_batch(ecx, torch_dev):
    """The same map over the same stripes: host and device batch paths agree byte for byte."""
    torch = torch_dev
    B, S = 65536, 40
    mat = np.zeros((4, 12), np.uint8)
    for g in range(4):
        mat[g, 3 * g:3 * g + 3] = 1
    gmap = ecx.GfMap.from_matrix(mat, in_slot=[g * 4 + r for g in range(4) for r in range(3)],
                                 out_slot=[g * 4 + 3 for g in range(4)])
    dev = torch.empty((S, 16, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(dev, dev.numel(), 23)
    host = dev.cpu().numpy().copy()
    gmap.apply_batch(dev, 16 * B, B, dev, 16 * B, B, S, B)
    torch.cuda.synchronize()
    gmap.apply_batch_host(host, 16 * B, B, host, 16 * B, B, S, B)
    assert (dev.cpu().numpy() == host).all()


@pytest.mark.parametrize("k,m,v,erased,B", [(4, 2, 0, [0, 3], 4096 * 2 + 1000), (4, 2, 0, [4, 5], 3 * 1024),
                                            (10, 4, 2, [3], 4096), (6, 3, 0, [1, 7], 1024 + 16),
                                            (4, 2, 0, [1], 4096 * 3)])
def test_multitile_launch_shapes_agree(ecx, torch_dev, k, m, v, erased, B):
    """Every launch shape gives the same bytes: the LDS tile-group kernel
    (k_gf_apply_lds, 1 KiB chunks + byte-safe tail) and the one-workgroup-per-tile
    kernel with its split tables read from SGPRs only or partly from LDS
    (lds_tables 0 / 1 / 2), with `nt sc0 sc1` output stores, in chunk-major block
    order and with one-wave workgroups over 1 KiB chunks, the unstaged tile-group
    kernel (k_gf_apply_grp) and wide tiles (k_gf_apply_wide); all match the oracle on a sampled stripe.  The last
    case is a single-tile map (Clay(4,2) repair)."""
    torch = torch_dev
    step = ecx.ClayCodeErasureDecodingStep(erased, k, m, virtualUnits=v)
    n, a = k + m, step.subPacketSize
    S = 5
    pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 31)
    outs = []
    for wg, lt, sc, cm, bt, wd in ((1, 1, 0, 0, 256, 0), (0, 0, 0, 0, 256, 0), (0, 1, 0, 0, 256, 0),
                                   (0, 2, 0, 0, 256, 0), (0, 1, 1, 0, 256, 0), (0, 1, 0, 1, 256, 0),
                                   (0, 1, 0, 0, 64, 0), (0, 2, 0, 1, 64, 0), (2, 1, 0, 0, 256, 0),
                                   (0, 1, 0, 0, 256, 2), (0, 1, 0, 0, 256, -1)):
        if wg and not diag_build():
            continue  # the tile-group kernels are in the diagnostic library only (make DIAG=1)
        # wd < 0: the generated bit-plane kernel forced (ecx_tune "map_planes" 2; maps of <= 16 rows)
        ecx.tune("map_planes", 2 if wd < 0 else 0)
        wd = max(wd, 0)
        if diag_build():
            ecx.tune("wave_groups", wg)
        ecx.tune("lds_tables", lt)
        ecx.tune("store_scope", sc)
        ecx.tune("chunk_major", cm)
        ecx.tune("block_threads", bt)
        ecx.tune("wide_tiles", wd)
        o = torch.full((S, len(erased) * a, B), 7, dtype=torch.uint8, device="cuda")
        step.performCodingBatch(pool, n * a * B, B, o, len(erased) * a * B, B, S, B)
        torch.cuda.synchronize()
        outs.append(o.cpu().numpy())
    if diag_build():
        ecx.tune("wave_groups", 0)  # the defaults
    ecx.tune("lds_tables", 1)
    ecx.tune("store_scope", 0)
    ecx.tune("chunk_major", 0)
    ecx.tune("block_threads", 0)
    ecx.tune("wide_tiles", 1)
    ecx.tune("map_planes", 1)
    for o in outs[1:]:
        assert (o == outs[0]).all()
    if v == 0:
        host = pool[S - 1].cpu().numpy()
        inputs = [None if (i % n) in erased else host[i].copy() for i in range(n * a)]
        ref = [np.zeros(B, np.uint8) for _ in range(len(erased) * a)]
        O.Clay(k, m, erased).perform_coding(inputs, ref, B)
        assert all((outs[0][S - 1, j] == ref[j]).all() for j in range(len(ref)))


def test_lrc_batch_abi_encode_and_decode(ecx, torch_dev):
    """ecx_lrc_encode_batch / ecx_lrc_decode_batch on BASELINE config 3 shapes (64 KiB
    blocks): parities equal the oracle's RS(3,1) encodeParity; erasing one block in each
    of three groups and decoding in place restores every block."""
    torch = torch_dev
    B, S = 65536, 24
    pool = torch.empty((S, 16, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 71)
    ecx.LRCErasureCode.encodeBatch(pool, 16 * B, B, S, B)
    torch.cuda.synchronize()
    host = pool[S - 1].cpu().numpy()
    for g in range(4):
        b = [host[4 * g + j].copy() for j in range(4)]
        O.ReedSolomon(3, 1).encode_parity(b, 0, B)
        assert (b[3] == host[4 * g + 3]).all()
    orig = pool.clone()
    present = [True] * 16
    for i in (1, 7, 14):
        present[i] = False
        pool[:, i] = 0
    ecx.LRCErasureCode.decodeBatch(pool, 16 * B, B, present, S, B)
    torch.cuda.synchronize()
    assert torch.equal(pool, orig)


@pytest.mark.parametrize("L", [1, 4097, 300000])
def test_per_call_paths_agree(ecx, L):
    """Per-call host entry points: the pinned gather path (one H2D / one D2H), the
    zero-copy gather path (the kernel reads and writes pinned memory over PCIe) and
    the per-slot copy path give the oracle's bytes for encode, check and decodeMissing."""
    rng = np.random.default_rng(L)
    base = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(6)]
    ref = [b.copy() for b in base]
    O.ReedSolomon(4, 2).encode_parity(ref, 0, L)
    rs = ecx.ReedSolomon.create(4, 2)
    try:
        for gather_kib, zc in ((0, 0), (1 << 20, 0), (1 << 20, 1)):
            ecx.tune("host_gather_kib", gather_kib)
            ecx.tune("host_zero_copy", zc)
            sh = [b.copy() for b in base]
            rs.encodeParity(sh, 0, L)
            assert all((sh[i] == ref[i]).all() for i in range(6))
            assert rs.isParityCorrect(sh, 0, L)
            sh[5][L // 2] ^= 0x40
            assert not rs.isParityCorrect(sh, 0, L)
            sh[5][L // 2] ^= 0x40
            present = [True, False, True, False, True, True]
            sh[1][:] = 0
            sh[3][:] = 0
            rs.decodeMissing(sh, present, 0, L)
            assert all((sh[i] == ref[i]).all() for i in range(6))
    finally:
        ecx.tune("host_gather_kib", 512)
        ecx.tune("host_zero_copy", 1)


@pytest.mark.parametrize("contexts", [1, 0])
def test_per_call_concurrent_threads(ecx, contexts):
    """The reference's callers are per-process pub/sub threads (SURVEY.md section 8b,
    "Threading"); the C ABI is documented thread-safe.  Eight host threads call the
    per-call entry points at once -- two sharing one RS(4,2) codec, the others with
    their own RS or Clay(4,2) objects -- over sizes that take the zero-copy gather
    path (4 KiB, 32 KiB) and the per-slot copy path (300,000 B); every result must be
    the oracle's, with contexts leased per call (host_contexts 1: calls overlap on
    separate streams) and with one shared context (0)."""
    import threading
    ecx.tune("host_contexts", contexts)

    sizes = (4096, 32768, 300000)
    rng = np.random.default_rng(99)
    rs_data = {}
    for L in sizes:
        base = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(6)]
        ref = [b.copy() for b in base]
        O.ReedSolomon(4, 2).encode_parity(ref, 0, L)
        rs_data[L] = (base, ref)
    clay_data = {}
    for e in (0, 1, 4):
        B = 4096
        inputs = [None if (i % 6) == e else rng.integers(0, 256, B, dtype=np.uint8) for i in range(48)]
        ref = [np.zeros(B, np.uint8) for _ in range(8)]
        O.Clay(4, 2, [e]).perform_coding(inputs, ref, B)
        clay_data[e] = (inputs, ref)
    shared_rs = ecx.ReedSolomon.create(4, 2)
    errors = []

    def rs_worker(tid, rs):
        try:
            for it in range(12):
                L = sizes[(tid + it) % len(sizes)]
                base, ref = rs_data[L]
                sh = [b.copy() for b in base]
                rs.encodeParity(sh, 0, L)
                if not all((sh[i] == ref[i]).all() for i in range(6)):
                    errors.append(("encode", tid, it, L))
                present = [True] * 6
                present[it % 6] = present[(it + 3) % 6] = False
                sh[it % 6][:] = 0
                sh[(it + 3) % 6][:] = 0
                rs.decodeMissing(sh, present, 0, L)
                if not all((sh[i] == ref[i]).all() for i in range(6)):
                    errors.append(("decode", tid, it, L))
        except Exception as exc:  # noqa: BLE001 -- reported below
            errors.append(("raised", tid, repr(exc)))

    def clay_worker(tid):
        try:
            e = (0, 1, 4)[tid % 3]
            step = ecx.ClayCodeErasureDecodingStep([e], 4, 2)
            inputs, ref = clay_data[e]
            for it in range(12):
                got = [np.zeros(4096, np.uint8) for _ in range(8)]
                step.performCoding(inputs, got, 4096)
                if not all((got[o] == ref[o]).all() for o in range(8)):
                    errors.append(("clay", tid, it, e))
        except Exception as exc:  # noqa: BLE001
            errors.append(("raised", tid, repr(exc)))

    threads = [threading.Thread(target=rs_worker, args=(0, shared_rs)),
               threading.Thread(target=rs_worker, args=(1, shared_rs))]
    threads += [threading.Thread(target=rs_worker, args=(t, ecx.ReedSolomon.create(4, 2))) for t in (2, 3, 4)]
    threads += [threading.Thread(target=clay_worker, args=(t,)) for t in (5, 6, 7)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=90)
    ecx.tune("host_contexts", 1)
    assert not any(t.is_alive() for t in threads), "a worker thread hung"
    assert not errors, errors[:5]


@pytest.mark.parametrize("seed", range(24))
def test_random_maps_on_device(ecx, torch_dev, seed):
    """Random GF(256) maps of every shape class (single- and multi-tile, sparse and
    dense, coefficient-1 entries, scattered slots) applied by the device batch path at
    ring depths 2 to 24 (deep rings: single-tile maps), with and without the LDS table copy, with 256- and 64-thread
    workgroups, on wide tiles and with the skewed chunk order, on a ragged byte count
    over several stripes: each equals the oracle's table-driven product."""
    from conftest import gf_apply_numpy
    torch = torch_dev
    rng = np.random.default_rng(1000 + seed)
    n_out, n_in = int(rng.integers(1, 41)), int(rng.integers(1, 41))
    m = rng.integers(2, 256, (n_out, n_in)).astype(np.uint8)
    m[rng.random((n_out, n_in)) < 0.2] = 1
    m[rng.random((n_out, n_in)) >= rng.uniform(0.1, 1.0)] = 0
    in_slot = sorted(rng.choice(2 * n_in, n_in, replace=False).tolist())
    out_slot = rng.permutation(rng.choice(2 * n_out, n_out, replace=False)).tolist()
    gm = ecx.GfMap.from_matrix(m, in_slot=in_slot, out_slot=out_slot)
    S, L = 3, 4096 * 3 + int(rng.integers(0, 4096))
    ni, no = 2 * n_in, 2 * n_out
    inp = torch.empty((S, ni, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(inp, inp.numel(), seed)
    host = inp.cpu().numpy()
    ref = [gf_apply_numpy(m, [host[s, j] for j in in_slot]) for s in range(S)]
    for depth, lt, bt, wd, sk in ((4, 0, 256, 0, 0), (4, 2, 256, 0, 0), (8, 0, 256, 0, 0), (8, 2, 256, 0, 0),
                                  (8, 2, 64, 0, 0), (4, 0, 64, 0, 0), (2, 0, 256, 0, 0), (2, 2, 256, 0, 0),
                                  (4, 0, 256, 2, 0), (8, 0, 256, 2, 0), (8, 0, 256, 0, 2), (4, 0, 256, 0, 4),
                                  (10, 0, 256, 0, 0), (12, 0, 256, 0, 0), (16, 0, 256, 0, 0), (20, 0, 256, 0, 0),
                                  (24, 0, 256, 0, 0), (20, 2, 256, 0, 0), (4, 0, 256, 0, -2), (2, 0, 256, 0, -2)):
        # sk < 0: the bit-sliced kernel forced (ecx_tune "bitslice" 2), at ring depth 4 / 2 --
        # in the diagnostic library only (make DIAG=1)
        if sk < 0 and not diag_build():
            continue
        if diag_build():
            ecx.tune("bitslice", 2 if sk < 0 else 0)
        sk = max(sk, 0)
        ecx.tune("depth", depth)
        ecx.tune("lds_tables", lt)
        ecx.tune("block_threads", bt)
        ecx.tune("wide_tiles", wd)
        ecx.tune("skew_chunks", sk)
        out = torch.full((S, no, L), 0x5A, dtype=torch.uint8, device="cuda")
        gm.apply_batch(inp, ni * L, L, out, no * L, L, S, L)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        for s in range(S):
            for o, slot in enumerate(out_slot):
                assert (got[s, slot] == ref[s][o]).all(), (depth, lt, bt, wd, sk, s, o)
    ecx.tune("depth", 0)
    ecx.tune("lds_tables", 1)
    ecx.tune("block_threads", 0)
    ecx.tune("wide_tiles", 1)
    ecx.tune("skew_chunks", 1)
    if diag_build():
        ecx.tune("bitslice", 0)


def test_codec_eviction_frees_and_recreates_device_plans(ecx, torch_dev):
    """Reference-counted codecs on the device: 80 distinct RS(k, 2) codecs, each created,
    used for a device batch encode and destroyed, push the first ones out of the 64-codec
    idle cache (their device plans freed); re-creating and using them again rebuilds the
    plans, and every encode equals the oracle's."""
    import ctypes
    torch = torch_dev
    stats = ecx.lib().ecx_codec_stats
    stats.argtypes, stats.restype = [ctypes.POINTER(ctypes.c_int)] * 4, ctypes.c_int

    def idle():
        v = ctypes.c_int()
        stats(None, ctypes.byref(v), None, None)
        return v.value

    L, S = 256, 3

    def encode_and_check(k):
        rs = ecx.ReedSolomon.create(k, 2)
        pool = torch.zeros((S, k + 2, L), dtype=torch.uint8, device="cuda")
        data = torch.randint(0, 256, (S, k, L), dtype=torch.uint8, device="cuda")
        pool[:, :k] = data
        rs.encodeParityBatch(pool, (k + 2) * L, L, S, 0, L)
        torch.cuda.synchronize()
        host = pool.cpu().numpy()
        for s_ in (0, S - 1):
            shards = [host[s_, i].copy() for i in range(k)] + [np.zeros(L, np.uint8) for _ in range(2)]
            O.ReedSolomon(k, 2).encode_parity(shards, 0, L)
            assert all((host[s_, k + p] == shards[k + p]).all() for p in range(2)), (k, s_)
        del rs  # ecx_rs_destroy: the last reference

    for k in range(100, 180):
        encode_and_check(k)
    assert idle() == 64
    for k in (100, 101, 179):  # 100, 101 were evicted (device plans freed); 179 is idle
        encode_and_check(k)


@pytest.mark.parametrize("k,m,L,block", [(17, 3, 200000, 0), (12, 4, 3 * 65536 + 4096, 0), (4, 2, 104449, 4096),
                                         (5, 5, 1001, 64), (3, 1, 34, 0)])
def test_rs_blocked_batches_vs_oracle(ecx, torch_dev, k, m, L, block):
    """The blocked layout contract (ecx_rs_encode_parity_blocked_batch /
    ecx_rs_decode_missing_blocked_batch): stripes laid out block-major with the
    tails apart (blocked_pack), encoded / decoded in place, read back (blocked_unpack), equal the
    oracle's encodeParity / decodeMissing on the natural shards -- the published RS(17,3)
    200,000-B shape (3 blocks + a 3,392-B tail), a tail-free RS(12,4)-like shape, an odd shard
    size with 4 KiB blocks, a block of 64 B and a 34-B word (one block); decode on non-codewords."""
    torch = torch_dev
    n, S = k + m, 5
    rs = ecx.ReedSolomon.create(k, m)
    b = block or rs.blockedLayout(L)[0]
    nat = torch.empty((S, n, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(nat, nat.numel(), 900 + k + L)
    host = nat.cpu().numpy()
    flat = ecx.blocked_pack(nat, b)
    rs.encodeParityBlockedBatch(flat, S, L, block)
    torch.cuda.synchronize()
    got = ecx.blocked_unpack(flat, S, n, L, b).cpu().numpy()
    for s in (0, S - 1):
        ref = [host[s, i].copy() for i in range(n)]
        O.ReedSolomon(k, m).encode_parity(ref, 0, L)
        assert all((got[s, i] == ref[i]).all() for i in range(n)), s
    present = [True] * n
    for i in (0, n - 1)[:m]:
        present[i] = False
    flat = ecx.blocked_pack(nat, b)  # the random (non-codeword) stripes again
    rs.decodeMissingBlockedBatch(flat, present, S, L, block)
    torch.cuda.synchronize()
    got = ecx.blocked_unpack(flat, S, n, L, b).cpu().numpy()
    for s in (0, S // 2, S - 1):
        ref = [host[s, i].copy() for i in range(n)]
        O.ReedSolomon(k, m).decode_missing(ref, present, 0, L)
        assert all((got[s, i] == ref[i]).all() for i in range(n)), (s, present)


@pytest.mark.parametrize("k,m,L,block,pinned,small,devs", [
    (17, 3, 200000, 0, True, False, None), (17, 3, 200000, 0, False, True, [0, 0]),
    (12, 4, 3 * 65536, 0, True, True, None), (4, 2, 104449, 4096, False, False, [0, 0, 0]),
    (5, 5, 1001, 64, True, True, [0, 0]), (3, 1, 34, 0, False, False, None), (3, 1, 34, 0, True, True, [0, 0, 0])])
def test_rs_blocked_batches_host_vs_oracle(ecx, torch_dev, k, m, L, block, pinned, small, devs):
    """The blocked batches from HOST memory (ecx_rs_encode_parity_blocked_batch_host /
    ecx_rs_decode_missing_blocked_batch_host: the full blocks, then the tails, each a pipelined host
    batch; the _devices forms split the stripes over a device list, here device 0 two or three
    times), pageable and pinned, with the default chunks and with one stripe per chunk (ring reuse):
    every stripe equals the oracle's encodeParity / decodeMissing on its natural shards, the
    present shards of a decode are left as they were, and nothing past the batch is written."""
    torch = torch_dev
    n, S = k + m, 6
    rs = ecx.ReedSolomon.create(k, m)
    b = block or rs.blockedLayout(L)[0]
    rng = np.random.default_rng(1300 + k + L)
    nat = rng.integers(0, 256, (S, n, L), dtype=np.uint8)
    total = S * n * L
    if small:
        ecx.tune("host_chunk_kib", 16)
    try:
        for op in ("encode", "decode"):
            packed = ecx.blocked_pack(torch.from_numpy(nat), b).numpy()
            if pinned:
                hb = ecx.HostBuffer(total + 64)
                buf = hb.array
            else:
                buf = np.empty(total + 64, np.uint8)
            buf[:total] = packed
            buf[total:] = 0xE7
            present = [True] * n
            if op == "encode":
                if devs:
                    rs.encodeParityBlockedBatchHostDevices(buf, S, L, devs, block)
                else:
                    rs.encodeParityBlockedBatchHost(buf, S, L, block)
            else:
                for i in (0, n - 1)[:m]:
                    present[i] = False
                if devs:
                    rs.decodeMissingBlockedBatchHostDevices(buf, present, S, L, devs, block)
                else:
                    rs.decodeMissingBlockedBatchHost(buf, present, S, L, block)
            assert (buf[total:] == 0xE7).all()
            got = ecx.blocked_unpack(torch.from_numpy(buf[:total].copy()), S, n, L, b).numpy()
            for s in range(S):
                ref = [nat[s, i].copy() for i in range(n)]
                if op == "encode":
                    O.ReedSolomon(k, m).encode_parity(ref, 0, L)
                else:
                    O.ReedSolomon(k, m).decode_missing(ref, present, 0, L)
                assert all((got[s, i] == ref[i]).all() for i in range(n)), (op, s)
                assert all((got[s, i] == nat[s, i]).all() for i in range(n) if present[i] and (op == "decode" or i < k))
    finally:
        ecx.tune("host_chunk_kib", 65536)


@pytest.mark.parametrize("k,m", [(4, 2), (12, 4), (3, 1)])
def test_rs_batch_codec_entry_points(ecx, torch_dev, k, m):
    """ecx_rs_encode_parity_batch / ecx_rs_decode_missing_batch: encodeParity and
    decodeMissing over many device-resident stripes, in place, with a byte window
    (offset, ragged count) and a padded shard pitch.  Every stripe matches the oracle's
    encode_parity / decode_missing on the same bytes, including non-codeword inputs
    (the exact first-k-present map), for several erasure patterns."""
    torch = torch_dev
    n, S, pitch, off, cnt = k + m, 4, 3072 + 16, 16, 2983
    rs = ecx.ReedSolomon.create(k, m)
    dev = torch.empty((S, n, pitch), dtype=torch.uint8, device="cuda")
    ecx.fill_random(dev, dev.numel(), 77 + k)
    host = dev.cpu().numpy()
    rs.encodeParityBatch(dev, n * pitch, pitch, S, off, cnt)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    for s in range(S):
        ref = [host[s, i].copy() for i in range(n)]
        O.ReedSolomon(k, m).encode_parity(ref, off, cnt)
        assert all((got[s, i] == ref[i]).all() for i in range(n)), s
    rng = np.random.default_rng(k)
    for _ in range(4):
        present = [True] * n
        for i in rng.choice(n, m, replace=False):
            present[i] = False
        dev = torch.empty((S, n, pitch), dtype=torch.uint8, device="cuda")
        ecx.fill_random(dev, dev.numel(), int(rng.integers(1 << 30)))  # non-codeword stripes
        host = dev.cpu().numpy()
        rs.decodeMissingBatch(dev, present, n * pitch, pitch, S, off, cnt)
        torch.cuda.synchronize()
        got = dev.cpu().numpy()
        for s in range(S):
            ref = [host[s, i].copy() for i in range(n)]
            O.ReedSolomon(k, m).decode_missing(ref, present, off, cnt)
            assert all((got[s, i] == ref[i]).all() for i in range(n)), (present, s)
    with pytest.raises(ecx.EcxError) as e:
        rs.decodeMissingBatch(dev, [False] * (m + 1) + [True] * (k - 1), n * pitch, pitch, S, off, cnt)
    assert e.value.code == -2


@pytest.mark.parametrize("off,pitch,cnt", [(4, 3072 + 20, 2990), (8, 4096 + 8, 4000), (1, 3072 + 17, 2983),
                                            (0, 200000, 200000), (0, 200000 + 4, 200000 - 4)])
def test_rs173_byte_safe_alignment_classes(ecx, torch_dev, off, pitch, cnt):
    """RS(17,3) encodeParity over device stripes whose lanes fall in each alignment class of
    the byte-safe kernels (apply.hpp load_partial / store_partial): 16-B aligned full lanes
    of a tail chunk (200,000-B shards, the published benchmark's shape), dword-aligned
    layouts (offset 4 / 8, pitch = 4 mod 16), byte-aligned ones, and ragged counts.
    Every stripe equals the oracle's encode_parity on the same bytes."""
    torch = torch_dev
    k, m, S = 17, 3, 3
    n = k + m
    rs = ecx.ReedSolomon.create(k, m)
    dev = torch.empty((S, n, pitch), dtype=torch.uint8, device="cuda")
    ecx.fill_random(dev, dev.numel(), 1703 + off)
    host = dev.cpu().numpy()
    rs.encodeParityBatch(dev, n * pitch, pitch, S, off, cnt)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    for s in range(S):
        ref = [host[s, i].copy() for i in range(n)]
        O.ReedSolomon(k, m).encode_parity(ref, off, cnt)
        assert all((got[s, i] == ref[i]).all() for i in range(n)), s


@pytest.mark.parametrize("n_out", [1, 2, 3, 4])
def test_small_tile_variants(ecx, torch_dev, n_out):
    """Single-tile maps of at most 2 / 4 rows on the small-tile kernel variants
    (ecx_tune "small_tiles"): ring depths 4, 8 and 12 (tiles padded to multiples of
    12), 1 to 24 entries, coefficient-1 entries, an unaligned tail; each equals the
    8-row kernel and the oracle's table-driven product."""
    from conftest import gf_apply_numpy
    torch = torch_dev
    rng = np.random.default_rng(50 + n_out)
    for n_in in (1, 3, 12, 13, 24):
        m = rng.integers(1, 256, (n_out, n_in)).astype(np.uint8)
        m[rng.random((n_out, n_in)) < 0.2] = 1
        gm = ecx.GfMap.from_matrix(m, in_slot=list(range(n_in)), out_slot=list(range(n_out)))
        S, L = 3, 4096 * 2 + 100
        inp = torch.empty((S, n_in, L), dtype=torch.uint8, device="cuda")
        ecx.fill_random(inp, inp.numel(), n_in)
        host = inp.cpu().numpy()
        ref = [gf_apply_numpy(m, [host[s, j] for j in range(n_in)]) for s in range(S)]
        for st, depth in ((0, 0), (2, 0), (1, 4), (1, 8), (1, 12), (1, 0)):
            ecx.tune("small_tiles", st)
            ecx.tune("depth", depth)
            out = torch.full((S, n_out, L), 0xA5, dtype=torch.uint8, device="cuda")
            gm.apply_batch(inp, n_in * L, L, out, n_out * L, L, S, L)
            torch.cuda.synchronize()
            got = out.cpu().numpy()
            for s in range(S):
                for o in range(n_out):
                    assert (got[s, o] == ref[s][o]).all(), (n_in, st, depth, s, o)
    ecx.tune("small_tiles", 2)
    ecx.tune("depth", 0)


def test_small_tiles_auto_picks_lrc_repair(ecx, torch_dev):
    """ecx_tune "small_tiles" 2 (auto): an LRC block repair (1 row over 3 inputs, 16-B
    aligned layout) runs the 2-row kernel variant, a 4-row LRC encode the 8-row kernel,
    and both give the forced-off kernel's bytes."""
    torch = torch_dev
    S, L = 4, 4096 * 2 + 96
    inp = torch.empty((S, 16, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(inp, inp.numel(), 12)
    enc = np.zeros((4, 16), np.uint8)
    for g in range(4):
        enc[g, 4 * g:4 * g + 3] = 1
    cases = [(ecx.GfMap.from_matrix(np.array([[1, 1, 1]], np.uint8), in_slot=[0, 1, 3], out_slot=[0]), 1, ", 2>"),
             (ecx.GfMap.from_matrix(enc[:, :15], in_slot=list(range(15)), out_slot=[0, 1, 2, 3]), 4, ", 8>")]
    try:
        for gm, n_out, tail in cases:
            outs = []
            for st in (2, 0):
                ecx.tune("small_tiles", st)
                o = torch.zeros((S, n_out, L), dtype=torch.uint8, device="cuda")
                gm.apply_batch(inp, 16 * L, L, o, n_out * L, L, S, L)
                torch.cuda.synchronize()
                outs.append((o, ecx.last_kernel()))
            assert outs[0][1].endswith(tail), outs[0][1]
            assert outs[1][1].endswith(", 8>"), outs[1][1]
            assert torch.equal(outs[0][0], outs[1][0])
    finally:
        ecx.tune("small_tiles", 2)


@pytest.mark.parametrize("nbytes", [8192 * 3 + 4096, 4096 * 9 + 100, 65536])
def test_skew_chunks_agree(ecx, torch_dev, nbytes):
    """k_gf_apply_skew (ecx_tune "skew_chunks" 2 / 4: several chunks per workgroup,
    rotated chunk order; on 256-thread workgroups, and in the diagnostic build on one-wave
    workgroups, whose 1 KiB columns take the same 4 KiB-spaced rotation) gives the bytes of the one-chunk kernel for 2-,
    4- and 8-row single-tile maps, with chunk counts that leave a remainder for the
    one-chunk kernel and a ragged tail, in place (RS) and with accumulation (partial sums)."""
    torch = torch_dev
    S = 3
    rs = ecx.ReedSolomon.create(12, 4)
    maps = [rs.decode_map([False, False] + [True] * 14)]                  # 2 rows
    encm = np.zeros((4, 16), np.uint8)
    for g in range(4):
        encm[g, 4 * g:4 * g + 3] = 1
    maps.append(ecx.GfMap.from_matrix(encm, in_slot=list(range(16)), out_slot=[3, 7, 11, 15]))  # 4 rows
    maps.append(ecx.ClayCodeErasureDecodingStep([1], 4, 2).map())         # 8 rows
    pitch = nbytes + 512
    src = torch.empty((S, 48, pitch), dtype=torch.uint8, device="cuda")
    ecx.fill_random(src, src.numel(), 11)
    try:
        for mp in maps:
            nin = int(mp.matrix()[1].max()) + 1
            nout = int(mp.matrix()[2].max()) + 1
            outs = []
            for bt in (0, 256, 64):
                ecx.tune("block_threads", bt)
                for skew in (0, 2, 4, 1):
                    ecx.tune("skew_chunks", skew)
                    for acc in (False, True):
                        o = torch.zeros((S, nout, pitch), dtype=torch.uint8, device="cuda")
                        if acc:
                            o.fill_(0x5A)
                            mp.accumulate_batch(src, 48 * pitch, pitch, o, nout * pitch, pitch, S, nbytes)
                        else:
                            mp.apply_batch(src, 48 * pitch, pitch, o, nout * pitch, pitch, S, nbytes)
                        torch.cuda.synchronize()
                        outs.append((bt, skew, acc, o, ecx.last_kernel()))
            for bt, skew, acc, o, kern in outs:
                ref = [x for b2, s2, a2, x, _ in outs if b2 == 0 and s2 == 0 and a2 == acc][0]
                assert torch.equal(o, ref), (mp.info(), bt, skew, acc, nin, kern)
            if diag_build() and nbytes == 65536 and mp.info()["n_out"] <= 4:  # one-wave skew: diagnostic build
                assert any(k.startswith("k_gf_apply_skew") and k.endswith(", 64>") for *_, k in outs), outs
    finally:
        ecx.tune("skew_chunks", 1)
        ecx.tune("block_threads", 0)


@pytest.mark.parametrize("nbytes", [200000, 2 * 4096 + 16, 4096 + 4080, 1024 + 48, 64, 4000])
def test_partial_last_chunk_in_main_launch(ecx, torch_dev, nbytes):
    """A shard whose byte count is a multiple of 16 but not of the chunk (RS(17,3) on the
    published 200,000-B shards) runs its partial last chunk in the main k_gf_apply launch
    as a workgroup over the shard's last chunk-sized window that stores only the partial
    chunk (kernels.hip launch_apply_core); shards shorter than one chunk and layouts whose
    outputs are inputs of the same launch keep the byte-safe launch.  RS(17,3) encode in place
    (3 rows), a 2-row decode to a separate buffer in 256-thread and one-wave workgroups,
    overwrite and accumulate, and an in-place map whose output slot is also an input slot:
    every result equals the oracle's, and no byte outside the shards changes."""
    torch = torch_dev
    S = 5
    pitch = nbytes + 4096 + 48  # guard bytes after every slot (and 16-B aligned slots)
    rs = ecx.ReedSolomon.create(17, 3)
    pool = torch.empty((S, 20, pitch), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 5)
    before = pool.clone()
    rs.encode_map().apply_batch(pool, 20 * pitch, pitch, pool, 20 * pitch, pitch, S, nbytes)
    torch.cuda.synchronize()
    host, ref_host = pool.cpu().numpy(), before.cpu().numpy()
    for s in (0, S - 1):
        shards = [ref_host[s, i, :nbytes].copy() for i in range(20)]
        O.ReedSolomon(17, 3).encode_parity(shards, 0, nbytes)
        for i in range(20):
            assert (host[s, i, :nbytes] == shards[i]).all(), (s, i)
    assert (host[:, :, nbytes:] == ref_host[:, :, nbytes:]).all()  # nothing past the shards
    # 2-row decode to a separate buffer, both workgroup sizes, overwrite and accumulate
    r12 = ecx.ReedSolomon.create(12, 4)
    mat, ins, outs = r12.decode_map([False, False] + [True] * 14).matrix()
    dmap = r12.decode_map([False, False] + [True] * 14)
    src = pool[:, :16]
    try:
        for bt in (0, 256, 64):
            ecx.tune("block_threads", bt)
            for acc in (False, True):
                o = torch.full((S, 2, pitch), 0x3C if acc else 0, dtype=torch.uint8, device="cuda")
                if acc:
                    dmap.accumulate_batch(pool, 20 * pitch, pitch, o, 2 * pitch, pitch, S, nbytes)
                else:
                    dmap.apply_batch(pool, 20 * pitch, pitch, o, 2 * pitch, pitch, S, nbytes)
                torch.cuda.synchronize()
                oh = o.cpu().numpy()
                for s in (0, S - 1):
                    want = gf_apply_numpy(mat, [host[s, int(j), :nbytes] for j in ins])
                    for r in range(2):
                        w = want[r] ^ np.uint8(0x3C) if acc else want[r]
                        assert (oh[s, int(outs[r]), :nbytes] == w).all(), (bt, acc, s, r)
                assert (oh[:, :, nbytes:] == (0x3C if acc else 0)).all(), (bt, acc)
    finally:
        ecx.tune("block_threads", 0)
    del src
    # in place, an output slot that is also an input slot (slot 0 <- slot 0 + 2 * slot 1):
    # every output byte must come from the inputs as they were before the launch
    gm = ecx.GfMap.from_matrix(np.array([[1, 2]], np.uint8), in_slot=[0, 1], out_slot=[0])
    buf = pool[:, :2].contiguous()
    b0 = buf.cpu().numpy()
    gm.apply_batch(buf, 2 * pitch, pitch, buf, 2 * pitch, pitch, S, nbytes)
    torch.cuda.synchronize()
    b1 = buf.cpu().numpy()
    want = gf_apply_numpy(np.array([[1, 2]], np.uint8), [b0[:, 0, :nbytes].reshape(-1), b0[:, 1, :nbytes].reshape(-1)])[0]
    assert (b1[:, 0, :nbytes].reshape(-1) == want).all()
    assert (b1[:, 1] == b0[:, 1]).all() and (b1[:, 0, nbytes:] == b0[:, 0, nbytes:]).all()


@pytest.mark.parametrize("S", [7, 16])
def test_stagger_unit_orders_agree(ecx, torch_dev, S):
    """The stagger unit order (ecx_tune "stagger" G: G stripes interleaved, stripe j of a
    group starting at chunk j*C/G, stripes past the last whole group stripe-major) is a
    bijection of the (stripe, chunk) units for every G, under 4 KiB and one-wave workgroups
    and skewed chunks, with a ragged tail chunk and a stripe count that leaves a partial
    group: every setting writes the bytes of the stripe-major launch, and those equal the
    oracle's decodeMissing on a stripe, in overwrite and in accumulate mode."""
    torch = torch_dev
    L = 9 * 4096 + 1000
    pitch = (L + 512 + 15) // 16 * 16  # 16-B aligned slots: the full chunks run the fast kernels
    rs = ecx.ReedSolomon.create(12, 4)
    dmap = rs.decode_map([False, False] + [True] * 14)
    src = torch.empty((S, 16, pitch), dtype=torch.uint8, device="cuda")
    ecx.fill_random(src, src.numel(), 71)
    outs = {}
    try:
        for G in (0, 2, 3, 4, 8, 64):
            for bt, skew in ((256, 0), (64, 0), (256, 4), (256, 2), (64, 4), (64, 2)):
                ecx.tune("stagger", G)
                ecx.tune("block_threads", bt)
                ecx.tune("skew_chunks", skew)
                for acc in (False, True):
                    o = torch.full((S, 2, pitch), 0x5A if acc else 0, dtype=torch.uint8, device="cuda")
                    if acc:
                        dmap.accumulate_batch(src, 16 * pitch, pitch, o, 2 * pitch, pitch, S, L)
                    else:
                        dmap.apply_batch(src, 16 * pitch, pitch, o, 2 * pitch, pitch, S, L)
                    torch.cuda.synchronize()
                    outs[(G, bt, skew, acc)] = o
    finally:
        ecx.tune("stagger", 0)
        ecx.tune("block_threads", 0)
        ecx.tune("skew_chunks", 1)
    for (G, bt, skew, acc), o in outs.items():
        assert bool(torch.equal(o, outs[(0, 256, 0, acc)])), (G, bt, skew, acc)
    host = src[S - 1].cpu().numpy()
    shards = [np.zeros(L, np.uint8) if i < 2 else host[i, :L].copy() for i in range(16)]
    O.ReedSolomon(12, 4).decode_missing(shards, [i >= 2 for i in range(16)], 0, L)
    got = outs[(0, 256, 0, False)][S - 1].cpu().numpy()
    assert (got[0, :L] == shards[0]).all() and (got[1, :L] == shards[1]).all()


def test_every_product_on_device(ecx, torch_dev):
    """Every GF(256) product c*x through the device kernel's split tables: a 256 x 1
    map whose row c has coefficient c (0 and 1 included), over an input holding every
    byte value at every lane position, equals the oracle's MULTIPLICATION_TABLE
    (Galois.java:178,298-306) -- for each byte lane of the 16-B loads and for the
    ragged byte-safe tail."""
    torch = torch_dev
    mt = O.mul_table()
    gm = ecx.GfMap.from_matrix(np.arange(256, dtype=np.uint8).reshape(256, 1), in_slot=[0],
                               out_slot=list(range(256)))
    L = 256 * 17 + 5  # every byte value at 17 different 16-B lane offsets, plus a ragged tail
    x = (np.arange(L) * 7 + np.arange(L) // 256) % 256
    inp = torch.from_numpy(x.astype(np.uint8)).reshape(1, 1, L).cuda()
    out = torch.zeros((1, 256, L), dtype=torch.uint8, device="cuda")
    gm.apply_batch(inp, L, L, out, 256 * L, L, 1, L)
    torch.cuda.synchronize()
    got = out.cpu().numpy()[0]
    assert (got == mt[:, x]).all()


def test_code_some_shards_plan_cache(ecx):
    """CodingLoop.codeSomeShards / checkSomeShards / InputOutputByteTableCodingLoopSingle
    with the plan cache: repeated matrices (hits), matrices differing in one
    coefficient or in shape (separate entries), and a cache of 2 plans cycled through
    5 matrices (evictions) all give the oracle's bytes."""
    rng = np.random.default_rng(77)
    mats = [rng.integers(0, 256, (2, 4), dtype=np.uint8) for _ in range(3)]
    mats.append(mats[0].copy())
    mats[3][1, 2] ^= 0x11                      # one coefficient apart from mats[0]
    mats.append(rng.integers(0, 256, (3, 4), dtype=np.uint8))  # another shape
    loop = ecx.CodingLoop()
    try:
        for cap in (256, 2, 0):
            ecx.tune("plan_cache", cap)
            for it in range(3):
                for mi, m in enumerate(mats):
                    L = 1000 + 37 * it + mi
                    ins = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(4)]
                    outs = [np.zeros(L, np.uint8) for _ in range(m.shape[0])]
                    ref = [np.zeros(L, np.uint8) for _ in range(m.shape[0])]
                    O.code_some_shards(list(m), ins, ref, 0, L)
                    loop.codeSomeShards(m, ins, 4, outs, m.shape[0], 0, L)
                    assert all((a == b).all() for a, b in zip(outs, ref)), (cap, it, mi)
                    assert loop.checkSomeShards(m, ins, 4, outs, m.shape[0], 0, L)
                    outs[-1][L // 3] ^= 1
                    assert not loop.checkSomeShards(m, ins, 4, outs, m.shape[0], 0, L)
                    x = rng.integers(0, 256, L, dtype=np.uint8)
                    o = rng.integers(0, 256, L, dtype=np.uint8)
                    exp = o ^ O.mul_table()[m[0][1]][x]
                    ecx.InputOutputByteTableCodingLoopSingle().codeSomeShards(m, x, 1, o, 0, 0, L, False)
                    assert (o == exp).all()
    finally:
        ecx.tune("plan_cache", 256)


def test_rs_max_shards_on_device(ecx):
    """The largest codec the reference accepts (ReedSolomon.java:48-50: at most 256
    shards): RS(224,32) encode and a 32-shard decode (data and parity mixed) through
    the per-call host path, against the oracle; one more shard is rejected."""
    k, m, L = 224, 32, 4096 + 3
    rng = np.random.default_rng(256)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    a = [d.copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(m)]
    b = [d.copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(m)]
    rs = ecx.ReedSolomon.create(k, m)
    rs.encodeParity(a, 0, L)
    O.ReedSolomon(k, m).encode_parity(b, 0, L)
    assert all((x == y).all() for x, y in zip(a, b))
    erased = sorted(rng.choice(k + m, m, replace=False).tolist())
    present = [i not in erased for i in range(k + m)]
    t = [s.copy() for s in a]
    for i in erased:
        t[i][:] = 0
    rs.decodeMissing(t, present, 0, L)
    assert all((x == y).all() for x, y in zip(a, t)), erased
    with pytest.raises(ecx.EcxError) as e:
        ecx.ReedSolomon.create(k, m + 1)
    assert e.value.code == -4


def test_batch_empty_calls_are_noops(ecx, torch_dev):
    """Zero stripes or a zero byte count (the reference's zero-size encode,
    ReedSolomonTest.java:32-37, at the batch level) launch nothing and touch nothing."""
    torch = torch_dev
    B = 4096
    pool = torch.full((2, 48, B), 7, dtype=torch.uint8, device="cuda")
    out = torch.full((2, 8, B), 9, dtype=torch.uint8, device="cuda")
    step = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
    step.performCodingBatch(pool, 48 * B, B, out, 8 * B, B, 0, B)
    step.performCodingBatch(pool, 48 * B, B, out, 8 * B, B, 2, 0)
    rs = ecx.ReedSolomon.create(12, 4)
    rs.encodeParityBatch(pool, 48 * B, B, 0, 0, B)
    rs.encodeParityBatch(pool, 48 * B, B, 2, 0, 0)
    torch.cuda.synchronize()
    assert (out == 9).all() and (pool == 7).all()


@pytest.mark.parametrize("stride", [(1 << 31) - 8192, (1 << 31) + 4096])
def test_multitile_slot_offset_near_2gib(ecx, torch_dev, stride):
    """launch_apply's offsets32 gate (kernels.hip): the buffer-descriptor kernels
    (multi-tile maps with LDS tables, wide tiles) address an input slot by a 32-bit
    scalar offset, valid only while max_in_slot * in_slot_stride + 4 KiB < 2^31.  A
    16 x 2 map (two 8-row tiles sharing both inputs) with slot 1 just under and just
    over 2 GiB from slot 0 -- the descriptor path, and the 64-bit fallback -- equals
    the oracle's table product, with wide tiles on and off, and with the generated
    bit-plane kernel forced (map_planes 2: it runs under the limit and yields to the
    64-bit composed kernels over it)."""
    from conftest import gf_apply_numpy
    torch = torch_dev
    rng = np.random.default_rng(stride & 0xFFFF)
    m = rng.integers(1, 256, (16, 2)).astype(np.uint8)
    L = 8192
    gm = ecx.GfMap.from_matrix(m, in_slot=[0, 1], out_slot=list(range(16)))
    buf = torch.empty(stride + L, dtype=torch.uint8, device="cuda")
    ecx.fill_random(buf[:L], L, 7)
    ecx.fill_random(buf[stride:], L, 8)
    x0, x1 = buf[:L].cpu().numpy(), buf[stride:].cpu().numpy()
    ref = gf_apply_numpy(m, [x0, x1])
    try:
        for wide, planes in ((0, 0), (2, 0), (1, 2)):
            ecx.tune("wide_tiles", wide)
            ecx.tune("map_planes", planes)
            out = torch.full((16, L), 0x5A, dtype=torch.uint8, device="cuda")
            gm.apply_batch(buf, stride + L, stride, out, 16 * L, L, 1, L)
            torch.cuda.synchronize()
            assert (out.cpu().numpy() == ref).all(), (stride, wide, ecx.last_kernel())
            if planes:
                assert (ecx.last_kernel() == "k_map_planes") == (stride < (1 << 31)), ecx.last_kernel()
    finally:
        ecx.tune("wide_tiles", 1)
        ecx.tune("map_planes", 1)
    del buf
    torch.cuda.empty_cache()


@pytest.mark.diag
@pytest.mark.parametrize("case", ["clay104", "clay42", "rs124", "dense40x24", "ones"])
@pytest.mark.parametrize("depth", [2, 4])
def test_bitslice_kernel_vs_table_product(ecx, torch_dev, case, depth):
    """k_gf_bits (apply_bits.hip, forced by ecx_tune "bitslice" 2) equals the oracle's
    table-driven product of the map on every stripe: maps with 32 tiles (Clay(10,4)),
    one tile (Clay(4,2), RS(12,4)), a dense random map and an all-ones map, over
    whole 4 KiB chunks plus a byte-safe tail."""
    from conftest import gf_apply_numpy
    torch = torch_dev
    rng = np.random.default_rng(77)
    if case == "clay104":
        m, ins, outs = ecx.ClayCodeErasureDecodingStep([3], 10, 4, virtualUnits=2).map().matrix()
    elif case == "clay42":
        m, ins, outs = ecx.ClayCodeErasureDecodingStep([1], 4, 2).map().matrix()
    elif case == "rs124":
        m, ins, outs = ecx.ReedSolomon.create(12, 4).decode_map([False, False] + [True] * 14).matrix()
    elif case == "dense40x24":
        m = rng.integers(0, 256, (40, 24)).astype(np.uint8)
        ins, outs = np.arange(24), np.arange(40)
    else:
        m = np.ones((16, 20), np.uint8)
        ins, outs = np.arange(20), np.arange(16)
    gm = ecx.GfMap.from_matrix(m, in_slot=[int(i) for i in ins], out_slot=[int(o) for o in outs])
    ni, no = int(max(ins)) + 1, int(max(outs)) + 1
    S, L = 3, 4096 * 2 + 112  # 16-B aligned rows (the bit-sliced kernel's layout) with a tail
    inp = torch.empty((S, ni, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(inp, inp.numel(), 5)
    host = inp.cpu().numpy()
    try:
        ecx.tune("bitslice", 2)
        ecx.tune("depth", depth)
        out = torch.full((S, no, L), 0x5A, dtype=torch.uint8, device="cuda")
        gm.apply_batch(inp, ni * L, L, out, no * L, L, S, L)
        torch.cuda.synchronize()
        assert ecx.last_kernel() == "k_gf_bits<%s, %d>" % ("true" if len(m) <= 8 else "false", depth)
    finally:
        ecx.tune("bitslice", 0)
        ecx.tune("depth", 0)
    got = out.cpu().numpy()
    for s in range(S):
        ref = gf_apply_numpy(m, [host[s, j] for j in ins])
        for o, slot in enumerate(outs):
            bad = np.nonzero(got[s, slot] != ref[o])[0]
            assert bad.size == 0, (case, s, o, bad[:8], got[s, slot][bad[:8]], ref[o][bad[:8]])


@pytest.mark.diag
@pytest.mark.parametrize("case", ["clay104", "clay42", "rs124", "dense40x24", "ones", "dense8x30"])
@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("acc", [False, True])
def test_lds_lut_kernel_vs_table_product(ecx, torch_dev, case, mode, acc):
    """k_gf_lut (apply_lut.hip, forced by ecx_tune "lds_lut"): mode 1 (log/antilog tables
    in LDS) on every map, mode 2 (one product row per coefficient, single-tile maps of
    <= 256 general coefficients) where it applies, overwriting or accumulating, equals
    the oracle's table-driven product on every stripe, over whole 4 KiB chunks plus a
    byte-safe tail; more stripes than one persistent grid covers at once."""
    from conftest import gf_apply_numpy
    torch = torch_dev
    rng = np.random.default_rng(78)
    if case == "clay104":
        m, ins, outs = ecx.ClayCodeErasureDecodingStep([3], 10, 4, virtualUnits=2).map().matrix()
    elif case == "clay42":
        m, ins, outs = ecx.ClayCodeErasureDecodingStep([1], 4, 2).map().matrix()
    elif case == "rs124":
        m, ins, outs = ecx.ReedSolomon.create(12, 4).decode_map([False, False] + [True] * 14).matrix()
    elif case.startswith("dense"):
        r, c = (int(v) for v in case[5:].split("x"))
        m = rng.integers(0, 256, (r, c)).astype(np.uint8)
        ins, outs = np.arange(c), np.arange(r)
    else:
        m = np.ones((16, 20), np.uint8)
        ins, outs = np.arange(20), np.arange(16)
    m = np.asarray(m)
    single_tile = len(m) <= 8
    runs_lut = mode == 1 or (single_tile and int((m > 1).sum()) <= 256)
    gm = ecx.GfMap.from_matrix(m, in_slot=[int(i) for i in ins], out_slot=[int(o) for o in outs])
    ni, no = int(max(ins)) + 1, int(max(outs)) + 1
    S = 3 if case == "clay104" else 700  # Clay(4,2): 700 stripes x 2 chunks > 256 CUs x occupancy
    L = 4096 * 2 + 112
    inp = torch.empty((S, ni, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(inp, inp.numel(), 6)
    host = inp.cpu().numpy()
    out = torch.empty((S, no, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(out, out.numel(), 7)
    before = out.cpu().numpy()
    try:
        ecx.tune("lds_lut", mode)
        if acc:
            gm.accumulate_batch(inp, ni * L, L, out, no * L, L, S, L)
        else:
            gm.apply_batch(inp, ni * L, L, out, no * L, L, S, L)
        torch.cuda.synchronize()
        kern = ecx.last_kernel()
    finally:
        ecx.tune("lds_lut", 0)
    if runs_lut:
        assert kern == "k_gf_lut<%d, %s>" % (mode - 1, "true" if single_tile else "false"), kern
    else:
        assert not kern.startswith("k_gf_lut"), kern
    got = out.cpu().numpy()
    for s in sorted({0, 1, S // 2, S - 1}):
        ref = gf_apply_numpy(m, [host[s, j] for j in ins])
        for o, slot in enumerate(outs):
            want = ref[o] ^ before[s, slot] if acc else ref[o]
            bad = np.nonzero(got[s, slot] != want)[0]
            assert bad.size == 0, (case, mode, s, o, bad[:8])


@pytest.mark.parametrize("k,m,v,e,B,S", [(4, 2, 0, 1, 4096 * 2 + 112, 3), (4, 2, 0, 4, 4096, 9), (4, 2, 0, 0, 8192, 3),
                                         (10, 4, 2, 3, 4096, 3), (10, 4, 2, 13, 4096 + 16, 3), (10, 4, 2, 9, 4096, 17),
                                         (12, 4, 0, 5, 4096, 3), (12, 4, 0, 15, 8192 + 512, 5), (8, 4, 0, 0, 4096, 3),
                                         (6, 3, 0, 2, 4096 * 2, 5), (2, 2, 0, 3, 4096, 3)])
def test_clay_rtc_kernel_vs_composed_and_oracle(ecx, torch_dev, k, m, v, e, B, S):
    """The per-helper-plane repair kernel (clay_rtc.hpp: generated for the repair
    program and compiled with hiprtc) over whole 4 KiB chunks, the composed-map kernel
    over the tail: every stripe equals the composed-map kernel alone (ecx_tune
    "clay_rtc" 0), and a sampled stripe equals the oracle (unshortened codes)."""
    torch = torch_dev
    step = ecx.ClayCodeErasureDecodingStep([e], k, m, virtualUnits=v)
    n, a = k + m, step.subPacketSize
    pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 41 + e)
    # (clay_rtc, rtc_xcd, rtc_group, rtc_persist, rtc_lookahead)
    modes = [(0, 0, 0, 0, 1), (2, 0, 0, 0, 1), (2, 1, 0, 0, 1)]  # composed; per-plane, both block orders
    if m == 4:
        # the plane-group kernel: both block orders, persistent grid, every schedule bit
        modes += [(2, 0, 1, 0, 1), (2, 1, 1, 0, 1), (2, 2, 1, 0, 1), (2, 3, 1, 0, 1), (2, 4, 1, 0, 1), (2, 1, 1, 0, 0),
                  (2, 1, 1, 0, 3), (2, 1, 1, 0, 5), (2, 1, 1, 0, 6), (2, 1, 1, 0, 12)]
        if diag_build():
            modes += [(2, 1, 1, 2, 1)]  # the persistent grid: diagnostic library only
    outs = {}
    try:
        for rtc, xcd, grp, persist, la in modes:
            ecx.tune("clay_rtc", rtc)
            ecx.tune("rtc_xcd", xcd)
            ecx.tune("rtc_group", grp)
            if diag_build():
                ecx.tune("rtc_persist", persist)
            ecx.tune("rtc_lookahead", la)
            ecx.tune("rtc_sched", 2 if la == 1 else 0)  # the default schedule, and rtc_lookahead's for the rest
            o = torch.full((S, a, B), 0x77, dtype=torch.uint8, device="cuda")
            step.performCodingBatch(pool, n * a * B, B, o, a * B, B, S, B)
            torch.cuda.synchronize()
            outs[(rtc, xcd, grp, persist, la)] = (o.cpu().numpy(), ecx.last_kernel())
    finally:
        ecx.tune("clay_rtc", 1)
        ecx.tune("rtc_xcd", 2)
        ecx.tune("rtc_group", 1)
        if diag_build():
            ecx.tune("rtc_persist", 0)
        ecx.tune("rtc_lookahead", 1)
        ecx.tune("rtc_sched", 2)
    ref0 = outs[(0, 0, 0, 0, 1)][0]
    for mode in modes[1:]:
        want = "k_clay_repair_grp" if mode[2] else "k_clay_repair"
        assert outs[mode][1] == want, (mode, outs[mode][1])
        assert (outs[mode][0] == ref0).all(), mode
    host = pool[S - 1].cpu().numpy()
    inputs = [None if (i % n) == e else host[i].copy() for i in range(n * a)]
    if v == 0:
        ref = [np.zeros(B, np.uint8) for _ in range(a)]
        O.Clay(k, m, [e]).perform_coding(inputs, ref, B)
    else:  # shortened: the reference Clay(k+v, m) with the virtual nodes zero-filled
        ref = shortened_clay_oracle(k, m, v, [e], inputs, B)
    for mode in modes:
        bad = [z for z in range(a) if not (outs[mode][0][S - 1, z] == ref[z]).all()]
        assert not bad, (mode, bad[:8])


@pytest.mark.parametrize("e", [0, 3, 9, 10, 13])
def test_clay104_shipped_repair_kernel_vs_shortened_oracle(ecx, torch_dev, e):
    """BASELINE config 4 as shipped: the default launch of a shortened Clay(10,4)
    single-node repair (4 KiB sub-chunks of 1 MiB node blocks) runs the plane-group
    kernel k_clay_repair_grp, and its output on random NON-codeword stripes equals the
    oracle Clay(12,4) (ClayCodeErasureDecodingStep.java:171-203 stage sequence) with the
    two virtual data nodes zero-filled, on every sub-chunk of first, middle and last
    stripe.  e covers a data node of each node row (0, 3, 9), the first parity node (10)
    and the last (13)."""
    torch = torch_dev
    k, m, v, B, S = 10, 4, 2, 4096, 5
    step = ecx.ClayCodeErasureDecodingStep([e], k, m, virtualUnits=v)
    n, a = k + m, step.subPacketSize
    assert a == 256
    pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 1000 + e)
    o = torch.full((S, a, B), 0x5A, dtype=torch.uint8, device="cuda")
    step.performCodingBatch(pool, n * a * B, B, o, a * B, B, S, B)
    torch.cuda.synchronize()
    assert ecx.last_kernel() == "k_clay_repair_grp", ecx.last_kernel()
    got = o.cpu().numpy()
    for s in (0, S // 2, S - 1):
        host = pool[s].cpu().numpy()
        inputs = [None if (i % n) == e else host[i].copy() for i in range(n * a)]
        ref = shortened_clay_oracle(k, m, v, [e], inputs, B)
        bad = [z for z in range(a) if not (got[s, z] == ref[z]).all()]
        assert not bad, (e, s, bad[:8])


def test_clay104_wide_address_kernel_equals_narrow(ecx, torch_dev):
    """The plane-group kernel's 64-bit-address form (forced with ecx_tune "rtc_wide" 1 on the
    4 KiB sub-chunk layout, where the 32-bit form also runs) writes exactly the 32-bit form's
    bytes on random non-codeword stripes, for a data node and a parity node."""
    torch = torch_dev
    k, m, v, B, S = 10, 4, 2, 4096, 6
    n, a = k + m, 256
    pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 77)
    for e in (3, 12):
        step = ecx.ClayCodeErasureDecodingStep([e], k, m, virtualUnits=v)
        outs = []
        for wide in (0, 1):
            ecx.tune("rtc_wide", wide)
            try:
                o = torch.full((S, a, B), 0xA5, dtype=torch.uint8, device="cuda")
                step.performCodingBatch(pool, n * a * B, B, o, a * B, B, S, B)
                torch.cuda.synchronize()
                assert ecx.last_kernel() == "k_clay_repair_grp", ecx.last_kernel()
                outs.append(o)
            finally:
                ecx.tune("rtc_wide", 0)
        assert torch.equal(outs[0], outs[1]), e


def test_clay104_one_mib_sub_chunks(ecx, torch_dev):
    """Config 4's other reading: CLAY_BLOCK_SIZE = 1 MiB sub-chunks (PipelineUtil.kt:13-28,
    ClayCodeErasureDecodingStep.java:72-73), alpha = 256, a 256 MiB node block, a 3.5 GiB
    stripe.  Encode on the GPU, erase node 3 (and 13), repair, compare with the originals
    (the round trip); then repair a random NON-codeword stripe and compare a 64 KiB window
    of every one of the 256 repaired sub-chunks with the oracle Clay(12,4) (zero-filled
    virtual nodes) run on the same window of every input sub-chunk: the map acts bytewise,
    so a window pins it."""
    torch = torch_dev
    k, m, v, B, S, W = 10, 4, 2, 1 << 20, 2, 65536
    n = k + m
    enc = ecx.ClayCodeErasureDecodingStep(list(range(k, n)), k, m, virtualUnits=v)
    a = enc.subPacketSize
    pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 1044)
    par = torch.empty((S, m * a, B), dtype=torch.uint8, device="cuda")
    enc.performCodingBatch(pool, n * a * B, B, par, m * a * B, B, S, B)
    pool.view(S, a, n, B)[:, :, k:, :] = par.view(S, a, m, B)
    del par
    out = torch.empty((S, a, B), dtype=torch.uint8, device="cuda")
    for e in (3, 13):
        out.fill_(0x5A)
        ecx.ClayCodeErasureDecodingStep([e], k, m, virtualUnits=v).performCodingBatch(
            pool, n * a * B, B, out, a * B, B, S, B)
        torch.cuda.synchronize()
        assert torch.equal(out, pool.view(S, a, n, B)[:, :, e, :]), e
    # a non-codeword stripe: the exact linear map, window by window
    e = 3
    ecx.fill_random(pool, pool[0].numel(), 1045)
    step = ecx.ClayCodeErasureDecodingStep([e], k, m, virtualUnits=v)
    step.performCodingBatch(pool, n * a * B, B, out, a * B, B, 1, B)
    torch.cuda.synchronize()
    assert ecx.last_kernel() == "k_clay_repair_grp", ecx.last_kernel()
    for w0 in (0, B - W):
        host = pool[0, :, w0:w0 + W].cpu().numpy()
        got = out[0, :, w0:w0 + W].cpu().numpy()
        inputs = [None if (i % n) == e else host[i].copy() for i in range(n * a)]
        ref = shortened_clay_oracle(k, m, v, [e], inputs, W)
        bad = [z for z in range(a) if not (got[z] == ref[z]).all()]
        assert not bad, (w0, bad[:8])


def test_clay_rtc_first_use_from_two_streams(ecx, torch_dev):
    """The per-helper-plane kernel's program table is uploaded synchronously before the
    loaded module is published (ClayRtc::prepare), so a second thread that launches the
    kernel on another stream right after first use never reads a table still queued
    behind the first caller's stream.  Two threads, two streams, one fresh shortened
    Clay(9,4) step (Clay(12,4) with 3 virtual nodes, rtc_group 0): the first thread's
    stream is kept busy with a large fill when it reaches the kernel; both repairs equal
    the composed-map kernel and the oracle."""
    import threading
    torch = torch_dev
    k, m, v, e, B, S = 9, 4, 3, 2, 4096, 8
    step = ecx.ClayCodeErasureDecodingStep([e], k, m, virtualUnits=v)
    n, a = k + m, step.subPacketSize
    pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 77)
    busy = torch.empty(2 << 30, dtype=torch.uint8, device="cuda")
    outs = [torch.full((S, a, B), 0x77, dtype=torch.uint8, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    barrier, errors = threading.Barrier(2), []

    def worker(i):
        try:
            st = streams[i]
            mine = ecx.ClayCodeErasureDecodingStep([e], k, m, virtualUnits=v)  # the same shared codec
            if i == 0:
                for _ in range(4):
                    ecx.fill_random(busy, busy.numel(), 3, stream=st)
            barrier.wait()
            mine.performCodingBatch(pool, n * a * B, B, outs[i], a * B, B, S, B, stream=st)
            st.synchronize()
        except Exception as err:  # pragma: no cover - reported below
            errors.append(err)

    ecx.tune("clay_rtc", 2)
    ecx.tune("rtc_group", 0)
    try:
        th = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors, errors
        ecx.tune("clay_rtc", 0)
        ref0 = torch.zeros((S, a, B), dtype=torch.uint8, device="cuda")
        step.performCodingBatch(pool, n * a * B, B, ref0, a * B, B, S, B)
        torch.cuda.synchronize()
    finally:
        ecx.tune("clay_rtc", 1)
        ecx.tune("rtc_group", 1)
    assert bool(torch.equal(outs[0], ref0)) and bool(torch.equal(outs[1], ref0))
    host = pool[S - 1].cpu().numpy()
    inputs = [None if (i % n) == e else host[i].copy() for i in range(n * a)]
    ref = shortened_clay_oracle(k, m, v, [e], inputs, B)
    got = ref0[S - 1].cpu().numpy()
    assert all((got[z] == ref[z]).all() for z in range(a))


_NO_HIPRTC_SCRIPT = r"""
import sys
import numpy as np
import torch
import rpamd
sys.path.insert(0, sys.argv[1])
import oracle as O
from conftest import shortened_clay_oracle
ecx = rpamd.load()
# Clay(10,4) single repair: auto (clay_rtc 1) would run k_clay_repair_grp
k, m, v, e, B, S = 10, 4, 2, 3, 4096, 2
step = ecx.ClayCodeErasureDecodingStep([e], k, m, virtualUnits=v)
n, a = k + m, step.subPacketSize
pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
ecx.fill_random(pool, pool.numel(), 5)
o = torch.zeros((S, a, B), dtype=torch.uint8, device="cuda")
step.performCodingBatch(pool, n * a * B, B, o, a * B, B, S, B)
torch.cuda.synchronize()
kern = ecx.last_kernel()
assert not kern.startswith("k_clay_repair"), kern
host = pool[S - 1].cpu().numpy()
inputs = [None if (i % n) == e else host[i].copy() for i in range(n * a)]
ref = shortened_clay_oracle(k, m, v, [e], inputs, B)
got = o[S - 1].cpu().numpy()
assert all((got[z] == ref[z]).all() for z in range(a))
ecx.tune("clay_rtc", 2)
try:
    step.performCodingBatch(pool, n * a * B, B, o, a * B, B, S, B)
    raise SystemExit("forced clay_rtc without hiprtc did not fail")
except ecx.EcxError as err:
    assert err.code == -10, err
ecx.tune("clay_rtc", 1)
# Clay(4,2) repair of {0, 3}: auto (map_planes 1) would run k_map_planes on >= 64 MiB
B2, S2 = 32768, 64
step2 = ecx.ClayCodeErasureDecodingStep([0, 3], 4, 2)
pool2 = torch.empty((S2, 48, B2), dtype=torch.uint8, device="cuda")
ecx.fill_random(pool2, pool2.numel(), 6)
o2 = torch.zeros((S2, 16, B2), dtype=torch.uint8, device="cuda")
step2.performCodingBatch(pool2, 48 * B2, B2, o2, 16 * B2, B2, S2, B2)
torch.cuda.synchronize()
kern2 = ecx.last_kernel()
assert kern2 != "k_map_planes", kern2
h2 = pool2[S2 - 1].cpu().numpy()
ins2 = [None if (i % 6) in (0, 3) else h2[i].copy() for i in range(48)]
ref2 = [np.zeros(B2, np.uint8) for _ in range(16)]
O.Clay(4, 2, [0, 3]).perform_coding(ins2, ref2, B2)
g2 = o2[S2 - 1].cpu().numpy()
assert all((g2[z] == ref2[z]).all() for z in range(16))
print("fallback ok", kern, kern2)
"""


def test_generated_kernels_fall_back_without_hiprtc(tmp_path):
    """No usable libhiprtc: the auto Clay(10,4) repair and the auto Clay(4,2) two-node
    repair run the composed-map kernels instead of the generated ones, with oracle-exact
    results; forcing the generated kernel (clay_rtc 2) fails loudly with ECX_E_DEVICE.
    A child process, because hiprtc is bound once per process."""
    import os
    import subprocess
    import sys
    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, ECX_HIPRTC_LIB=str(tmp_path / "no-libhiprtc.so"),
               PYTHONPATH=os.pathsep.join([str(root), str(root / "oracle")]))
    r = subprocess.run([sys.executable, "-c", _NO_HIPRTC_SCRIPT, str(root / "tests")], capture_output=True,
                       text=True, env=env, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "fallback ok" in r.stdout


def test_clay_rtc_kernel_far_stripes(ecx, torch_dev):
    """Stripe bases beyond 2 and 4 GiB from the allocation start (a 2.25 GiB stripe
    pitch): the generated kernel's 64-bit stripe addressing (a sign-extended low half
    would corrupt the buffer descriptor) matches the composed-map kernel on every stripe."""
    torch = torch_dev
    k, m, v, e, B = 10, 4, 2, 3, 4096
    step = ecx.ClayCodeErasureDecodingStep([e], k, m, virtualUnits=v)
    n, a = k + m, step.subPacketSize
    pitch, S = (9 << 28) + 4096, 3
    used = n * a * B
    buf = torch.empty((S - 1) * pitch + used, dtype=torch.uint8, device="cuda")
    for s in range(S):
        ecx.fill_random(buf[s * pitch:s * pitch + used], used, 90 + s)
    outs = []
    try:
        for rtc, grp in ((0, 0), (2, 0), (2, 1)):
            ecx.tune("clay_rtc", rtc)
            ecx.tune("rtc_group", grp)
            o = torch.full((S, a, B), 0x33, dtype=torch.uint8, device="cuda")
            step.performCodingBatch(buf, pitch, B, o, a * B, B, S, B)
            torch.cuda.synchronize()
            outs.append((o.cpu().numpy(), ecx.last_kernel()))
    finally:
        ecx.tune("clay_rtc", 1)
        ecx.tune("rtc_group", 1)
    assert outs[1][1] == "k_clay_repair" and outs[2][1] == "k_clay_repair_grp"
    assert (outs[0][0] == outs[1][0]).all() and (outs[0][0] == outs[2][0]).all()
    del buf
    torch.cuda.empty_cache()


@pytest.mark.parametrize("seed", range(6))
def test_map_planes_random_maps(ecx, torch_dev, seed):
    """The bit-plane kernel generated per map (k_map_planes, map_rtc.cpp; ecx_tune
    "map_planes" 2) on random maps of 1-16 rows over up to 40 scattered input slots
    (coefficient-1 entries, zero rows and unread inputs), ragged byte counts (the tail
    runs on the composed plan), at load lookaheads 0-8 and 1-3 waves per SIMD, and in
    accumulate mode (out ^= M * in): each equals the oracle's table-driven product."""
    from conftest import gf_apply_numpy
    torch = torch_dev
    rng = np.random.default_rng(7000 + seed)
    n_out, n_in = int(rng.integers(1, 17)), int(rng.integers(1, 41))
    m = rng.integers(2, 256, (n_out, n_in)).astype(np.uint8)
    m[rng.random((n_out, n_in)) < 0.2] = 1
    m[rng.random((n_out, n_in)) >= rng.uniform(0.2, 1.0)] = 0
    if n_out > 2 and seed % 2:
        m[1] = 0
    in_slot = sorted(rng.choice(2 * n_in, n_in, replace=False).tolist())
    out_slot = rng.permutation(rng.choice(2 * n_out, n_out, replace=False)).tolist()
    gm = ecx.GfMap.from_matrix(m, in_slot=in_slot, out_slot=out_slot)
    S, L = 3, 4096 * int(rng.integers(1, 4)) + (0 if seed == 0 else int(rng.integers(1, 4096)))
    ni, no = 2 * n_in, 2 * n_out
    inp = torch.empty((S, ni, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(inp, inp.numel(), 70 + seed)
    host = inp.cpu().numpy()
    ref = [gf_apply_numpy(m, [host[s, j] for j in in_slot]) for s in range(S)]
    try:
        ecx.tune("map_planes", 2)
        for la, waves, acc in ((4, 2, False), (0, 2, False), (1, 3, False), (8, 1, False), (4, 2, True)):
            ecx.tune("planes_lookahead", la)
            ecx.tune("planes_waves", waves)
            out = torch.empty((S, no, L), dtype=torch.uint8, device="cuda")
            ecx.fill_random(out, out.numel(), 90 + seed)
            prev = out.cpu().numpy()
            if acc:
                gm.accumulate_batch(inp, ni * L, L, out, no * L, L, S, L)
            else:
                gm.apply_batch(inp, ni * L, L, out, no * L, L, S, L)
            torch.cuda.synchronize()
            assert ecx.last_kernel() == "k_map_planes"
            got = out.cpu().numpy()
            for s in range(S):
                for o, slot in enumerate(out_slot):
                    want = ref[s][o] ^ prev[s, slot] if acc else ref[s][o]
                    assert (got[s, slot] == want).all(), (la, waves, acc, s, o)
            untouched = sorted(set(range(no)) - set(out_slot))
            assert (got[:, untouched] == prev[:, untouched]).all()
    finally:
        ecx.tune("map_planes", 1)
        ecx.tune("planes_lookahead", 12)
        ecx.tune("planes_waves", 2)


@pytest.mark.parametrize("erased", [[0, 3], [4, 5], [1, 2]])
def test_map_planes_auto_clay42_batches(ecx, torch_dev, erased):
    """Clay(4,2) two-node repairs and the encode on a batch big enough for the auto rule
    (64 stripes x 32 KiB sub-chunks): the generated bit-plane kernel runs (ecx_last_kernel),
    and its bytes equal the split-table kernels' (map_planes 0) and, on a sampled
    stripe, the oracle's performCoding."""
    torch = torch_dev
    k, m, B, S = 4, 2, 32768, 64
    n, a = k + m, 8
    step = ecx.ClayCodeErasureDecodingStep(erased, k, m)
    pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 41)
    outs = []
    try:
        for mode in (1, 0):
            ecx.tune("map_planes", mode)
            o = torch.full((S, len(erased) * a, B), 7, dtype=torch.uint8, device="cuda")
            step.performCodingBatch(pool, n * a * B, B, o, len(erased) * a * B, B, S, B)
            torch.cuda.synchronize()
            if mode == 1:
                assert ecx.last_kernel() == "k_map_planes"
            outs.append(o.cpu().numpy())
    finally:
        ecx.tune("map_planes", 1)
    assert (outs[0] == outs[1]).all()
    host = pool[S // 2].cpu().numpy()
    inputs = [None if (i % n) in erased else host[i].copy() for i in range(n * a)]
    ref = [np.zeros(B, np.uint8) for _ in range(len(erased) * a)]
    O.Clay(k, m, erased).perform_coding(inputs, ref, B)
    assert all((outs[0][S // 2, j] == ref[j]).all() for j in range(len(ref)))


def test_map_planes_every_clay42_erasure_pattern(ecx, torch_dev):
    """Every Clay(4,2) single and two-node erasure pattern (6 + 15 maps, performCoding's
    doDecodeSingle / doDecodeMulti compositions) on the generated bit-plane kernel
    (map_planes forced), two 4 KiB chunks plus a ragged tail: bit-exact against the
    oracle's stage-by-stage performCoding on the last stripe and equal to the
    split-table kernels on every stripe."""
    import itertools
    torch = torch_dev
    k, m, B, S = 4, 2, 2 * 4096 + 272, 3
    n, a = k + m, 8
    pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 57)
    host = pool[S - 1].cpu().numpy()
    patterns = [[e] for e in range(n)] + [list(p) for p in itertools.combinations(range(n), 2)]
    try:
        for erased in patterns:
            step = ecx.ClayCodeErasureDecodingStep(erased, k, m)
            got = []
            for mode in (2, 0):
                ecx.tune("map_planes", mode)
                o = torch.full((S, len(erased) * a, B), 0xA5, dtype=torch.uint8, device="cuda")
                step.performCodingBatch(pool, n * a * B, B, o, len(erased) * a * B, B, S, B)
                torch.cuda.synchronize()
                if mode == 2:
                    assert ecx.last_kernel() == "k_map_planes", erased
                got.append(o.cpu().numpy())
            assert (got[0] == got[1]).all(), erased
            inputs = [None if (i % n) in erased else host[i].copy() for i in range(n * a)]
            ref = [np.zeros(B, np.uint8) for _ in range(len(erased) * a)]
            O.Clay(k, m, erased).perform_coding(inputs, ref, B)
            assert all((got[0][S - 1, j] == ref[j]).all() for j in range(len(ref))), erased
    finally:
        ecx.tune("map_planes", 1)


@pytest.mark.parametrize("pitch", [(4 << 20), (1 << 20) + 4096])
def test_layout_select_is_measured_and_exact(ecx, torch_dev, pitch):
    """layout_select (include/ecx_tune.h): the first calls of a large RS(12,4) decode batch at
    a new layout run the candidate launch shapes in turn (static rules, 4 KiB and one-wave
    workgroups, skewed chunks, staggered stripes), each timed with events on the caller's
    stream, and the fastest median is then kept for that layout.  Every call's in-place
    output equals the erased originals (and the oracle on one stripe), in overwrite and in
    accumulate mode; with layout_select 0 nothing is selected."""
    torch = torch_dev
    L = 1 << 20
    S = (320 << 20) // (12 * L) + 1  # >= 256 MiB of input: selection runs
    rs = ecx.ReedSolomon.create(12, 4)
    present = [False, False] + [True] * 14
    pool = torch.empty((S, 16, pitch), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 88)
    rs.encode_map().apply_batch(pool, 16 * pitch, pitch, pool, 16 * pitch, pitch, S, L)
    orig = pool[:, 0:2, :L].clone()
    mat, ins_, outs_ = rs.decode_map(present).matrix()
    fresh = lambda: ecx.GfMap.from_matrix(mat, in_slot=[int(i) for i in ins_],  # noqa: E731
                                          out_slot=[int(o) for o in outs_])    # nothing selected yet
    dmap = fresh()
    kernels = set()
    for call in range(38):  # 7 candidates x 5 timings, harvested on later calls
        assert dmap.layout_choice(pitch) == -1 or call > 35
        pool[:, 0:2, :L] = 0
        dmap.apply_batch(pool, 16 * pitch, pitch, pool, 16 * pitch, pitch, S, L)
        torch.cuda.synchronize()
        kernels.add(ecx.last_kernel())
        assert bool(torch.equal(pool[:, 0:2, :L], orig)), call
    choice, ms = dmap.layout_choice(pitch, with_times=True)
    assert choice != -1, ms
    assert all(t > 0 for t in ms[:7]), ms
    # a batch of another stripe count in the same size class reuses the choice: no exploring
    dmap.apply_batch(pool, 16 * pitch, pitch, pool, 16 * pitch, pitch, S, L)
    torch.cuda.synchronize()
    kept = ecx.last_kernel()
    for _ in range(3):
        pool[:, 0:2, :L] = 0
        dmap.apply_batch(pool, 16 * pitch, pitch, pool, 16 * pitch, pitch, S - 1, L)
        torch.cuda.synchronize()
        assert ecx.last_kernel() == kept
        assert bool(torch.equal(pool[:S - 1, 0:2, :L], orig[:S - 1]))
    assert any(k.startswith("k_gf_apply_skew") for k in kernels) and any(", 64, " in k for k in kernels), kernels
    static_ms = ms[0]
    assert min(ms[:7]) <= static_ms
    # the oracle on one stripe
    host = pool[S - 1].cpu().numpy()
    shards = [np.zeros(L, np.uint8) if i < 2 else host[i, :L].copy() for i in range(16)]
    O.ReedSolomon(12, 4).decode_missing(shards, [i >= 2 for i in range(16)], 0, L)
    assert (shards[0] == orig[S - 1, 0].cpu().numpy()).all() and (shards[1] == orig[S - 1, 1].cpu().numpy()).all()
    # accumulate mode: every candidate XOR-accumulates exactly once per call
    acc_map = fresh()
    acc = torch.zeros((S, 2, pitch), dtype=torch.uint8, device="cuda")
    for _ in range(37):
        acc_map.accumulate_batch(pool, 16 * pitch, pitch, acc, 2 * pitch, pitch, S, L)
        torch.cuda.synchronize()
    assert acc_map.layout_choice(pitch) != -1
    assert bool(torch.equal(acc[:, :, :L], orig))  # 37 accumulations: an odd count leaves M * in
    # off: the static rules only
    off_map = fresh()
    try:
        ecx.tune("layout_select", 0)
        for _ in range(4):
            off_map.apply_batch(pool, 16 * pitch, pitch, pool, 16 * pitch, pitch, S, L)
        torch.cuda.synchronize()
    finally:
        ecx.tune("layout_select", 1)
    assert off_map.layout_choice(pitch) == -1
    assert bool(torch.equal(pool[:, 0:2, :L], orig))


@pytest.mark.parametrize("e,B,S", [(3, 4096, 5), (13, 8192 + 16, 3), (0, 4096, 17)])
def test_clay_grp_two_slice_units_vs_oracle(ecx, torch_dev, e, B, S):
    """rtc_units 2 (two 512-B slices per workgroup, the second slice's rows loaded while the
    first finishes) and rtc_sched 1 (the lean load schedule, 1-4 pairs ahead), in every
    block order and at 2-4 waves per SIMD, equal the default kernel and the zero-filled
    Clay(12,4) oracle (ClayCodeErasureDecodingStep.java:171-203) on a shortened Clay(10,4)."""
    torch = torch_dev
    k, m, v = 10, 4, 2
    step = ecx.ClayCodeErasureDecodingStep([e], k, m, virtualUnits=v)
    n, a = k + m, step.subPacketSize
    pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 300 + e)
    outs = []
    try:
        for units, xcd, waves, sched, la in [(1, 2, 3, 2, 1), (1, 2, 3, 0, 1), (2, 2, 3, 0, 1), (2, 1, 3, 0, 1),
                                             (2, 3, 2, 0, 1), (2, 4, 3, 0, 1), (2, 0, 2, 0, 1), (1, 2, 4, 1, 1),
                                             (1, 2, 3, 1, 0), (1, 3, 4, 1, 3), (2, 2, 3, 1, 2), (1, 2, 4, 2, 0),
                                             (2, 2, 2, 2, 1)]:
            if units == 2 and not diag_build():
                continue  # two-slice units: diagnostic library only (make DIAG=1)
            if diag_build():
                ecx.tune("rtc_units", units)
            ecx.tune("rtc_xcd", xcd)
            ecx.tune("rtc_waves", waves)
            ecx.tune("rtc_sched", sched)
            ecx.tune("rtc_lookahead", la)
            o = torch.full((S, a, B), 0x6B, dtype=torch.uint8, device="cuda")
            step.performCodingBatch(pool, n * a * B, B, o, a * B, B, S, B)
            torch.cuda.synchronize()
            assert ecx.last_kernel() == "k_clay_repair_grp"
            outs.append(o.cpu().numpy())
    finally:
        if diag_build():
            ecx.tune("rtc_units", 1)
        ecx.tune("rtc_xcd", 2)
        ecx.tune("rtc_waves", 3)
        ecx.tune("rtc_sched", 2)
        ecx.tune("rtc_lookahead", 1)
    assert all((x == outs[0]).all() for x in outs[1:])
    host = pool[S - 1].cpu().numpy()
    inputs = [None if (i % n) == e else host[i].copy() for i in range(n * a)]
    ref = shortened_clay_oracle(k, m, v, [e], inputs, B)
    assert all((outs[0][S - 1, z] == ref[z]).all() for z in range(a))


@pytest.mark.parametrize("e,B,S", [(3, 4096, 5), (11, 4096 + 48, 3)])
def test_clay_rtc_nontemporal_policies_vs_oracle(ecx, torch_dev, e, B, S):
    """Every non-temporal load policy (ecx_tune rtc_nt: cached, the read-once rows, the
    row-yc own / partner loads, the default 5, all; bit 8 the per-plane kernel's loads)
    gives the same repair on both generated Clay kernels, equal to the zero-filled
    Clay(12,4) oracle (ClayCodeErasureDecodingStep.java:171-203) on a shortened Clay(10,4)."""
    torch = torch_dev
    k, m, v = 10, 4, 2
    step = ecx.ClayCodeErasureDecodingStep([e], k, m, virtualUnits=v)
    n, a = k + m, step.subPacketSize
    pool = torch.empty((S, n * a, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 500 + e)
    outs = []
    try:
        for grp, nt in [(1, 5), (1, 0), (1, 1), (1, 2), (1, 3), (1, 4), (1, 7), (1, 15), (0, 0), (0, 8), (0, 5)]:
            ecx.tune("rtc_group", grp)
            ecx.tune("rtc_nt", nt)
            o = torch.full((S, a, B), 0x3C, dtype=torch.uint8, device="cuda")
            step.performCodingBatch(pool, n * a * B, B, o, a * B, B, S, B)
            torch.cuda.synchronize()
            assert ecx.last_kernel() == ("k_clay_repair_grp" if grp else "k_clay_repair")
            outs.append(o.cpu().numpy())
    finally:
        ecx.tune("rtc_group", 1)
        ecx.tune("rtc_nt", 5)
    assert all((x == outs[0]).all() for x in outs[1:])
    host = pool[S - 1].cpu().numpy()
    inputs = [None if (i % n) == e else host[i].copy() for i in range(n * a)]
    ref = shortened_clay_oracle(k, m, v, [e], inputs, B)
    assert all((outs[0][S - 1, z] == ref[z]).all() for z in range(a))


def test_layout_selection_serialized_streams_drop_nothing(ecx, torch_dev):
    """Round-5 advice: callers on their own streams whose calls never overlap (JVM threads
    serialised by @Synchronized, ClayCodeNode.kt:76-347) must not lose their timing probes.
    Two streams take turns on one batch layout, each call finished before the next starts: a
    launch of the other stream that finds a probe already done does not drop it, so the
    selection concludes with nothing dropped, and every call's output is the oracle's parity."""
    torch = torch_dev
    k, m, L, S = 12, 4, 1 << 20, 24
    rs = ecx.ReedSolomon.create(k, m)
    emap = rs.encode_map()
    pool = torch.empty((S, 16, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 310)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for i in range(80):
        st = streams[i % 2]
        emap.apply_batch(pool, 16 * L, L, pool, 16 * L, L, S, L, stream=st)
        st.synchronize()
    state, dropped = emap.layout_state(L)
    assert emap.layout_choice(L) != -1 and state in (1, 2, 3) and dropped == 0, (state, dropped)
    host = pool[S - 1].cpu().numpy()
    ref = [host[i].copy() for i in range(16)]
    for i in range(k, 16):
        ref[i][:] = 0
    O.ReedSolomon(k, m).encode_parity(ref, 0, L)
    assert all((host[i] == ref[i]).all() for i in range(k, 16))


def test_layout_selection_two_streams(ecx, torch_dev):
    """Round-4 verdict item 3: two threads, each on its own stream, drive one batch layout of
    one map at once (RS(12,4) encode in place, 4 MiB shards, 1.5 GiB per batch -- eligible for
    the per-layout selection, and long enough (~0.25 ms) that the two threads' kernels really
    overlap despite the Python overhead between calls).  Every launch computes the same bytes
    whatever candidate it runs, so both pools end with the oracle's parity; the selection still
    concludes (a kept shape, or the static rules once the probes kept overlapping the other
    stream's launches: state 4, "contended"), and no timing that overlapped the other stream
    was used."""
    import threading
    torch = torch_dev
    k, m, L, S = 12, 4, 4 << 20, 24
    rs = ecx.ReedSolomon.create(k, m)
    emap = rs.encode_map()
    pools = [torch.empty((S, 16, L), dtype=torch.uint8, device="cuda") for _ in range(2)]
    for i, p in enumerate(pools):
        ecx.fill_random(p, p.numel(), 300 + i)
    torch.cuda.synchronize()
    errors = []

    def drive(i):
        try:
            st = torch.cuda.Stream()
            for _ in range(120):  # each caller waits for its launch, as a synchronous caller does:
                emap.apply_batch(pools[i], 16 * L, L, pools[i], 16 * L, L, S, L, stream=st)
                st.synchronize()  # finished probes are harvested on the next call
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(e)

    th = [threading.Thread(target=drive, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    assert not errors, errors
    choice = emap.layout_choice(L)
    state, dropped = emap.layout_state(L)
    assert choice != -1 and state in (1, 3, 4), (choice, state, dropped)
    assert dropped > 0  # the two streams' launches overlapped: those probes were not used
    for p in pools:
        for s in (0, S - 1):
            host = p[s].cpu().numpy()
            ref = [host[i].copy() for i in range(16)]
            for i in range(k, 16):
                ref[i][:] = 0
            O.ReedSolomon(k, m).encode_parity(ref, 0, L)
            assert all((ref[i] == host[i]).all() for i in range(k, 16)), s


@pytest.mark.diag
@pytest.mark.parametrize("units", [2, 4])
def test_multi_unit_workgroups_match(ecx, torch_dev, units):
    """k_gf_apply_multi (ecx_tune "units": several (stripe, chunk) units per workgroup, one load
    ring across them) writes the same bytes as k_gf_apply on every single-tile shape it serves --
    the 20-deep headline ring (Clay(4,2) repair), the RS(17,3) encode with its fused partial last
    chunk, one-wave RS(12,4) decode, accumulate mode -- with stripe counts that leave the last
    workgroup short, and the oracle agrees on a sampled stripe."""
    import oracle as O
    torch = torch_dev

    def run(fn, out):
        ecx.tune("units", 1)
        ecx.tune("layout_select", 0)
        try:
            ref = out.clone()
            fn(ref)
            ecx.tune("units", units)
            got = out.clone()
            fn(got)
            torch.cuda.synchronize()
            return ref, got, ecx.last_kernel()
        finally:
            ecx.tune("units", 1)
            ecx.tune("layout_select", 1)

    # Clay(4,2) repair, 32 KiB, 7 stripes (odd)
    S, B = 7, 32768
    pool = torch.empty((S, 48, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 71)
    step = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
    out = torch.zeros((S, 8, B), dtype=torch.uint8, device="cuda")
    ref, got, kern = run(lambda o: step.performCodingBatch(pool, 48 * B, B, o, 8 * B, B, S, B), out)
    assert kern.startswith("k_gf_apply_multi<20"), kern
    assert torch.equal(ref, got)
    host = pool[S - 1].cpu().numpy()
    oref = [np.zeros(B, np.uint8) for _ in range(8)]
    O.Clay(4, 2, [1]).perform_coding([None if i % 6 == 1 else host[i].copy() for i in range(48)], oref, B)
    assert all((got[S - 1, z].cpu().numpy() == oref[z]).all() for z in range(8))
    # RS(17,3) encode in place on the published shape (fused partial chunk), 5 stripes
    S, L = 5, 200000
    rpool = torch.empty((S, 20, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(rpool, rpool.numel(), 72)
    rs = ecx.ReedSolomon.create(17, 3)
    ref, got, kern = run(lambda p: rs.encodeParityBatch(p, 20 * L, L, S, 0, L), rpool)
    assert kern.startswith("k_gf_apply_multi<8") and kern.endswith("true>"), kern
    assert torch.equal(ref, got)
    h = got[2].cpu().numpy()
    sh = [h[i].copy() for i in range(20)]
    for i in range(17, 20):
        sh[i][:] = 0
    O.ReedSolomon(17, 3).encode_parity(sh, 0, L)
    assert all((sh[i] == h[i]).all() for i in range(17, 20))
    # RS(12,4) decode {0, 1} into a separate buffer, one-wave workgroups forced; accumulate mode
    S, L = 3, 1 << 20
    dpool = torch.empty((S, 16, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(dpool, dpool.numel(), 73)
    dmap = ecx.ReedSolomon.create(12, 4).decode_map([False, False] + [True] * 14)
    acc0 = torch.empty((S, 2, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(acc0, acc0.numel(), 74)
    ecx.tune("block_threads", 64)
    try:
        ref, got, kern = run(lambda o: dmap.apply_batch(dpool, 16 * L, L, o, 2 * L, L, S, L), acc0)
        assert ", 64, " in kern and kern.startswith("k_gf_apply_multi"), kern
        assert torch.equal(ref, got)
        ref, got, kern = run(lambda o: dmap.accumulate_batch(dpool, 16 * L, L, o, 2 * L, L, S, L), acc0)
        assert torch.equal(ref, got) and not torch.equal(got, acc0)
    finally:
        ecx.tune("block_threads", 0)


def test_layout_selection_revalidates_once(ecx, torch_dev):
    """A layout's kept shape is re-validated once, after 512 further launches (kLayoutRevalidate):
    the state goes exploring -> chosen -> re-validated (3) with nothing dropped on one stream, the
    choice is still a candidate, and every launch wrote the oracle's bytes."""
    import oracle as O
    torch = torch_dev
    k, m, L, S = 12, 4, 1 << 20, 24  # 288 MiB of input per launch: selected per layout
    rs = ecx.ReedSolomon.create(k, m)
    pool = torch.empty((S, 16, L), dtype=torch.uint8, device="cuda")
    ecx.fill_random(pool, pool.numel(), 401)
    rs.encode_map().apply_batch(pool, 16 * L, L, pool, 16 * L, L, S, L)
    dmap = rs.decode_map([True] * 5 + [False] + [True] * 10)
    out = torch.empty((S, 16, L), dtype=torch.uint8, device="cuda")  # the map writes output slot 5
    states = set()
    for i in range(640):
        dmap.apply_batch(pool, 16 * L, L, out, 16 * L, L, S, L)
        torch.cuda.synchronize()
        if i % 16 == 0:
            states.add(dmap.layout_state(L)[0])
    state, dropped = dmap.layout_state(L)
    assert state == 3 and dropped == 0, (state, dropped, states)
    assert 1 in states or 2 in states, states
    assert dmap.layout_choice(L) != -1
    assert torch.equal(out[:, 5], pool[:, 5])
    host = pool[S - 1].cpu().numpy()
    shards = [host[i].copy() if i != 5 else np.zeros(L, np.uint8) for i in range(16)]
    O.ReedSolomon(k, m).decode_missing(shards, [i != 5 for i in range(16)], 0, L)
    assert (shards[5] == out[S - 1, 5].cpu().numpy()).all()


@pytest.mark.host_exec
def test_every_entry_kind_at_once(ecx, torch_dev):
    """Every kind of entry point from its own host thread at the same time, as one JVM's pub/sub
    threads would drive them: per-call calls on both sides of the host-executor threshold
    (2,174-B and 4 KiB calls on the calling thread, 32 KiB calls on the device), device batches on
    their own streams (RS(17,3) encodeParity then isParityCorrect on the published shape, LRC
    encode), and a host-memory Clay(4,2) batch split over the device list [0, 0].  Each thread
    checks its own results (the oracle's, or the verdicts the encode implies) on every iteration."""
    import threading
    torch = torch_dev
    ecx.tune("host_exec_kib", 8)
    rng = np.random.default_rng(2024)
    errors = []

    # per-call RS(4,2): 2,174 B and 4 KiB on the host executor, 32 KiB on the device
    rs_cases = {}
    for L in (2174, 4096, 32768):
        base = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(6)]
        ref = [b.copy() for b in base]
        O.ReedSolomon(4, 2).encode_parity(ref, 0, L)
        rs_cases[L] = (base, ref)
    # per-call Clay(4,2) repair of node 1, 4 KiB sub-chunks (host executor) and 32 KiB (device)
    clay_cases = {}
    for B in (4096, 32768):
        inputs = [None if i % 6 == 1 else rng.integers(0, 256, B, dtype=np.uint8) for i in range(48)]
        ref = [np.zeros(B, np.uint8) for _ in range(8)]
        O.Clay(4, 2, [1]).perform_coding(inputs, ref, B)
        clay_cases[B] = (inputs, ref)
    # host-memory Clay(4,2) batch, 37 stripes of 8 KiB sub-chunks, split over [0, 0]
    S_h, B_h = 37, 8192
    hin = rng.integers(0, 256, (S_h, 48, B_h), dtype=np.uint8)
    step_h = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
    href = np.zeros((S_h, 8, B_h), np.uint8)
    step_h.performCodingBatchHost(hin, 48 * B_h, B_h, href, 8 * B_h, B_h, S_h, B_h)  # one device, before the threads
    for s in (0, S_h - 1):
        o = [np.zeros(B_h, np.uint8) for _ in range(8)]
        O.Clay(4, 2, [1]).perform_coding([None if i % 6 == 1 else hin[s, i].copy() for i in range(48)], o, B_h)
        assert all((href[s, z] == o[z]).all() for z in range(8))

    def guarded(fn):
        def run():
            try:
                fn()
            except Exception as exc:  # noqa: BLE001 -- reported below
                errors.append((fn.__name__, repr(exc)))
        return run

    def per_call_rs():
        rs = ecx.ReedSolomon.create(4, 2)
        for it in range(24):
            L = (2174, 4096, 32768)[it % 3]
            base, ref = rs_cases[L]
            sh = [b.copy() for b in base]
            rs.encodeParity(sh, 0, L)
            if not all((sh[i] == ref[i]).all() for i in range(6)):
                errors.append(("rs encode", it, L))
            present = [True] * 6
            present[it % 4] = False
            sh[it % 4][:] = 0
            rs.decodeMissing(sh, present, 0, L)
            if not (sh[it % 4] == ref[it % 4]).all():
                errors.append(("rs decode", it, L))

    def per_call_clay():
        step = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
        for it in range(16):
            B = (4096, 32768)[it % 2]
            inputs, ref = clay_cases[B]
            got = [np.zeros(B, np.uint8) for _ in range(8)]
            step.performCoding(inputs, got, B)
            if not all((got[z] == ref[z]).all() for z in range(8)):
                errors.append(("clay", it, B))

    def rs173_batches():
        S, L = 96, 200000
        st = torch.cuda.Stream()
        rs = ecx.ReedSolomon.create(17, 3)
        with torch.cuda.stream(st):
            pool = torch.empty((S, 20, L), dtype=torch.uint8, device="cuda")
            verdict = torch.empty(S, dtype=torch.uint8, device="cuda")
        ecx.fill_random(pool, pool.numel(), 77, stream=st)
        for it in range(12):
            rs.encodeParityBatch(pool, 20 * L, L, S, 0, L, stream=st)
            rs.isParityCorrectBatch(pool, 20 * L, L, S, 0, L, verdict, stream=st)
            st.synchronize()
            if int(verdict.sum()) != S:
                errors.append(("rs173 verdict after encode", it, int(verdict.sum())))
            s = it % S
            with torch.cuda.stream(st):
                pool[s, it % 20, (it * 7919) % L] ^= 0x5A  # one flipped byte: exactly that stripe fails
            rs.isParityCorrectBatch(pool, 20 * L, L, S, 0, L, verdict, stream=st)
            st.synchronize()
            bad = torch.nonzero(verdict == 0).flatten().tolist()
            if bad != [s]:
                errors.append(("rs173 flipped", it, bad[:4]))
        h = pool[S - 1].cpu().numpy()
        sh = [h[i].copy() for i in range(20)]
        for i in range(17, 20):
            sh[i][:] = 0
        O.ReedSolomon(17, 3).encode_parity(sh, 0, L)
        if not all((sh[i] == h[i]).all() for i in range(17, 20)):
            errors.append(("rs173 oracle",))

    def lrc_batches():
        S, B = 64, 65536
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            pool = torch.empty((S, 16, B), dtype=torch.uint8, device="cuda")
        ecx.fill_random(pool, pool.numel(), 78, stream=st)
        for it in range(12):
            ecx.LRCErasureCode.encodeBatch(pool, 16 * B, B, S, B, stream=st)
        st.synchronize()
        h = pool[S // 2].cpu().numpy()
        for g in range(4):  # group g: blocks 4g..4g+2 and their XOR parity 4g+3
            want = h[4 * g] ^ h[4 * g + 1] ^ h[4 * g + 2]
            if not (h[4 * g + 3] == want).all():
                errors.append(("lrc group", g))

    def host_devices():
        step = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
        for it in range(6):
            out = np.zeros((S_h, 8, B_h), np.uint8)
            step.performCodingBatchHostDevices(hin, 48 * B_h, B_h, out, 8 * B_h, B_h, S_h, B_h, [0, 0])
            if not (out == href).all():
                errors.append(("host devices", it))

    threads = [threading.Thread(target=guarded(f))
               for f in (per_call_rs, per_call_rs, per_call_clay, rs173_batches, lrc_batches, host_devices)]
    try:
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=100)
    finally:
        ecx.tune("host_exec_kib", 0)
    assert not any(t.is_alive() for t in threads), "a worker thread hung"
    assert not errors, errors[:6]


@pytest.mark.parametrize("small", [False, True])
def test_host_batch_folded_runs_match_device_batch(ecx, torch_dev, small):
    """Host batches whose used slots repeat with a fixed step (host_pipe.cpp fold_runs: one strided
    copy of count x stripes rows per run of the first period) -- shortened Clay(10,4) single-node
    repairs of nodes in each of the four y-groups (periods of 2 to 8 runs a plane group), the
    Clay(4,2) two-node repair {0, 3} and a Clay(4,2) repair on a padded sub-chunk pitch -- write
    exactly what the device batch writes on the same stripes, with default chunks and with one
    stripe per chunk, and leave the output pitch's padding alone."""
    torch = torch_dev
    cases = [(10, 4, 2, [e], 512, 0) for e in (0, 3, 5, 9, 12)] + [(4, 2, 0, [0, 3], 1024, 0), (4, 2, 0, [1], 1000, 24)]
    if small:
        ecx.tune("host_chunk_kib", 16)
    try:
        for k, m, v, er, B, pad in cases:
            n = k + m
            step = ecx.ClayCodeErasureDecodingStep(er, k, m, virtualUnits=v)
            a = step.map().info()["n_out"] // len(er)
            S, P = 5, B + pad
            src = torch.empty((S, n * a, P), dtype=torch.uint8, device="cuda")
            ecx.fill_random(src, src.numel(), 300 + B + len(er) + er[0])
            dev_out = torch.zeros((S, len(er) * a, P), dtype=torch.uint8, device="cuda")
            step.performCodingBatch(src, n * a * P, P, dev_out, len(er) * a * P, P, S, B)
            torch.cuda.synchronize()
            host_in = src.cpu().numpy()
            host_out = np.full((S, len(er) * a, P), 0x3C, np.uint8)
            step.performCodingBatchHost(host_in, n * a * P, P, host_out, len(er) * a * P, P, S, B)
            want = dev_out.cpu().numpy()
            assert (host_out[:, :, :B] == want[:, :, :B]).all(), (k, m, er, B, pad)
            assert (host_out[:, :, B:] == 0x3C).all(), (k, m, er, B, pad)
    finally:
        ecx.tune("host_chunk_kib", 65536)


def test_host_batch_column_slices_match_device_batch(ecx, torch_dev):
    """A one-stripe host batch far larger than a chunk is pipelined in column slices (host_pipe.cpp:
    bytes [c0, c0 + slice) of every slot per unit, 3D copies per progression of runs): with 16 KiB
    chunks that happens at small sizes, so a Clay(4,2) repair with a ragged last slice, a shortened
    Clay(10,4) repair of node 3 (runs in 3D) and an in-place RS(12,4) decode on a padded pitch (one
    slot per run, the output slots between inputs) equal the device batch, with nothing outside the
    written slots' bytes touched."""
    torch = torch_dev
    ecx.tune("host_chunk_kib", 16)
    try:
        for k, m, v, er, B in [(4, 2, 0, [1], 3 * 4096 + 100), (10, 4, 2, [3], 2 * 4096 + 24)]:
            step = ecx.ClayCodeErasureDecodingStep(er, k, m, virtualUnits=v)
            a = step.map().info()["n_out"] // len(er)
            n = k + m
            assert step.map().host_plan(n * a * B, B, a * B, B, 1, B)["slices"] > 1
            src = torch.empty((1, n * a, B), dtype=torch.uint8, device="cuda")
            ecx.fill_random(src, src.numel(), 77 + B)
            dev_out = torch.empty((1, a, B), dtype=torch.uint8, device="cuda")
            step.performCodingBatch(src, n * a * B, B, dev_out, a * B, B, 1, B)
            torch.cuda.synchronize()
            host_out = np.full((1, a, B), 0x3C, np.uint8)
            step.performCodingBatchHost(src.cpu().numpy(), n * a * B, B, host_out, a * B, B, 1, B)
            assert (host_out == dev_out.cpu().numpy()).all(), (k, m, er, B)
        rs = ecx.ReedSolomon.create(12, 4)
        L, P = 5 * 4096 + 7, 5 * 4096 + 64
        present = [False, True, True, False] + [True] * 12
        dmap = rs.decode_map(present)
        assert dmap.host_plan(16 * P, P, 16 * P, P, 1, L)["slices"] > 1
        rng = np.random.default_rng(12)
        host = rng.integers(0, 256, (1, 16, P), dtype=np.uint8)
        dev = torch.from_numpy(host.copy()).cuda()
        dmap.apply_batch(dev, 16 * P, P, dev, 16 * P, P, 1, L)
        torch.cuda.synchronize()
        dmap.apply_batch_host(host, 16 * P, P, host, 16 * P, P, 1, L)
        assert (host == dev.cpu().numpy()).all()
    finally:
        ecx.tune("host_chunk_kib", 65536)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_host_batch_devices_split_columns_of_few_stripes(ecx, torch_dev, devices):
    """Fewer stripes than device entries: ecx_*_batch_host_devices splits the bytes of every slot
    (4 KiB units) over the entries instead of the stripes -- one Clay(4,2) stripe with a ragged byte
    count, and two in-place RS(12,4) stripes on a padded pitch -- and writes what the device batch
    writes, nothing else; the check ANDs the entries' verdicts, so a corrupted byte in any range
    fails its stripe."""
    torch = torch_dev
    B = 5 * 4096 + 100
    step = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
    src = torch.empty((1, 48, B), dtype=torch.uint8, device="cuda")
    ecx.fill_random(src, src.numel(), 5150)
    dev_out = torch.empty((1, 8, B), dtype=torch.uint8, device="cuda")
    step.performCodingBatch(src, 48 * B, B, dev_out, 8 * B, B, 1, B)
    torch.cuda.synchronize()
    host_out = np.full((1, 8, B), 0x3C, np.uint8)
    step.performCodingBatchHostDevices(src.cpu().numpy(), 48 * B, B, host_out, 8 * B, B, 1, B, devices)
    assert (host_out == dev_out.cpu().numpy()).all()
    rs = ecx.ReedSolomon.create(12, 4)
    L, P, S = 3 * 4096 + 5, 3 * 4096 + 48, 2
    dmap = rs.decode_map([False] + [True] * 14 + [False])
    host = np.random.default_rng(3).integers(0, 256, (S, 16, P), dtype=np.uint8)
    dev = torch.from_numpy(host.copy()).cuda()
    dmap.apply_batch(dev, 16 * P, P, dev, 16 * P, P, S, L)
    torch.cuda.synchronize()
    dmap.apply_batch_host_devices(host, 16 * P, P, host, 16 * P, P, S, L, devices + [0])
    assert (host == dev.cpu().numpy()).all()
    # the check: one corrupted byte in the last 4 KiB of stripe 1 fails it whichever entry checks it
    shards = host.copy()
    rs.encode_map().apply_batch_host(shards, 16 * P, P, shards, 16 * P, P, S, L)
    shards[1, 7, L - 3] ^= 0x5A
    verdict = np.full(S, 9, np.uint8)
    rs.isParityCorrectBatchHostDevices(shards, 16 * P, P, S, 0, L, verdict, devices + [0])
    assert verdict.tolist() == [1, 0]


def test_host_batch_random_layouts_match_device_batch(ecx, torch_dev):
    """apply_batch_host over 60 random layouts against apply_batch on the device, same bytes: random
    maps (1-24 inputs, 1-6 outputs, slot sets with gaps, repeats of a period or none), slot pitches
    equal to or above the byte count, stripe strides with slack, ragged byte counts, 1-9 stripes,
    and host_chunk_kib 16 / 64 / 65536 -- so every copy plan of host_pipe.cpp runs: merged runs,
    folded 2D periods, 3D progressions, lone runs, many chunks and column slices.  Outputs go to a
    separate buffer pre-filled with a marker that must survive outside the written slots."""
    torch = torch_dev
    rng = np.random.default_rng(20261019)
    try:
        for case in range(60):
            n_slots = int(rng.integers(2, 40))
            n_in = int(rng.integers(1, min(24, n_slots) + 1))
            if rng.random() < 0.4:  # a periodic slot set: every `step`-th group of `g` slots
                g = int(rng.integers(1, 4))
                step = g + int(rng.integers(1, 4))
                ins = [b + j for b in range(0, n_slots, step) for j in range(g) if b + j < n_slots][:n_in]
            else:
                ins = sorted(rng.choice(n_slots, n_in, replace=False).tolist())
            n_in = len(ins)
            n_out_slots = int(rng.integers(1, 12))
            n_out = int(rng.integers(1, min(6, n_out_slots) + 1))
            outs = sorted(rng.choice(n_out_slots, n_out, replace=False).tolist())
            M = rng.integers(0, 256, (n_out, n_in), dtype=np.uint8)
            gm = ecx.GfMap.from_matrix(M, ins, outs)
            L = int(rng.choice([1, 100, 4096, 5000, 12288, 20000]))
            pitch = L + int(rng.choice([0, 0, 16, 4096]))
            S = 1 if rng.random() < 0.3 else int(rng.integers(2, 10))  # one stripe: column slices
            in_ss = n_slots * pitch + int(rng.choice([0, 0, 64]))
            out_pitch = L + int(rng.choice([0, 32]))
            out_ss = n_out_slots * out_pitch + int(rng.choice([0, 128]))
            ecx.tune("host_chunk_kib", int(rng.choice([16, 64, 65536])))
            host_in = rng.integers(0, 256, S * in_ss, dtype=np.uint8)
            host_out = np.full(S * out_ss, 0xA5, np.uint8)
            dev_in = torch.from_numpy(host_in.copy()).cuda()
            dev_out = torch.full((S * out_ss,), 0xA5, dtype=torch.uint8, device="cuda")
            gm.apply_batch(dev_in, in_ss, pitch, dev_out, out_ss, out_pitch, S, L)
            torch.cuda.synchronize()
            gm.apply_batch_host(host_in, in_ss, pitch, host_out, out_ss, out_pitch, S, L)
            want = dev_out.cpu().numpy()
            assert (host_out == want).all(), (case, ins, outs, L, pitch, S, in_ss, out_pitch, out_ss)
    finally:
        ecx.tune("host_chunk_kib", 65536)


def test_host_check_batch_random_layouts(ecx):
    """isParityCorrectBatchHost(Devices) over 24 random layouts -- RS(k, m) with k + m <= 24,
    shard lengths 1 .. 20,000 B, byte windows at random offsets, padded pitches, 1 .. 9 stripes,
    one device or [0, 0], 16 KiB host chunks -- with a random half of the stripes given one
    flipped byte inside or outside the window: every verdict equals the oracle's isParityCorrect."""
    rng = np.random.default_rng(20261018)
    ecx.tune("host_chunk_kib", 16)
    try:
        for case in range(24):
            k = int(rng.integers(1, 18))
            m = int(rng.integers(1, min(8, 25 - k)))
            n = k + m
            L = int(rng.integers(1, 20001))
            off = int(rng.integers(0, 64))
            win = int(rng.integers(0, L + 1)) if rng.random() < 0.3 else L
            pitch = off + L + int(rng.integers(0, 3)) * 16
            S = int(rng.integers(1, 10))
            host = rng.integers(0, 256, (S, n, pitch), dtype=np.uint8)
            for s in range(S):
                O.ReedSolomon(k, m).encode_parity([host[s, i] for i in range(n)], off, L)
            for s in range(S):
                if rng.random() < 0.5:
                    host[s, int(rng.integers(0, n)), off + int(rng.integers(0, L))] ^= int(rng.integers(1, 256))
            want = [1 if O.ReedSolomon(k, m).is_parity_correct([host[s, i].copy() for i in range(n)], off, win) else 0
                    for s in range(S)]
            rs = ecx.ReedSolomon.create(k, m)
            verdict = np.full(S, 7, np.uint8)
            if case % 2:
                rs.isParityCorrectBatchHostDevices(host, n * pitch, pitch, S, off, win, verdict, [0, 0])
            else:
                rs.isParityCorrectBatchHost(host, n * pitch, pitch, S, off, win, verdict)
            assert verdict.tolist() == want, (case, k, m, L, off, win, pitch, S)
    finally:
        ecx.tune("host_chunk_kib", 65536)
