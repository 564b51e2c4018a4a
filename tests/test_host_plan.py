"""The host-memory batch plan (host_pipe.cpp make_plan, exported as ecx_map_host_plan; host-only,
no device): how a host batch is chunked and how many copies each chunk takes -- the 160-stripe
floor for many-run layouts, periodic runs folded into one 2D copy per period, and other
progressions of equal runs moved by one 3D copy each.  The GPU side (tests/test_gpu_parity.py::
test_host_batch_folded_runs_match_device_batch) checks the bytes those copies move."""
import numpy as np
import pytest


@pytest.fixture
def default_chunks(ecx):
    ecx.tune("host_chunk_kib", 65536)
    ecx.tune("host_buffers", 3)
    yield
    ecx.tune("host_chunk_kib", 65536)
    ecx.tune("host_buffers", 3)


def clay_plan(ecx, k, m, v, erased, B, nstripes):
    step = ecx.ClayCodeErasureDecodingStep(erased, k, m, virtualUnits=v)
    inf = step.map().info()
    a = inf["n_out"] // len(erased)
    n = k + m
    return step.map().host_plan(n * a * B, B, len(erased) * a * B, B, nstripes, B)


def test_headline_layout_keeps_64_mib_chunks(ecx, default_chunks):
    """Clay(4,2) node 1, 32 KiB sub-chunks (the headline's e2e leg): runs of 1, 5, 5, 5 and 4
    sub-chunks (planes 4-7 without node 1), no period spans the stripe, the three runs of 5 six
    slots apart are one 3D copy; 20 x 32 KiB of input per stripe -> 102 stripes per 64 MiB chunk."""
    p = clay_plan(ecx, 4, 2, 0, [1], 32768, 2048)
    assert p == {"chunk": 102, "chunks": 21, "buffers": 3, "h2d_copies": 3, "h2d_rows": 3, "d2h_copies": 1,
                 "d2h_rows": 1, "h2d_3d": 1, "d2h_3d": 0, "slices": 1}


def test_two_node_repair_folds_to_one_copy_per_chunk(ecx, default_chunks):
    """Clay(4,2) {0,3}: nodes 1-2 and 4-5 of all 8 planes, 16 runs of 2 at a fixed step of 3 slots
    -> one strided copy of 16 rows per stripe, so the chunks keep host_chunk_kib's 64 MiB."""
    p = clay_plan(ecx, 4, 2, 0, [0, 3], 32768, 2048)
    assert p["h2d_copies"] == 1 and p["h2d_rows"] == 16 and p["h2d_3d"] == 0  # folded 2D, not 3D
    assert p["d2h_copies"] == 1 and p["d2h_rows"] == 1  # the 16 repaired sub-chunks are one run
    assert p["chunk"] == 64 and p["chunks"] == 32  # one copy a chunk: no floor, 64 MiB of input


@pytest.mark.parametrize("erased,copies,rows,n3d,chunk", [([3], 3, 63, 1, 19), ([0], 1, 64, 1, 19), ([5], 17, 4, 0, 157),
                                                           ([9], 5, 16, 0, 19), ([12], 2, 64, 0, 19), ([13], 1, 64, 0, 19)])
def test_shortened_clay_runs_and_floor(ecx, default_chunks, erased, copies, rows, n3d, chunk):
    """Shortened Clay(10,4), 4 KiB sub-chunks, one erased node per node row y (its helper planes
    are those whose digit y is the node's x): row 0 (nodes 0-3) reads 64 consecutive planes -- node
    0 64 runs of 13 that do not span the stripe, node 3 one-slot holes (65 runs: 3, 63 x 13 fourteen
    slots apart, 10) -- moved by 3D copies (1 and 3 per chunk instead of 64 and 65); rows 1 and 2
    (nodes 4-9) read blocks of planes that repeat across the stripe (68 runs folded into 17 2D
    copies of 4 rows, 80 into 5 of 16); row 3 (nodes 10-13) every 4th plane (2 or 1 folded copies).
    832 x 4 KiB per stripe: 19 stripes per 64 MiB chunk, or, where a chunk still takes more than 8
    copies, the floor capped at 8 x 64 MiB of input = 157 stripes (2 chunks of a 219-stripe call)."""
    p = clay_plan(ecx, 10, 4, 2, erased, 4096, 219)
    assert (p["h2d_copies"], p["h2d_rows"], p["h2d_3d"]) == (copies, rows, n3d), p
    assert p["chunk"] == chunk and p["chunks"] == -(-219 // chunk) and p["buffers"] == min(3, p["chunks"])


def test_padded_pitch_reading_every_slot_folds(ecx, default_chunks):
    """A map reading every slot of a padded-pitch stripe: one run per slot, period 1 spanning the
    stripe -> one copy of n rows per stripe; the separate dense output is one run."""
    n, L, P = 6, 1000, 1024
    g = ecx.GfMap.from_matrix(np.ones((1, n), np.uint8), list(range(n)), [0])
    p = g.host_plan(n * P, P, L, L, 50, L)
    assert p["h2d_copies"] == 1 and p["h2d_rows"] == n
    assert p["d2h_copies"] == 1 and p["d2h_rows"] == 1
    # back to back the slots merge into one run: nothing to fold
    q = g.host_plan(n * L, L, L, L, 50, L)
    assert q["h2d_copies"] == 1 and q["h2d_rows"] == 1


def test_small_chunks_and_empty_batches(ecx):
    """host_chunk_kib 16 gives one stripe per chunk and a full ring; an empty batch moves nothing."""
    ecx.tune("host_chunk_kib", 16)
    try:
        p = clay_plan(ecx, 4, 2, 0, [1], 2048, 7)
        assert p["chunk"] == 1 and p["chunks"] == 7 and p["buffers"] == 3
    finally:
        ecx.tune("host_chunk_kib", 65536)
    assert set(clay_plan(ecx, 4, 2, 0, [1], 2048, 0).values()) == {0}
    assert set(clay_plan(ecx, 4, 2, 0, [1], 0, 5).values()) == {0}


def test_one_huge_stripe_is_pipelined_in_column_slices(ecx, default_chunks):
    """Config 4 with 1 MiB sub-chunks: one 3.5 GiB stripe per call, 832 MiB of input -- one chunk of
    stripes, so the batch is cut into 13 column slices of 80 KiB (~64 MiB of input each, 4 KiB
    multiples, the last 64 KiB) that run through the ring; per slice each progression of runs is one
    copy.  A batch of a few ordinary stripes is not sliced."""
    p = clay_plan(ecx, 10, 4, 2, [3], 1 << 20, 1)
    assert p["slices"] == 13 and p["buffers"] == 3 and p["chunks"] == 1
    assert p["h2d_copies"] == 3 and p["d2h_copies"] == 1
    q = clay_plan(ecx, 10, 4, 2, [3], 4096, 12)  # 12 x 3.4 MB: one chunk, less than 4 chunks of input
    assert q["slices"] == 1
