"""The host-memory batch plan (host_pipe.cpp make_plan, exported as ecx_map_host_plan; host-only,
no device): how a host batch is chunked and how many strided copies each chunk takes -- the
160-stripe floor for many-run layouts and the folding of periodic runs into one copy per period
(DESIGN.md section 6).  The GPU side (tests/test_gpu_parity.py::
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


def test_headline_layout_is_not_folded_and_keeps_64_mib_chunks(ecx, default_chunks):
    """Clay(4,2) node 1, 32 KiB sub-chunks (the headline's e2e leg): 5 runs of 1-5 sub-chunks, no
    period spans the stripe, 20 x 32 KiB of input per stripe -> 102 stripes per 64 MiB chunk."""
    p = clay_plan(ecx, 4, 2, 0, [1], 32768, 2048)
    assert p == {"chunk": 102, "chunks": 21, "buffers": 3, "h2d_copies": 5, "h2d_rows": 1, "d2h_copies": 1,
                 "d2h_rows": 1}


def test_two_node_repair_folds_to_one_copy_per_chunk(ecx, default_chunks):
    """Clay(4,2) {0,3}: nodes 1-2 and 4-5 of all 8 planes, 16 runs of 2 at a fixed step of 3 slots
    -> one strided copy of 16 rows per stripe; more than 8 runs, so at least 160 stripes a chunk."""
    p = clay_plan(ecx, 4, 2, 0, [0, 3], 32768, 2048)
    assert p["h2d_copies"] == 1 and p["h2d_rows"] == 16
    assert p["d2h_copies"] == 1 and p["d2h_rows"] == 1  # the 16 repaired sub-chunks are one run
    assert p["chunk"] == 160 and p["chunks"] == 13


@pytest.mark.parametrize("erased,copies", [([3], 65), ([0], 64)])
def test_shortened_clay_runs_and_floor(ecx, default_chunks, erased, copies):
    """Shortened Clay(10,4), 4 KiB sub-chunks: node 3's helpers fill planes 192-255 with one-slot
    holes (65 runs, first and last different), node 0's planes 0-63 (64 runs of 13 that do not
    span the stripe): neither folds; 832 x 4 KiB per stripe -> the floor capped at 8 x 64 MiB of
    input = 157 stripes, so the e2e leg's 219-stripe calls take 2 chunks."""
    p = clay_plan(ecx, 10, 4, 2, erased, 4096, 219)
    assert p["h2d_copies"] == copies and p["h2d_rows"] == 1
    assert p["chunk"] == 157 and p["chunks"] == 2 and p["buffers"] == 2


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
