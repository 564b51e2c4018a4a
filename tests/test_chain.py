"""Repair pipelining across ranks (repair-pipelining_amd/chain.py).

The CPU tests rehearse the chain's orchestration with gloo: slicing, the ring of
partial buffers, forwarding order, and delivery to a destination that is off the
chain.  They use world sizes 3 and 4, a ragged last slice, and the composed
Clay(4,2) and RS(12,4) maps.  The per-rank GF arithmetic is done by a test-only
numpy stand-in built on the oracle's multiplication table.  The GPU test runs
the same chain with the HIP kernels: 3 ranks, all on cuda:0, with gloo
transport.  The chain's output must equal the oracle's single-node repair.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class NumpyMap:
    """Test-only stand-in for GfMap (CPU tensors): out (^)= M * in per stripe."""

    def __init__(self, matrix, in_slot, out_slot):
        import oracle as O
        self.m, self.ins, self.outs = np.asarray(matrix), list(in_slot), list(out_slot)
        self.mt = O.mul_table()

    @classmethod
    def from_matrix(cls, matrix, in_slot, out_slot):
        return cls(matrix, in_slot, out_slot)

    def _run(self, inp, out, n, B, xor):
        x = inp.numpy().reshape(n, -1, B)
        a = out.numpy().reshape(n, -1, B)
        for s in range(n):
            for o, slot in enumerate(self.outs):
                acc = a[s, slot].copy() if xor else np.zeros(B, np.uint8)
                for c, j in zip(self.m[o], self.ins):
                    if c:
                        acc ^= self.mt[c][x[s, j]]
                a[s, slot] = acc

    def apply_batch(self, inp, iss, isl, out, oss, osl, n, B, stream=None):
        self._run(inp, out, n, B, False)

    def accumulate_batch(self, inp, iss, isl, out, oss, osl, n, B, stream=None):
        self._run(inp, out, n, B, True)


def _setup(rank, world, port):
    sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]
    import rpamd
    ecx = rpamd.load()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return ecx


def _clay_case(ecx, rank, world, node_rank, order, dest, S, B, slice_stripes, nbuf, device, factory):
    from repair_pipelining_amd.chain import RepairChain, clay_node_major_placement
    import oracle as O
    k, m, e, n, alpha = 4, 2, 1, 6, 8
    mat, ins, outs = ecx.ClayCodeErasureDecodingStep([e], k, m).map().matrix()
    rng = np.random.default_rng(11)
    stripes = rng.integers(0, 256, (S, n * alpha, B), dtype=np.uint8)  # plane-major, every rank the same
    place, nslots = clay_node_major_placement(n, alpha, node_rank)
    local = None
    if rank in nslots:
        loc = np.zeros((S, nslots[rank], B), np.uint8)
        for slot in range(n * alpha):
            r, ls = place(slot)
            if r == rank:
                loc[:, ls] = stripes[:, slot]
        local = torch.from_numpy(loc).to(device)
    chain = RepairChain(mat, ins, outs, place, order, rank, dest=dest, map_factory=factory)
    out = torch.zeros((S, alpha, B), dtype=torch.uint8, device=device) if rank == dest else None
    chain.run(local, S, B, out=out, slice_stripes=slice_stripes, n_buffers=nbuf, device=device)
    if rank != dest:
        return True
    got = out.cpu().numpy()
    ok = True
    for s in range(S):
        inputs = [None if (i % n) == e else stripes[s, i].copy() for i in range(n * alpha)]
        ref = [np.zeros(B, np.uint8) for _ in range(alpha)]
        O.Clay(k, m, [e]).perform_coding(inputs, ref, B)
        ok &= all((got[s, z] == ref[z]).all() for z in range(alpha))
    return bool(ok)


def _rs_case(ecx, rank, world, factory):
    """RS(12,4) 2-erasure decode along a chain of 3 ranks (4 shards each), dest = last."""
    from repair_pipelining_amd.chain import RepairChain, shard_placement
    k, m, S, L = 12, 4, 5, 96
    rs = ecx.ReedSolomon.create(k, m)
    present = [False, True, True, True, True, True, False] + [True] * 9
    mat, ins, outs = rs.decode_map(present).matrix()
    rng = np.random.default_rng(5)
    shards = rng.integers(0, 256, (S, 16, L), dtype=np.uint8)
    node_rank = [i * world // 16 for i in range(16)]
    place, nslots = shard_placement(node_rank)
    loc = np.zeros((S, nslots[rank], L), np.uint8)
    for sh in range(16):
        r, ls = place(sh)
        if r == rank:
            loc[:, ls] = shards[:, sh]
    chain = RepairChain(mat, ins, outs, place, list(range(world)), rank, map_factory=factory)
    dest = world - 1
    out = torch.zeros((S, 7, L), dtype=torch.uint8) if rank == dest else None  # out slots 0 and 6
    chain.run(torch.from_numpy(loc), S, L, out=out, slice_stripes=2, n_buffers=2)
    if rank != dest:
        return True
    import oracle as O
    ok = True
    for s in range(S):
        b = [shards[s, i].copy() for i in range(16)]
        O.ReedSolomon(k, m).decode_missing(b, present, 0, L)
        ok &= all((out[s, i].numpy() == b[i]).all() for i in (0, 6))
    return bool(ok)


def _cpu_worker(rank, world, port, q):
    ecx = _setup(rank, world, port)
    try:
        if world == 4:
            # nodes 0 | 2,3 | 4,5 on ranks 0..2; the rebuilt node 1 on rank 3, off the chain
            ok = _clay_case(ecx, rank, world, [0, 3, 1, 1, 2, 2], [0, 1, 2], 3, 7, 256, 2, 3, "cpu", NumpyMap)
        else:
            # dest = last rank of the chain; node 1 (erased) sits with rank 2
            ok = _clay_case(ecx, rank, world, [0, 2, 1, 1, 2, 2], [0, 1, 2], 2, 5, 128, 3, 2, "cpu", NumpyMap)
            ok &= _rs_case(ecx, rank, world, NumpyMap)
        dist.barrier()
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def _spawn(target, world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=280) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    return res


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [3, 4])
def test_chain_orchestration_gloo(world):
    assert _spawn(_cpu_worker, world) == {r: True for r in range(world)}


def test_chain_rejects_bad_order():
    sys.path[:0] = [str(ROOT), str(ROOT / "oracle")]
    import rpamd
    ecx = rpamd.load()
    from repair_pipelining_amd.chain import RepairChain, clay_node_major_placement
    mat, ins, outs = ecx.ClayCodeErasureDecodingStep([1], 4, 2).map().matrix()
    place, _ = clay_node_major_placement(6, 8, [0, 1, 1, 1, 2, 2])
    with pytest.raises(ValueError):
        RepairChain(mat, ins, outs, place, [0, 1], 0, map_factory=NumpyMap)  # rank 2 owns inputs
    with pytest.raises(ValueError):
        RepairChain(mat, ins, outs, place, [0, 1, 2], 0, dest=1, map_factory=NumpyMap)


def _gpu_worker(rank, world, port, q):
    ecx = _setup(rank, world, port)
    try:
        torch.cuda.set_device(0)
        ecx.set_device(0)
        ok = _clay_case(ecx, rank, world, [0, 2, 1, 1, 2, 2], [0, 1, 2], 2, 9, 4096, 4, 3, "cuda", None)
        torch.cuda.synchronize()
        dist.barrier()
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_chain_hip_kernels_three_ranks():
    """3 ranks on one GPU (gloo transport staged through the host), HIP partial-sum kernels."""
    assert _spawn(_gpu_worker, 3) == {0: True, 1: True, 2: True}
