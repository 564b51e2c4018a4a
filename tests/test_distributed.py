"""Multi-rank (N>1) path on CPU with the gloo backend, world_size 2: stripe
sharding covers the batch exactly once with no overlap, every rank plans the
identical composed map (the planner is deterministic), and the bench's
max-over-ranks timing reduction works.  The data path itself has no
collective (stripes are independent)."""
import hashlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root))
    import rpamd
    ecx = rpamd.load()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ok = True
        for total in (0, 1, 7, 1 << 20, 12345):
            b, e = ecx.shard_stripes(total, world, rank)
            t = torch.tensor([b, e], dtype=torch.int64)
            allr = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(allr, t)
            ranges = sorted(tuple(x.tolist()) for x in allr)
            cover = 0
            for (lo, hi) in ranges:
                ok &= lo == cover and hi >= lo
                cover = hi
            ok &= cover == total
        mat, ins, outs = ecx.ClayCodeErasureDecodingStep([1], 4, 2).map().matrix()
        dig = int(hashlib.sha256(mat.tobytes() + ins.tobytes() + outs.tobytes()).hexdigest()[:12], 16)
        d = torch.tensor([dig], dtype=torch.int64)
        alld = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(alld, d)
        ok &= len({int(x) for x in alld}) == 1
        el = torch.tensor([1.0 + rank], dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        ok &= float(el) == float(world)
        dist.barrier()
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_sharding_and_planning():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
