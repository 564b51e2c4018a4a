"""Pipelined repair chain across GPUs (repair-pipelining_amd/chain.py), Clay(4,2) e=1.

Launch one process per GPU:
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 scripts/chain_bench.py
Helper nodes 0,2,3,4,5 are spread round-robin over ranks 0..N-2, which form the chain.
The rebuilt node 1 lives on rank N-1, which is the destination (off the chain).  With
N=1, everything is on rank 0.  Each rank holds its nodes' sub-chunks node-major for
--stripes stripes.  Slices of --slice stripes flow along the chain as partial sums,
over RCCL P2P ("nccl") or, with ECX_CHAIN_BACKEND=gloo, staged through the host
(a rehearsal on a box with fewer GPUs than ranks).
Prints one driver-style JSON line on the destination rank (the bench.py fields: metric,
value, unit, n_gpus, ...): the algorithmic GiB/s of stripes repaired through the chain
(917,504 B per stripe, as in bench.py), the per-hop partial-sum rate in GB/s, the slice
size and the chain of ranks.  `--gpus N` without a launcher starts the N ranks itself
(torch.distributed.run as a child process, as bench.py does).  The reference's shape
is ClayCoordinator.kt:265-319 (decodeDecoupledData: the partial-sum chain along
nodesPath) and ClayCodeNode.kt:165-233 (each hop's decodeMissingSingle and forward).
"""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=2048)
    ap.add_argument("--slice", type=int, default=128)
    ap.add_argument("--buffers", type=int, default=3)
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE, else 1)")
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        import socket
        import subprocess
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
               "--master-addr=127.0.0.1", "--master-port=%d" % port, str(Path(__file__).resolve())] + sys.argv[1:]
        raise SystemExit(subprocess.run(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1")).returncode)
    import torch
    import torch.distributed as dist
    import rpamd
    ecx = rpamd.load()
    from repair_pipelining_amd.chain import RepairChain, clay_node_major_placement

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    backend = os.environ.get("ECX_CHAIN_BACKEND", "nccl")
    torch.cuda.set_device(local_rank)
    ecx.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    K, M, E, N, A, B = 4, 2, 1, 6, 8, 32768
    helpers = [i for i in range(N) if i != E]
    chain_ranks = max(1, world - 1)
    node_rank = [0] * N
    for j, node in enumerate(helpers):
        node_rank[node] = j % chain_ranks
    node_rank[E] = world - 1
    order = sorted(set(node_rank[h] for h in helpers))
    dest = world - 1
    mat, ins, outs = ecx.ClayCodeErasureDecodingStep([E], K, M).map().matrix()
    place, nslots = clay_node_major_placement(N, A, node_rank)
    S = args.stripes
    local = None
    if rank in nslots:
        local = torch.empty((S, nslots[rank], B), dtype=torch.uint8, device=dev)
        ecx.fill_random(local, local.numel(), 1000 + rank)
    out = torch.empty((S, A, B), dtype=torch.uint8, device=dev) if rank == dest else None
    chain = RepairChain(mat, ins, outs, place, order, rank, dest=dest)

    def once():
        chain.run(local, S, B, out=out, slice_stripes=args.slice, n_buffers=args.buffers, device=dev)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    once()
    best = None
    for _ in range(args.repeats):
        t0 = time.perf_counter()
        once()
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    if rank == dest:
        print(json.dumps({
            "metric": "GiB/s pipelined partial-sum repair chain (device-resident), Clay(4,2) 32 KiB blocks",
            "value": round(S * 917504 / best / 2**30, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "higher_is_better": True,
            "dtype": "u8",
            "data": "synthetic (device splitmix64 sub-chunks)",
            "config": {"workload": "Clay(4,2) repair of node 1 through a chain of %d rank(s), helpers node-major "
                                   "per rank, destination rank %d" % (len(order), dest),
                       "stripes": S, "slice_stripes": args.slice, "buffers": args.buffers},
            "backend": backend if world > 1 else "none",
            "chain": order,
            "dest": dest,
            "seconds": round(best, 4),
            "stripes_per_s": round(S / best, 1),
            "per_hop_GB_per_s": round(S * A * B / best / 1e9, 2),
            "per_hop_bytes_per_stripe": A * B,
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
