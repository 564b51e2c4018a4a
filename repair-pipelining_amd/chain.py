"""Repair pipelining across GPUs: the partial-sum chain.

This is the multi-GPU analogue of the reference's pipelined repair.
``ClayCoordinator.decodeDecoupledData`` (ClayCoordinator.kt:265-319) sends each
helper node an order along ``nodesPath``.  Each helper adds its
``decodeMissingSingle`` contribution to the running partial it received and
forwards the partial to the next helper (``ClayCodeNode.decodeAndSend``,
ClayCodeNode.kt:165-193).  The last helper ships the result to the node being
rebuilt (``sendDecodedData``, :205-233).  Before that chain runs, the reference
exchanges couple sub-chunks between helpers to decouple them
(``getAndStoreDecoupledData``, ClayCoordinator.kt:207-238).

Here each rank (one GPU) holds the sub-chunks of some nodes, node-major, for a
batch of stripes.  The whole repair is ONE composed GF(256) linear map ``M``
(the planner composes decouple, RS decode and re-couple).  So a node's share of
the output is just ``M[:, its columns] @ its sub-chunks``, and the decouple
exchange disappears:

    rank p in the chain:  partial  = recv(prev)          (p > 0)
                          partial ^= M_p @ local slice   (HIP accumulate kernel)
                          send(partial, next)            (unless p is last)

Each hop carries ``|outputs|`` sub-chunks per stripe, which is the reference's
per-hop traffic.  Stripes are cut into slices and sent with non-blocking P2P
(RCCL over xGMI with the "nccl" backend), so rank p computes slice s+1 while
slice s travels to rank p+1.  That pipelining is the point of the reference's
design.

The per-rank kernels are the library's compiled maps (``GfMap``); there is no CPU
fallback.  ``map_factory`` exists only so that CPU tests can rehearse the
orchestration with gloo and a test-only stand-in.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

Placement = Callable[[int], Tuple[int, int]]  # global input slot -> (rank, local slot)


def clay_node_major_placement(n: int, alpha: int, node_rank: Sequence[int]) -> Tuple[Placement, Dict[int, int]]:
    """Clay stripes stored node-major per rank: rank r holds its nodes (ascending),
    each as alpha consecutive sub-chunks, so the local slot of (node, plane z) is
    ``rank_local_node_index * alpha + z``.  The global slot is ``z * n + node``, the
    reference's plane-major order (ClayCodeErasureDecodingStep.java:84-97).
    Returns (placement, local slots per rank)."""
    nodes_of: Dict[int, List[int]] = {}
    for node, r in enumerate(node_rank):
        nodes_of.setdefault(r, []).append(node)
    local_index = {node: nodes_of[r].index(node) for node, r in enumerate(node_rank)}

    def place(slot: int) -> Tuple[int, int]:
        z, node = divmod(slot, n)
        return node_rank[node], local_index[node] * alpha + z

    return place, {r: len(v) * alpha for r, v in nodes_of.items()}


def shard_placement(node_rank: Sequence[int]) -> Tuple[Placement, Dict[int, int]]:
    """RS / LRC stripes: global slot = shard index, one shard per node."""
    nodes_of: Dict[int, List[int]] = {}
    for node, r in enumerate(node_rank):
        nodes_of.setdefault(r, []).append(node)

    def place(slot: int) -> Tuple[int, int]:
        r = node_rank[slot]
        return r, nodes_of[r].index(slot)

    return place, {r: len(v) for r, v in nodes_of.items()}


class RepairChain:
    """One rank's part of a pipelined partial-sum repair.

    matrix, in_slot, out_slot: the composed map (``GfMap.matrix()``), i.e. output row o
        is sum_j matrix[o, j] * input(in_slot[j]), written to output slot out_slot[o].
    placement: global input slot -> (rank, local slot) (see the helpers above).
    order: the chain, i.e. the ranks in forwarding order (``nodesPath``).  Only ranks
        owning a column with a non-zero coefficient need to appear.
    dest: rank that receives the repaired sub-chunks (the rebuilt node's GPU).
        ``None`` means the last rank of ``order``.
    """

    def __init__(self, matrix, in_slot, out_slot, placement: Placement, order: Sequence[int], rank: int,
                 dest: Optional[int] = None, group=None, map_factory=None):
        m = np.asarray(matrix, dtype=np.uint8)
        self.rank, self.order, self.group = rank, list(order), group
        self.dest = self.order[-1] if dest is None else dest
        self.n_out_slots = int(max(out_slot)) + 1
        cols_of: Dict[int, List[int]] = {}
        for j, slot in enumerate(in_slot):
            r, _ = placement(int(slot))
            if m[:, j].any():
                cols_of.setdefault(r, []).append(j)
        missing = sorted(set(cols_of) - set(self.order))
        if missing:
            raise ValueError(f"ranks {missing} own inputs of the map but are not on the chain")
        if self.dest in self.order and self.dest != self.order[-1]:
            raise ValueError("dest must be the last rank of the chain or off the chain (the rebuilt node)")
        self.pos = self.order.index(rank) if rank in self.order else -1
        self.map, self.n_cols = None, 0
        cols = cols_of.get(rank, []) if self.pos >= 0 else []
        if cols:
            if map_factory is None:
                from . import GfMap
                map_factory = GfMap.from_matrix
            local = [placement(int(in_slot[j]))[1] for j in cols]
            self.map = map_factory(np.ascontiguousarray(m[:, cols]), in_slot=local, out_slot=list(out_slot))
            self.n_cols = len(cols)

    # ---------------------------------------------------------------- transport
    def _isend(self, t, dst):
        import torch.distributed as dist
        if t.is_cuda and dist.get_backend(self.group) != "nccl":
            dist.send(t.cpu(), dst, group=self.group)  # gloo rehearsal: staged through the host
            return None
        return dist.isend(t, dst, group=self.group)

    def _irecv(self, t, src):
        import torch.distributed as dist
        if t.is_cuda and dist.get_backend(self.group) != "nccl":
            return _StagedRecv(t, src, self.group)
        return dist.irecv(t, src, group=self.group)

    # ---------------------------------------------------------------- run
    def run(self, local, nstripes: int, sub_bytes: int, out=None, slice_stripes: int = 64, n_buffers: int = 3,
            device=None):
        """Repair `nstripes` stripes.

        local: this rank's sub-chunks, a [nstripes][local slots][sub_bytes] uint8 tensor.
        out: on `dest`, a contiguous [nstripes][n_out_slots][sub_bytes] tensor that receives
            the repaired sub-chunks.
        device: where the partial-sum ring lives when this rank has neither `local` nor `out`
            (a forward-only chain member).
        Ranks off the chain (and not dest) return at once.
        """
        import torch
        if self.pos < 0 and self.rank != self.dest:
            return
        B, S = sub_bytes, nstripes
        row = self.n_out_slots * B
        n_slices = (S + slice_stripes - 1) // slice_stripes
        last = self.pos == len(self.order) - 1
        nxt = self.dest if last else (self.order[self.pos + 1] if self.pos >= 0 else None)
        prev = self.order[self.pos - 1] if self.pos > 0 else None
        if self.pos < 0:  # dest off the chain: receive finished slices straight into `out`
            for s in range(n_slices):
                lo, hi = s * slice_stripes, min(S, (s + 1) * slice_stripes)
                w = self._irecv(out[lo:hi], self.order[-1])
                w.wait()
            return
        deliver_here = last and self.dest == self.rank
        dev = device if device is not None else (local.device if local is not None else out.device)
        ring = [] if deliver_here else [torch.empty((slice_stripes, self.n_out_slots, B), dtype=torch.uint8,
                                                    device=dev) for _ in range(n_buffers)]
        sends: List[Optional[object]] = [None] * max(1, n_buffers)
        lstride = local.shape[1] * B if self.n_cols else 0

        def target(s, n):
            if deliver_here:
                lo = s * slice_stripes
                return out[lo:lo + n]
            k = s % n_buffers
            if sends[k] is not None:  # the ring slot's previous send must be done before reuse
                sends[k].wait()
                sends[k] = None
            return ring[k][:n]

        pending = None
        if prev is not None:
            n0 = min(S, slice_stripes)
            t0 = target(0, n0)
            pending = (t0, self._irecv(t0, prev))
        for s in range(n_slices):
            lo, hi = s * slice_stripes, min(S, (s + 1) * slice_stripes)
            n = hi - lo
            if pending is not None:
                acc, work = pending
                work.wait()
            else:
                acc = target(s, n)
            if prev is not None and s + 1 < n_slices:
                n1 = min(S, (s + 2) * slice_stripes) - (s + 1) * slice_stripes
                t1 = target(s + 1, n1)
                pending = (t1, self._irecv(t1, prev))
            else:
                pending = None
            if self.n_cols:
                src = local[lo:hi]
                if self.pos == 0:
                    self.map.apply_batch(src, lstride, B, acc, row, B, n, B)
                else:
                    self.map.accumulate_batch(src, lstride, B, acc, row, B, n, B)
            elif self.pos == 0:
                acc.zero_()
            if not deliver_here:
                sends[s % n_buffers] = self._isend(acc, nxt)
        for w in sends:
            if w is not None:
                w.wait()


class _StagedRecv:
    """gloo rehearsal of a device-tensor irecv: host receive then copy to the device."""

    def __init__(self, t, src, group):
        self.t, self.src, self.group = t, src, group

    def wait(self):
        import torch
        import torch.distributed as dist
        host = torch.empty(self.t.shape, dtype=self.t.dtype)
        dist.recv(host, self.src, group=self.group)
        self.t.copy_(host)
