"""Hierarchical collectives for multi-node data parallelism (SURVEY §8(f)
row 4; the reference runs multi-node through NCCL over sockets, README.md:75-77,
with one flat all-reduce per bucket).

One process per GPU, L = ranks per node (LOCAL_WORLD_SIZE under
torch.distributed.run), N = nodes.  A SUM of packed words runs as

    intra-node reduce-scatter   (RCCL over xGMI)  each local rank ends up with
                                                  1/L of the words, summed
                                                  over its node
    inter-node all-reduce       (RCCL over the    among the N ranks with the
      of that shard              network)         same local rank: every NIC
                                                  carries 1/L of the payload
    intra-node all-gather       (xGMI)            the full summed stream

The lanes are sized for the GLOBAL world (gc_lane_layout with W = L*N), so
every partial sum is carry-free and uint32 addition is associative modulo
2^32: the result equals a flat all-reduce bit for bit, whatever order the
partial sums run in.  MAX (the max-norm) and the thermometer-mask SUM take the
same two levels.  With gloo (CPU tests) the reduce-scatter is an intra
all-reduce plus a slice, and the all-gather the list form.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


class NodeTopology:
    """Process groups of a node-major rank layout (rank = node * L + local)."""

    def __init__(self, local_size: int | None = None):
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("NodeTopology needs an initialised default process group")
        world, rank = dist.get_world_size(), dist.get_rank()
        L = int(local_size or os.environ.get("LOCAL_WORLD_SIZE", world))
        if L < 1 or world % L:
            raise ValueError(f"world {world} is not a whole number of nodes of {L} ranks")
        self.world, self.rank, self.local_size, self.nodes = world, rank, L, world // L
        self.node, self.local_rank = divmod(rank, L)
        self.intra = self.inter = None
        # every rank creates every group, in the same order (torch.distributed.new_group contract)
        for nd in range(self.nodes):
            g = dist.new_group(list(range(nd * L, (nd + 1) * L)))
            if nd == self.node:
                self.intra = g
        for lr in range(L):
            g = dist.new_group([nd * L + lr for nd in range(self.nodes)])
            if lr == self.local_rank:
                self.inter = g
        self._nccl = dist.get_backend() == "nccl"

    def all_reduce(self, t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
        """In-place all-reduce of t over the whole world, in two levels."""
        if self.world == 1:
            return t
        if op != dist.ReduceOp.SUM or self.local_size == 1 or t.numel() < self.local_size:
            # small or idempotent reductions: intra then inter on the whole tensor
            if self.local_size > 1:
                dist.all_reduce(t, op=op, group=self.intra)
            if self.nodes > 1:
                dist.all_reduce(t, op=op, group=self.inter)
            return t
        flat = t.view(-1)
        L = self.local_size
        shard = (flat.numel() + L - 1) // L
        if shard * L == flat.numel():
            buf = flat
        else:
            buf = torch.zeros(shard * L, dtype=t.dtype, device=t.device)
            buf[: flat.numel()].copy_(flat)
        mine = torch.empty(shard, dtype=t.dtype, device=t.device)
        if self._nccl:
            dist.reduce_scatter_tensor(mine, buf, op=op, group=self.intra)
        else:
            dist.all_reduce(buf, op=op, group=self.intra)
            mine.copy_(buf[self.local_rank * shard:(self.local_rank + 1) * shard])
        if self.nodes > 1:
            dist.all_reduce(mine, op=op, group=self.inter)
        if self._nccl:
            dist.all_gather_into_tensor(buf, mine, group=self.intra)
        else:
            dist.all_gather(list(buf.view(L, shard).unbind(0)), mine, group=self.intra)
        if buf.data_ptr() != flat.data_ptr():
            flat.copy_(buf[: flat.numel()])
        return t
