"""Subscriber-range sharding across ranks.

Rank r of W holds the subscriptions of clients whose dense generator id lies
in [r*C/W, (r+1)*C/W).  The merge rule (packets.go:250-270) is per client, so
deduplication is shard-local and the shards' per-topic results are disjoint:
the node-wide result of a topic is the union of the shards' results and its
delivery count is their sum.  The publish batch enters at one rank and is
broadcast; per-topic counts are reduced back (RCCL over xGMI with the "nccl"
backend on GPUs, gloo on CPU in the tests).
"""

from __future__ import annotations

import numpy as np


def shard_bounds(n_clients: int, world: int, rank: int):
    return rank * n_clients // world, (rank + 1) * n_clients // world


def shard_workload(w, world: int, rank: int):
    """The subset of a tools.mqgen.Workload whose clients belong to `rank`,
    in the original subscribe order (so client/filter interning stays dense)."""
    from tools.mqgen import Strings

    n_clients = int(w.client_ids.max()) + 1 if len(w.client_ids) else 0
    lo, hi = shard_bounds(n_clients, world, rank)
    keep = np.nonzero((w.client_ids >= lo) & (w.client_ids < hi))[0]

    def sub(s):
        return Strings.from_list([bytes(s.data[s.offs[i]:s.offs[i + 1]]) for i in keep])

    class Shard:
        pass

    o = Shard()
    o.filters, o.clients = sub(w.filters), sub(w.clients)
    for k in ("qos", "no_local", "rap", "rh", "ident", "client_ids"):
        setattr(o, k, getattr(w, k)[keep])
    o.topics = w.topics
    return o


def broadcast_batch(dist, data, offs, src: int = 0):
    """Broadcast a topic batch (uint8 bytes + int64 offsets tensors) from
    `src`; other ranks pass tensors of the right size (sizes go first)."""
    import torch

    sizes = torch.tensor([data.numel(), offs.numel()], dtype=torch.int64, device=data.device)
    dist.broadcast(sizes, src=src)
    if dist.get_rank() != src and (data.numel() != int(sizes[0]) or offs.numel() != int(sizes[1])):
        raise ValueError("receiver buffers do not match the broadcast batch")
    dist.broadcast(data, src=src)
    dist.broadcast(offs, src=src)
    return data, offs


def reduce_counts(dist, counts, dst: int = 0):
    """Sum the shards' per-topic delivery counts at `dst`."""
    dist.reduce(counts, dst=dst)
    return counts
