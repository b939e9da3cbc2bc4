"""Subscriber-range sharding across ranks.

Rank r of W holds the subscriptions of clients whose dense generator id lies
in [r*C/W, (r+1)*C/W).  The merge rule (packets.go:250-270) is per client, so
deduplication is shard-local and the shards' per-topic results are disjoint:
the node-wide result of a topic is the union of the shards' results and its
delivery count is their sum.  The publish batch enters at one rank and is
broadcast; the shards' dense per-topic lists go back to it with point-to-point
send/recv (RCCL has no gatherv), where mqm_gather_shards (shard.hip) lays
them out as one node-wide CSR (RCCL over xGMI with the "nccl" backend on GPUs,
gloo on CPU in the tests).
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


def generated_shard(config: int, world: int, rank: int, **overrides):
    """Shard `rank` of `world` of an mqgen config, generated directly: only
    the filters of its client range are kept (the full filter sequence is
    still drawn, so every rank sees the same topics).  This is how a
    100M-filter config is sharded without any host holding all of it."""
    from tools import mqgen

    n_filters = overrides.get("n_filters") or mqgen.default_params(config)["n_filters"]
    n_clients = overrides.get("n_clients") or (n_filters + 3) // 4
    lo, hi = shard_bounds(n_clients, world, rank)
    return mqgen.generate(config, client_lo=lo, client_hi=hi, **overrides)


def local_client_map(w) -> np.ndarray:
    """For a generated shard: shard client id (first appearance in subscribe
    order, as the shard's index interns them) -> the generator's global client
    index, used as the node-wide client id."""
    cid = np.asarray(w.client_ids)
    g, first = np.unique(cid, return_index=True)
    return g[np.argsort(first)].astype(np.uint32)


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


def client_map(w, world: int, rank: int) -> np.ndarray:
    """Shard `rank`'s interned client id -> the node-wide id (the id an
    unsharded index interns for that client: first appearance in subscribe
    order, store.cpp Interner).  Both orders are first appearance, so the
    shard's k-th distinct client maps to its rank among all clients."""
    cid = np.asarray(w.client_ids)
    gids, first = np.unique(cid, return_index=True)
    node_id = np.empty(int(gids.max()) + 1 if len(gids) else 0, np.uint32)
    node_id[gids[np.argsort(first)]] = np.arange(len(gids), dtype=np.uint32)
    lo, hi = shard_bounds(len(gids) and int(gids.max()) + 1, world, rank)
    part = cid[(cid >= lo) & (cid < hi)]
    pg, pf = np.unique(part, return_index=True)
    return node_id[pg[np.argsort(pf)]]


def gather_maps(dist, client_map, dst: int = 0):
    """Every shard's client map (int32 tensor) -> on dst the list of maps in
    rank order (setup, outside the timed step); elsewhere None."""
    import torch

    world, rank = dist.get_world_size(), dist.get_rank()
    nm = torch.tensor([client_map.numel()], dtype=torch.int64, device=client_map.device)
    sizes = [torch.zeros_like(nm) for _ in range(world)]
    dist.all_gather(sizes, nm)
    if rank != dst:
        for r in dist.batch_isend_irecv([dist.P2POp(dist.isend, client_map, dst)]):
            r.wait()
        return None
    maps, ops = [], []
    for r in range(world):
        if r == rank:
            maps.append(client_map)
            continue
        m = torch.empty(int(sizes[r].item()), dtype=client_map.dtype, device=client_map.device)
        ops.append(dist.P2POp(dist.irecv, m, r))
        maps.append(m)
    if ops:
        for q in dist.batch_isend_irecv(ops):
            q.wait()
    return maps


def gather_lists(dist, offsets, deliveries, dst: int = 0):
    """Send every shard's dense CSR (int64 offsets [n+1], int64 deliveries =
    packed mqm_delivery) to `dst` with point-to-point send/recv; -> on dst the
    per-rank (offsets, deliveries) tensors in rank order (its own included),
    elsewhere None.  Delivery counts travel first so receive buffers fit."""
    import torch

    world, rank = dist.get_world_size(), dist.get_rank()
    nd = torch.tensor([deliveries.numel()], dtype=torch.int64, device=offsets.device)
    sizes = [torch.zeros_like(nd) for _ in range(world)]
    dist.all_gather(sizes, nd)
    if rank != dst:
        ops = [dist.P2POp(dist.isend, offsets, dst), dist.P2POp(dist.isend, deliveries, dst)]
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        return None
    parts, ops = [], []
    for r in range(world):
        if r == rank:
            parts.append((offsets, deliveries))
            continue
        o = torch.empty_like(offsets)
        d = torch.empty(int(sizes[r].item()), dtype=deliveries.dtype, device=deliveries.device)
        ops += [dist.P2POp(dist.irecv, o, r), dist.P2POp(dist.irecv, d, r)]
        parts.append((o, d))
    if ops:
        for q in dist.batch_isend_irecv(ops):
            q.wait()
    return parts
