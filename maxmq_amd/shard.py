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


def _ranks(dist, group):
    """(world size, this rank) within `group` (None = the default group)"""
    return dist.get_world_size(group), dist.get_rank(group)


def _peer(dist, group, r: int) -> int:
    """global rank of group rank r (point-to-point ops take global ranks)"""
    return r if group is None else dist.get_global_rank(group, r)


def broadcast_batch(dist, data, offs, src: int = 0, group=None):
    """Broadcast a topic batch (uint8 bytes + int64 offsets tensors) from
    global rank `src` to `group`; other ranks pass tensors of the right size
    (sizes go first)."""
    import torch

    sizes = torch.tensor([data.numel(), offs.numel()], dtype=torch.int64, device=data.device)
    dist.broadcast(sizes, src=src, group=group)
    if dist.get_rank() != src and (data.numel() != int(sizes[0]) or offs.numel() != int(sizes[1])):
        raise ValueError("receiver buffers do not match the broadcast batch")
    dist.broadcast(data, src=src, group=group)
    dist.broadcast(offs, src=src, group=group)
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


def gather_maps(dist, client_map, dst: int = 0, group=None):
    """Every shard's client map (int32 tensor) -> on global rank dst the list
    of maps in group rank order (setup, outside the timed step); elsewhere
    None."""
    import torch

    world, rank = _ranks(dist, group)
    nm = torch.tensor([client_map.numel()], dtype=torch.int64, device=client_map.device)
    sizes = [torch.zeros_like(nm) for _ in range(world)]
    dist.all_gather(sizes, nm, group=group)
    if dist.get_rank() != dst:
        for r in dist.batch_isend_irecv([dist.P2POp(dist.isend, client_map, dst, group)]):
            r.wait()
        return None
    maps, ops = [], []
    for r in range(world):
        if r == rank:
            maps.append(client_map)
            continue
        m = torch.empty(int(sizes[r].item()), dtype=client_map.dtype, device=client_map.device)
        ops.append(dist.P2POp(dist.irecv, m, _peer(dist, group, r), group))
        maps.append(m)
    if ops:
        for q in dist.batch_isend_irecv(ops):
            q.wait()
    return maps


def _recv_buf(cache, key, count, dtype, device):
    """a receive buffer of at least `count` elements, kept across steps
    (grown, never shrunk) -> its first `count` elements"""
    import torch

    t = cache.get(key) if cache is not None else None
    if t is None or t.numel() < count or t.dtype != dtype:
        t = torch.empty(max(int(count * 1.25), 1), dtype=dtype, device=device)
        if cache is not None:
            cache[key] = t
    return t[:count]


def gather_lists(dist, offsets, deliveries, dst: int = 0, group=None, cache=None, tag=""):
    """Send every shard's dense CSR (int64 offsets [n+1], int64 deliveries =
    packed mqm_delivery) to global rank `dst` of `group` with point-to-point
    send/recv; -> on dst the per-rank (offsets, deliveries) tensors in group
    rank order (its own included), elsewhere None.  Delivery counts travel
    first so receive buffers fit; with `cache` (a dict kept by the caller)
    the receive buffers are reused from step to step (one set per `tag`: the
    lists of two gathers of one step must not share buffers)."""
    import torch

    world, rank = _ranks(dist, group)
    nd = torch.tensor([deliveries.numel()], dtype=torch.int64, device=offsets.device)
    sizes = [torch.zeros_like(nd) for _ in range(world)]
    dist.all_gather(sizes, nd, group=group)
    if dist.get_rank() != dst:
        ops = [dist.P2POp(dist.isend, offsets, dst, group), dist.P2POp(dist.isend, deliveries, dst, group)]
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        return None
    parts, ops = [], []
    for r in range(world):
        if r == rank:
            parts.append((offsets, deliveries))
            continue
        o = _recv_buf(cache, (tag, "o", r), offsets.numel(), offsets.dtype, offsets.device)
        d = _recv_buf(cache, (tag, "d", r), int(sizes[r].item()), deliveries.dtype, deliveries.device)
        peer = _peer(dist, group, r)
        ops += [dist.P2POp(dist.irecv, o, peer, group), dist.P2POp(dist.irecv, d, peer, group)]
        parts.append((o, d))
    if ops:
        for q in dist.batch_isend_irecv(ops):
            q.wait()
    return parts


# ---- the node step (bench.py --mode sharded / hybrid) --------------------------


def plan_chunk(n_topics: int, node_deliveries_per_topic: float, node_shared_per_topic: float,
               budget_bytes: float) -> int:
    """Topics per gather so that one gathered chunk fits `budget_bytes` on
    the receiving rank: it holds every shard's received dense lists (8 B per
    delivery, 4 B per shared candidate) and the node-wide CSR laid out from
    them (the same again), plus 4 int64 offset arrays per shard and node."""
    per_topic = 16.0 * node_deliveries_per_topic + 8.0 * node_shared_per_topic + 64.0
    return int(max(1, min(n_topics, budget_bytes // per_topic)))


def node_step(dist, data, offs, match_chunk, layout, chunk: int, src: int = 0, group=None, cache=None):
    """One subscriber-sharded node step over `group` (None = every rank):
    global rank `src` broadcasts the batch (bytes + offsets), then for every
    chunk [t0, t1) of at most `chunk` topics each shard matches it
    (match_chunk(t0, t1) -> this shard's dense (offsets, deliveries,
    shared_offsets, shared) of the chunk, offsets rebased to 0) and sends the
    lists to `src`, which lays them out (layout(t0, t1, parts, shared_parts)).
    Chunking bounds what `src` holds at once (plan_chunk).  -> (this shard's
    deliveries, shared candidates) summed over the chunks."""
    broadcast_batch(dist, data, offs, src=src, group=group)
    n = offs.numel() - 1
    nd = ns = 0
    for t0 in range(0, n, max(1, chunk)):
        t1 = min(n, t0 + max(1, chunk))
        o, d, so, sh = match_chunk(t0, t1)
        nd += int(d.numel())
        ns += int(sh.numel())
        parts = gather_lists(dist, o, d, dst=src, group=group, cache=cache, tag="deliveries")
        sparts = gather_lists(dist, so, sh, dst=src, group=group, cache=cache, tag="shared")
        if parts is not None:
            layout(t0, t1, parts, sparts)
    return nd, ns


def hybrid_layout(world: int, shards: int):
    """Hybrid node layout: `shards` subscriber shards x world // shards topic
    replicas.  Global rank r is shard r % shards of replica group r // shards;
    each group's leader (its shard 0) receives and broadcasts the group's batch
    and lays the group's node-wide result out.  -> (groups as lists of global
    ranks, for every rank (group index, shard index))."""
    if shards < 1 or world % shards:
        raise ValueError(f"{world} ranks do not split into groups of {shards} shards")
    groups = [list(range(g * shards, (g + 1) * shards)) for g in range(world // shards)]
    return groups, [(r // shards, r % shards) for r in range(world)]
