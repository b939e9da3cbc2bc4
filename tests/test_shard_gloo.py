"""N > 1 path on CPU: world_size-2 gloo run of the subscriber-range sharding
used by `bench.py --mode sharded` (maxmq_amd/shard.py), shared subscriptions
included.  The per-shard matcher here is the oracle (no GPU in this
container); the GPU run swaps in the HIP index and the "nccl" (RCCL) backend,
with the same partition, broadcast and gather code."""

import hashlib

import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _key(filt, client) -> int:
    h = hashlib.blake2b(f"{filt}\0{client}".encode("utf-8", "surrogateescape"), digest_size=7).digest()
    return int.from_bytes(h, "little")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from maxmq_amd import shard
    from oracle.binding import OracleIndex
    from tools import mqgen

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = mqgen.generate(1, n_filters=4000, n_topics=3000, p_shared=0.1)
        # the batch exists on rank 0 only; the others receive it
        if rank == 0:
            data = torch.from_numpy(w.topics.data.copy())
            offs = torch.from_numpy(w.topics.offs.view(np.int64).copy())
        else:
            data = torch.zeros(len(w.topics.data), dtype=torch.uint8)
            offs = torch.zeros(len(w.topics.offs), dtype=torch.int64)
        shard.broadcast_batch(dist, data, offs, src=0)
        part = shard.shard_workload(w, world, rank)
        gen = shard.generated_shard(1, world, rank, n_filters=4000, n_topics=3000, p_shared=0.1)
        same_shard = bool(np.array_equal(gen.filters.data, part.filters.data)) and \
            bool(np.array_equal(gen.client_ids, part.client_ids))
        maps = shard.gather_maps(dist, torch.from_numpy(shard.local_client_map(gen).astype(np.int32)), dst=0)
        idx = OracleIndex()
        idx.subscribe_workload(part)
        doffs, dout, soffs, sout, _ = idx.match(data.numpy(), offs.numpy().view(np.uint64))
        counts = torch.from_numpy(np.diff(doffs).astype(np.int64))
        shard.reduce_counts(dist, counts, dst=0)
        # the shard's dense CSR: client id in the low word, QoS above it
        # (the GPU path sends packed mqm_delivery the same way)
        offs_t = torch.from_numpy(doffs.astype(np.int64))
        dl = torch.from_numpy(dout["client"].astype(np.int64) | (dout["qos"].astype(np.int64) << 32))
        parts = shard.gather_lists(dist, offs_t, dl, dst=0)
        # shared candidates: the GPU path sends shard-local shared ids and tags
        # them with the shard (mqm_gather_shards_shared); here each candidate
        # is a 56-bit key of (filter, client) names, tagged the same way
        keys = np.array([_key(idx.filter_name(int(f)), idx.client_name(int(c))) | (rank << 56)
                         for f, c in zip(sout["filter"], sout["client"])], dtype=np.int64)
        sparts = shard.gather_lists(dist, torch.from_numpy(soffs.astype(np.int64)), torch.from_numpy(keys), dst=0)
        if rank == 0:
            full = OracleIndex()
            full.subscribe_workload(w)
            fo, fd, fso, fs, _ = full.match(w.topics.data, w.topics.offs)
            nt = len(fo) - 1
            # mqm_gather_shards' layout, restated: topic t = shard 0's segment,
            # shard 1's, ...; clients through each shard's client map
            rows = []
            for t in range(nt):
                for r, (o, d) in enumerate(parts):
                    cm = shard.client_map(w, world, r)
                    seg = d.numpy()[int(o[t]):int(o[t + 1])]
                    rows += [(t, int(cm[c & 0xFFFFFFFF]), int(c >> 32)) for c in seg]
            node = [(t, int(c), int(q)) for t, c, q in zip(np.repeat(np.arange(nt), np.diff(fo).astype(np.int64)),
                                                        fd["client"], fd["qos"])]
            names_ok = all(full.client_name(i) == w.clients.data[w.clients.offs[j]:w.clients.offs[j + 1]].tobytes()
                           .decode() for i, j in [(0, 0)])
            srows = [(t, int(v) & ((1 << 56) - 1), r) for t in range(nt) for r, (o, d) in enumerate(sparts)
                     for v in d.numpy()[int(o[t]):int(o[t + 1])]]
            tags_ok = all(int(v) >> 56 == r for r, (o, d) in enumerate(sparts) for v in d.numpy())
            snode = [(int(t), _key(full.filter_name(int(f)), full.client_name(int(c))))
                     for t, f, c in zip(np.repeat(np.arange(nt), np.diff(fso).astype(np.int64)), fs["filter"], fs["client"])]
            shared_ok = tags_ok and len(snode) > 0 and sorted((t, k) for t, k, _ in srows) == sorted(snode)
            # every rank's client map reached rank 0, and maps shard ids to global client indexes
            cids = np.asarray(w.client_ids)
            maps_ok = same_shard and all(
                np.array_equal(maps[r].numpy().astype(np.uint32),
                               shard.local_client_map(shard.shard_workload(w, world, r))) and
                set(maps[r].numpy().tolist()) == set(cids[(cids >= shard.shard_bounds(int(cids.max()) + 1, world, r)[0]) &
                                                          (cids < shard.shard_bounds(int(cids.max()) + 1, world, r)[1])].tolist())
                for r in range(world))
            shared_ok = shared_ok and maps_ok
            out_q.put((np.array_equal(counts.numpy(), np.diff(fo).astype(np.int64)), sorted(rows) == sorted(node),
                       len(rows), len(rows) == len(set(rows)) and names_ok, shared_ok))
    finally:
        dist.destroy_process_group()


def test_subscriber_sharding_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    counts_ok, union_ok, n, disjoint, shared_ok = q.get(timeout=5)
    assert n > 0
    assert counts_ok, "sum of shard counts != node-wide counts"
    assert union_ok, "union of shard results != node-wide result"
    assert disjoint, "a (topic, client) pair came from two shards"
    assert shared_ok, "union of shard shared candidates != node-wide shared candidates"
