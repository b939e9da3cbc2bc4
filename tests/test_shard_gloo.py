"""N > 1 path on CPU: world_size-2 gloo run of the subscriber-range sharding
used by `bench.py --mode sharded` (maxmq_amd/shard.py).  The per-shard matcher
here is the oracle (no GPU in this container); the GPU run swaps in the HIP
index and the "nccl" (RCCL) backend, with the same partition, broadcast and
reduce code."""

import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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
        w = mqgen.generate(1, n_filters=4000, n_topics=3000, p_shared=0.0)
        # the batch exists on rank 0 only; the others receive it
        if rank == 0:
            data = torch.from_numpy(w.topics.data.copy())
            offs = torch.from_numpy(w.topics.offs.view(np.int64).copy())
        else:
            data = torch.zeros(len(w.topics.data), dtype=torch.uint8)
            offs = torch.zeros(len(w.topics.offs), dtype=torch.int64)
        shard.broadcast_batch(dist, data, offs, src=0)
        part = shard.shard_workload(w, world, rank)
        idx = OracleIndex()
        idx.subscribe_workload(part)
        doffs, dout, _, _, _ = idx.match(data.numpy(), offs.numpy().view(np.uint64))
        counts = torch.from_numpy(np.diff(doffs).astype(np.int64))
        shard.reduce_counts(dist, counts, dst=0)
        # the shard's dense CSR: client id in the low word, QoS above it
        # (the GPU path sends packed mqm_delivery the same way)
        offs_t = torch.from_numpy(doffs.astype(np.int64))
        dl = torch.from_numpy(dout["client"].astype(np.int64) | (dout["qos"].astype(np.int64) << 32))
        parts = shard.gather_lists(dist, offs_t, dl, dst=0)
        if rank == 0:
            full = OracleIndex()
            full.subscribe_workload(w)
            fo, fd, _, _, _ = full.match(w.topics.data, w.topics.offs)
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
            out_q.put((np.array_equal(counts.numpy(), np.diff(fo).astype(np.int64)), sorted(rows) == sorted(node),
                       len(rows), len(rows) == len(set(rows)) and names_ok))
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
    counts_ok, union_ok, n, disjoint = q.get(timeout=5)
    assert n > 0
    assert counts_ok, "sum of shard counts != node-wide counts"
    assert union_ok, "union of shard results != node-wide result"
    assert disjoint, "a (topic, client) pair came from two shards"
