"""The sharded node step of `bench.py --mode sharded|hybrid` on CPU (gloo):
maxmq_amd.shard.node_step with a small gather chunk (world size 2, one group
of 2 subscriber shards: the batch is gathered in several chunks so the
receiving rank never holds the whole node-wide result), and the hybrid layout
(world size 4 = 2 subscriber shards x 2 topic replicas: each replica group
broadcasts, matches and gathers its own batch inside its own process group).
The per-shard matcher is the oracle (no GPU here); the GPU run swaps in the
HIP index, RCCL and mqm_gather_shards with the same step code.  Every group's
laid-out node-wide result must equal an unsharded oracle's result for that
group's batch: deliveries by (topic, node client, QoS), shared candidates by
(topic, filter name, client name)."""

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


def _worker(rank, world, shards, chunk, port, out_q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from maxmq_amd import shard
    from oracle.binding import OracleIndex
    from tools import mqgen
    from tools.mqgen import Strings

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        groups, lay = shard.hybrid_layout(world, shards)
        pgs = [dist.new_group(g) for g in groups]  # every rank creates every group, in order
        g, s = lay[rank]
        pg, leader = pgs[g], groups[g][0]
        w = mqgen.generate(1, n_filters=4000, n_topics=3000, p_shared=0.1)
        # replica group g's batch: its slice of the topics (held by its leader only)
        per = len(w.topics) // len(groups)
        mine = Strings.from_list([w.topics[i] for i in range(g * per, (g + 1) * per)])
        if rank == leader:
            data = torch.from_numpy(mine.data.copy())
            offs = torch.from_numpy(mine.offs.view(np.int64).copy())
        else:
            data = torch.zeros(len(mine.data), dtype=torch.uint8)
            offs = torch.zeros(len(mine.offs), dtype=torch.int64)
        part = shard.shard_workload(w, shards, s)
        idx = OracleIndex()
        idx.subscribe_workload(part)

        def match_chunk(t0, t1):
            o = offs.numpy().view(np.uint64)[t0:t1 + 1]
            d = data.numpy()[int(o[0]):int(o[-1])]
            doffs, dout, soffs, sout, _ = idx.match(d, o - o[0])
            dl = torch.from_numpy(dout["client"].astype(np.int64) | (dout["qos"].astype(np.int64) << 32))
            keys = np.array([_key(idx.filter_name(int(f)), idx.client_name(int(c))) | (s << 56)
                             for f, c in zip(sout["filter"], sout["client"])], dtype=np.int64)
            return (torch.from_numpy(doffs.astype(np.int64)), dl, torch.from_numpy(soffs.astype(np.int64)),
                    torch.from_numpy(keys))

        rows, srows, chunks = [], [], []
        cmaps = [shard.client_map(w, shards, r) for r in range(shards)]

        def layout(t0, t1, parts, sparts):  # mqm_gather_shards' layout, restated
            chunks.append((t0, t1))
            for t in range(t1 - t0):
                for r, (o, d) in enumerate(parts):
                    rows.extend((t0 + t, int(cmaps[r][c & 0xFFFFFFFF]), int(c >> 32))
                                for c in d.numpy()[int(o[t]):int(o[t + 1])])
                for r, (o, d) in enumerate(sparts):
                    srows.extend((t0 + t, int(v) & ((1 << 56) - 1), int(v) >> 56) for v in d.numpy()[int(o[t]):int(o[t + 1])])

        cache = {}
        for _ in range(2):  # two steps: receive buffers reused from the cache
            rows.clear(), srows.clear(), chunks.clear()
            shard.node_step(dist, data, offs, match_chunk, layout, chunk, src=leader, group=pg, cache=cache)
        if rank == leader:
            full = OracleIndex()
            full.subscribe_workload(w)
            fo, fd, fso, fs, _ = full.match(mine.data, mine.offs)
            nt = len(fo) - 1
            node = sorted(zip(np.repeat(np.arange(nt), np.diff(fo).astype(np.int64)).tolist(),
                              fd["client"].tolist(), fd["qos"].tolist()))
            snode = sorted((int(t), _key(full.filter_name(int(f)), full.client_name(int(c))))
                           for t, f, c in zip(np.repeat(np.arange(nt), np.diff(fso).astype(np.int64)),
                                              fs["filter"], fs["client"]))
            covered = sorted(chunks) == [(a, min(nt, a + chunk)) for a in range(0, nt, chunk)]
            out_q.put((g, sorted(rows) == node, len(rows), len(rows) == len(set(rows)),
                       sorted((t, k) for t, k, _ in srows) == snode and len(snode) > 0, covered, len(chunks)))
    finally:
        dist.destroy_process_group()


def _run(world, shards, chunk):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, shards, chunk, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return [q.get(timeout=5) for _ in range(world // shards)]


def test_node_step_chunked_gather_two_shards():
    (g, union_ok, n, disjoint, shared_ok, covered, nchunks), = _run(2, 2, 700)
    assert n > 0 and nchunks == 5  # 3000 topics in chunks of 700
    assert covered, "the chunks do not tile the batch"
    assert union_ok, "chunked node-wide result != unsharded result"
    assert disjoint, "a (topic, client) pair came from two shards"
    assert shared_ok, "chunked node-wide shared candidates != unsharded ones"


def test_hybrid_two_shards_by_two_replicas():
    res = _run(4, 2, 1000)
    assert sorted(r[0] for r in res) == [0, 1]  # both replica groups reported
    for g, union_ok, n, disjoint, shared_ok, covered, nchunks in res:
        assert n > 0 and covered and nchunks == 2, (g, n, covered, nchunks)
        assert union_ok, f"group {g}: node-wide result != unsharded result"
        assert disjoint, f"group {g}: a (topic, client) pair came from two shards"
        assert shared_ok, f"group {g}: shared candidates differ"
