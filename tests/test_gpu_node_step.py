"""The subscriber-sharded node step (maxmq_amd.shard.node_step, the step of
`bench.py --mode sharded --gather device`) with two real rank processes and
the HIP matcher: both ranks hold their shard's index on the one GPU of the box
(two processes, two HIP contexts on cuda:0), the batch is broadcast, every
chunk is matched on the device (mqm_match_device + mqm_dense_device), the
shards' dense lists travel to rank 0 (gloo point-to-point: RCCL cannot put two
ranks on one device) and rank 0 lays them out with mqm_gather_shards on the
device.  The node-wide rows (topic, node client, QoS) must equal an unsharded
oracle's (oracle/mochi_ref.c, topics.go:484-555); shared candidates (filter,
client) likewise, gathered as name keys.  tests/test_node_step_gloo.py runs
the same step code with the oracle as the per-shard matcher on the CPU."""

import os
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests.test_node_step_gloo import _free_port, _key

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _worker(rank, world, chunk, port, out_q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import maxmq_amd
    from maxmq_amd import shard
    from oracle.binding import OracleIndex
    from tools import mqgen

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        w = mqgen.generate(1, n_filters=6000, n_topics=4000, p_shared=0.1, seed=0x90DE)
        if rank == 0:
            data = torch.from_numpy(w.topics.data.copy())
            offs = torch.from_numpy(w.topics.offs.view(np.int64).copy())
        else:
            data = torch.zeros(len(w.topics.data), dtype=torch.uint8)
            offs = torch.zeros(len(w.topics.offs), dtype=torch.int64)
        part = shard.shard_workload(w, world, rank)
        idx = maxmq_amd.TopicsIndex(device=0, autocommit=False)
        idx.subscribe_workload(part)
        idx.commit()
        cmaps = [torch.from_numpy(shard.client_map(w, world, r).astype(np.int32)).to(dev) for r in range(world)]
        from maxmq_amd.devbuf import dev_view_copy

        def match_chunk(t0, t1):
            o = offs.numpy().view(np.uint64)[t0:t1 + 1]
            tb = torch.from_numpy(data.numpy()[int(o[0]):int(o[-1])].copy()).to(dev)
            to = torch.from_numpy((o - o[0]).astype(np.int64)).to(dev)
            m = t1 - t0
            r = idx.match_device(tb.data_ptr(), to.data_ptr(), m)
            d = idx.dense_device()
            dofs = dev_view_copy(d.offsets, m + 1, torch.int64, dev).cpu()
            dl = dev_view_copy(d.deliveries, int(r.n_deliveries), torch.int64, dev).cpu()
            torch.cuda.synchronize()
            # shared candidates as (filter, client) name keys, from the host path
            res = idx.match_batch(data.numpy()[int(o[0]):int(o[-1])], o - o[0])
            keys = np.array([_key(idx.filter_name(int(x["filter"])), idx.client_name(int(x["client"])))
                             for x in res.sub_infos(res.shared, shared=True)], dtype=np.int64)
            return dofs, dl, torch.from_numpy(res.shared_offsets.astype(np.int64)), torch.from_numpy(keys)

        rows, srows = [], []

        def layout(t0, t1, parts, sparts):  # rank 0: mqm_gather_shards on the device
            m = t1 - t0
            tot = sum(int(dl.numel()) for _, dl in parts)
            dparts = [(o.to(dev), dl.to(dev)) for o, dl in parts]
            out_o = torch.empty(m + 1, dtype=torch.int64, device=dev)
            out_d = torch.empty(max(tot, 1), dtype=torch.int64, device=dev)
            maxmq_amd.gather_shards(m, [(o.data_ptr(), dl.data_ptr(), cmaps[i].data_ptr(), cmaps[i].numel())
                                        for i, (o, dl) in enumerate(dparts)], out_o.data_ptr(), out_d.data_ptr())
            oo, dd = out_o.cpu().numpy(), out_d[:tot].cpu().numpy()
            for t in range(m):
                for e in dd[int(oo[t]):int(oo[t + 1])]:
                    rows.append((t0 + t, int(e) & 0xFFFFFFFF, (int(e) >> 60) & 3))
            for so, sk in sparts:
                so, sk = so.numpy(), sk.numpy()
                for t in range(m):
                    srows.extend((t0 + t, int(k)) for k in sk[int(so[t]):int(so[t + 1])])

        shard.node_step(dist, data, offs, match_chunk, layout, chunk, src=0)
        if rank == 0:
            full = OracleIndex()
            full.subscribe_workload(w)
            fo, fd, fso, fs, _ = full.match(w.topics.data, w.topics.offs)
            nt = len(fo) - 1
            node = sorted(zip(np.repeat(np.arange(nt), np.diff(fo).astype(np.int64)).tolist(),
                              fd["client"].tolist(), fd["qos"].tolist()))
            snode = sorted((int(t), _key(full.filter_name(int(f)), full.client_name(int(c))))
                           for t, f, c in zip(np.repeat(np.arange(nt), np.diff(fso).astype(np.int64)),
                                              fs["filter"], fs["client"]))
            out_q.put((sorted(rows) == node, len(rows), len(node), sorted(srows) == snode, len(snode)))
        idx.close()
    finally:
        dist.destroy_process_group()


def test_node_step_two_ranks_hip_matcher():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, 1500, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    rows_ok, n, n_ref, shared_ok, n_shared = q.get(timeout=5)
    assert n_ref > 1000 and n_shared > 0, (n_ref, n_shared)
    assert rows_ok, f"node-wide rows ({n}) != unsharded oracle ({n_ref})"
    assert shared_ok, "node-wide shared candidates != unsharded oracle"
