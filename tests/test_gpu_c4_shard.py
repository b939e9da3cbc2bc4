"""BASELINE configs[3] (100M filters, subscriber-sharded over 8 GPUs) as the
per-GPU unit of a node step: shard 0 of the 8-way client-range split
(maxmq_amd/shard.py: 12.5M filters, generated directly) against the full
10M-topic batch, through the same mqm_match_device call `bench.py --shard 0/8
--config 4` and the sharded node step time.

C4 is the config that drove the widest merges before '#' subscriptions after a
literal parent became solo (kFlagParentLit, snapshot.h): with the old marking
(MQM_HASH_MULTI=1, the same store flattened again) hub topics carry
thousands of multi entries (the k_multi<4096> tier); the test
asserts the k_multi<4096> tier ran there and that both markings give the same
result for every topic (per-topic counts, and checksums over (client, first
filter, QoS, NoLocal): sids are snapshot positions, which the marking moves).  On the default index
it checks:
  * over all 10M topics (~6G deliveries, walked in chunks of whole topics):
    dense CSR monotone and summing to n_deliveries, client ids below the
    shard's client count, QoS <= 2, no client twice in a topic, run-to-run
    equality of every topic's checksum (mix64 sum of its entries);
  * bit-exact against oracle/mochi_ref.c built from the same shard on a
    sample of 50k random topics plus the 300 topics with the most deliveries
    (the widest merges): the full-batch rows of
    those topics equal the host-path rows, which equal the oracle's field by
    field (client, max QoS, NoLocal, first filter, its identifier, RAP, RH;
    shared candidates by (filter, client)).
Reference: vendor/github.com/mochi-co/mqtt/v2/topics.go:484-555 (Subscribers,
gatherSubscriptions, gatherSharedSubscriptions), packets/packets.go:250-270
(Subscription.Merge); north_star C4."""

import numpy as np
import pytest

import maxmq_amd
from maxmq_amd import shard
from oracle.binding import OracleIndex
from tests.gpu_util import assert_same, canon_gpu, canon_oracle
from tools.mqgen import Strings

pytestmark = pytest.mark.gpu


def _filter_map(idx, w, dev):
    """sid -> interned filter id of the index's current snapshot (device int64)"""
    import torch

    nsub = int(idx.snapshot_stats()["subs"])
    res = idx.match_batch(*_one_topic(w))
    f = res.sub_infos(np.arange(nsub, dtype=np.uint32))["filter"].astype(np.int64)
    return torch.from_numpy(f).to(dev)


def _one_topic(w):
    s = Strings.from_list([w.topics[0]])
    return s.data, s.offs


def _stable_mix(e, fmap, tid):
    """a delivery (client | packed << 32) as (client, first filter, QoS | NoLocal), mixed with its topic"""
    from maxmq_amd.devbuf import mix64

    packed = e >> 32
    key = (e & 0xFFFFFFFF) | (fmap[packed & 0x0FFFFFFF] << 32)
    return mix64(key ^ mix64(((packed >> 28) & 7) ^ mix64(tid)))


def test_config4_shard0of8_full_batch():
    import torch

    from maxmq_amd.devbuf import dev_view_copy, iter_csr_chunks, mix64

    w = shard.generated_shard(4, 8, 0)
    n = len(w.topics)
    assert n == 10_000_000 and len(w.filters) > 12_000_000, (n, len(w.filters))
    idx = maxmq_amd.TopicsIndex(0, autocommit=False)
    idx.subscribe_workload(w)
    idx.commit()
    dev = torch.device("cuda:0")
    tb = torch.from_numpy(w.topics.data).to(dev)
    to = torch.from_numpy(w.topics.offs.view(np.int64)).to(dev)
    ncl = idx.num_clients()

    def run():
        r = idx.match_device(tb.data_ptr(), to.data_ptr(), n)
        d = idx.dense_device()
        offs = dev_view_copy(d.offsets, n + 1, torch.int64, dev)
        torch.cuda.synchronize()
        return r, d, offs

    r1, d1, offs = run()
    nd = int(r1.n_deliveries)
    assert nd > 300 * n, nd  # ~620 deliveries per topic on this shard
    print(f"C4 shard 0/8 default marking: tiers t2={r1.n_tier2} t3={r1.n_tier3} part={r1.n_part} "
          f"dfs={r1.n_fallback}")
    assert int(offs[0]) == 0 and int(offs[-1]) == nd
    assert bool((offs[1:] >= offs[:-1]).all())
    # every entry of every topic, in chunks of whole topics: client in range,
    # QoS <= 2, no client twice in a topic, per-topic checksum
    sums1 = torch.zeros(n, dtype=torch.int64, device=dev)
    # per-topic checksums over (client, first filter, QoS, NoLocal): sids are
    # snapshot positions and differ between snapshots built with different
    # markings (a range lists its solo entries first), filter ids do not
    fmap = _filter_map(idx, w, dev)
    stable1 = torch.zeros(n, dtype=torch.int64, device=dev)
    for lo, hi, a, e, sid in iter_csr_chunks(offs, d1.deliveries, torch.int64):
        stable1.index_add_(0, sid, _stable_mix(e, fmap, sid))
        client = e & 0xFFFFFFFF
        assert int(client.max()) < ncl
        assert int(((e >> 60) & 3).max()) <= 2  # packed word (high half): qos at its bits 28..29
        key = torch.sort((sid << 32) | client).values
        assert not bool((key[1:] == key[:-1]).any()), f"a client appears twice in one topic of [{lo}, {hi})"
        sums1.index_add_(0, sid, mix64(e ^ mix64(sid)))
        del client, key
    # the bit-exact sample: 50k random topics + the 300 with the most deliveries
    rng = np.random.default_rng(4)
    o = offs.cpu().numpy()
    top = np.argsort(np.diff(o))[-300:]
    small = np.unique(np.concatenate([rng.choice(n, size=50000, replace=False), top]))
    cnt = (o[small + 1] - o[small]).astype(np.int64)
    pos = torch.from_numpy(np.repeat(o[small] - np.concatenate([[0], np.cumsum(cnt)[:-1]]), cnt)
                           + np.arange(cnt.sum())).to(dev)
    # run-to-run: the same call again gives the same per-topic checksums; the
    # sample's rows are taken from this second result
    r2, d2, offs2 = run()
    assert torch.equal(offs2, offs)
    sums2 = torch.zeros(n, dtype=torch.int64, device=dev)
    full_rows = torch.empty(len(pos), dtype=torch.int64, device=dev)
    for lo, hi, a, e, sid in iter_csr_chunks(offs2, d2.deliveries, torch.int64):
        sums2.index_add_(0, sid, mix64(e ^ mix64(sid)))
        inside = torch.nonzero((pos >= a) & (pos < a + e.numel())).flatten()
        full_rows[inside] = e[pos[inside] - a]
    assert torch.equal(sums2, sums1), "run-to-run per-topic checksums differ"

    full_rows = full_rows.cpu().numpy().view(np.uint64)
    del offs2, sums2, pos, d1, d2
    sub = Strings.from_list([w.topics[int(i)] for i in small])
    res = idx.match_batch(sub.data, sub.offs)
    assert np.array_equal(cnt, np.diff(res.offsets).astype(np.int64)), "per-topic counts differ from the host path"
    tid = np.repeat(np.arange(len(small), dtype=np.uint64), cnt)
    host_rows = res.deliveries.view(np.uint64)
    assert np.array_equal(np.unique(np.stack([tid, full_rows], 1), axis=0),
                          np.unique(np.stack([tid, host_rows], 1), axis=0)), "full-batch rows != host-path rows"
    del full_rows, host_rows, tid
    g, gs = canon_gpu(res)
    del res
    ora = OracleIndex()
    ora.subscribe_workload(w)
    ref, rs = canon_oracle(*ora.match(sub.data, sub.offs, nthreads=16)[:4])
    ora.close()
    assert len(g) > 1_000_000
    assert_same(g, ref, "C4 shard 0/8 deliveries (sample)")
    assert_same(gs, rs, "C4 shard 0/8 shared (sample)")
    # the old marking ('#' subscriptions after a literal parent multi): the wide
    # merge tiers and the DFS path under load, and the same result per topic.
    # The same store is flattened again with MQM_HASH_MULTI=1 (read at
    # flatten time): a Subscribe + Unsubscribe of a path no topic reaches moves
    # the store version (a commit at an unchanged version is a no-op) and
    # leaves the trie as it was (its names intern after every existing id), so
    # no second 12.5M-filter store is built
    import os

    idx_h = idx
    assert idx_h.subscribe("zz-marking-probe", maxmq_amd.Subscription("zz/marking/probe", 0))
    assert idx_h.unsubscribe("zz/marking/probe", "zz-marking-probe")
    os.environ["MQM_HASH_MULTI"] = "1"
    try:
        idx_h.commit()
    finally:
        del os.environ["MQM_HASH_MULTI"]
    rh = idx_h.match_device(tb.data_ptr(), to.data_ptr(), n)
    dh = idx_h.dense_device()
    offs_h = dev_view_copy(dh.offsets, n + 1, torch.int64, dev)
    torch.cuda.synchronize()
    # (no C4 topic has more than 3072 multi entries, so the client-partitioned
    # merge does not run here: tests/test_gpu_parity.py's 4000-entry topic covers it)
    assert rh.n_tier3 > 0, "the k_multi<4096> tier never ran"
    # (no C4 topic has more than 64 hits since the walk records a '#' child
    # after a literal once; the DFS path is covered by test_gpu_queued.py and
    # test_gpu_parity.py's edge cases)
    print(f"C4 shard 0/8 old marking: tiers t2={rh.n_tier2} t3={rh.n_tier3} part={rh.n_part} dfs={rh.n_fallback}")
    assert torch.equal(offs_h, offs), "per-topic counts differ between the two markings"
    fmap_h = _filter_map(idx_h, w, dev)
    stable_h = torch.zeros(n, dtype=torch.int64, device=dev)
    for lo, hi, a, e, sid in iter_csr_chunks(offs_h, dh.deliveries, torch.int64):
        stable_h.index_add_(0, sid, _stable_mix(e, fmap_h, sid))
    assert torch.equal(stable_h, stable1), "per-topic (client, first filter, QoS, NoLocal) differ between the markings"
    del dh, offs_h, stable_h
    idx_h.close()
