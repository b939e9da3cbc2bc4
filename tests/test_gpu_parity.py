"""GPU parity tests (MI355X): the HIP match path, called through the C ABI,
against the hand-derived known-answer table, the frozen golden fixture, the C
oracle on the same seeded inputs, and size-independent properties at the
BASELINE sizes.  Bit-exact: every (topic, client, max QoS, NoLocal, first
filter, its identifier, RAP, RH) row and every shared (topic, filter, client)
candidate must be identical."""

import os
import random

import numpy as np
import pytest

import maxmq_amd
from maxmq_amd import capi
from oracle import mochi_ref as pyref
from oracle.binding import OracleIndex
from tests.gpu_util import assert_same, canon_gpu, canon_gpu_idents, canon_oracle, canon_oracle_idents
from tools import mqgen
from tools.mqgen import Strings

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gpu_and_oracle(filters, topics, clients=None, subs=None):
    idx = maxmq_amd.TopicsIndex(0)
    ora = OracleIndex()
    for i, f in enumerate(filters):
        c = clients[i] if clients else f"c{i}"
        q, nl, rap, rh, ident = subs[i] if subs else (i % 3, 0, 0, 0, 0)
        idx.subscribe(c, maxmq_amd.Subscription(f, q, ident, bool(nl), bool(rap), rh))
        ora.subscribe(c, f, q, nl, rap, rh, ident)
    s = Strings.from_list(topics)
    res = idx.match_batch(s.data, s.offs)
    g, gs = canon_gpu(res)
    r, rs = canon_oracle(*ora.match(s.data, s.offs)[:4])
    return (g, gs), (r, rs), res


def test_kat_forward(kat):
    for case in kat["forward"]:
        idx = maxmq_amd.TopicsIndex(0)
        for i, f in enumerate(case["filters"]):
            idx.subscribe(f"c{i}", maxmq_amd.Subscription(f, qos=1))
        got = idx.subscribers(case["topic"])
        assert sorted(s.filter for s in got.subscriptions.values()) == sorted(case["subs"]), case
        assert sorted(got.shared) == sorted(case["shared"]), case


def test_kat_merge(kat):
    for case in kat["merge"]:
        idx = maxmq_amd.TopicsIndex(0)
        for c, f, q, nl, rap, rh, ident in case["subs"]:
            idx.subscribe(c, maxmq_amd.Subscription(f, q, ident, bool(nl), bool(rap), rh))
        got = idx.subscribers(case["topic"])
        out = {c: dict(qos=s.qos, no_local=int(s.no_local), first=s.filter, first_ident=s.identifier,
                       rap=int(s.retain_as_published), rh=s.retain_handling) for c, s in got.subscriptions.items()}
        assert out == case["expect"], case


def test_golden_fixture():
    z = np.load(os.path.join(ROOT, "tests", "golden", "c1_fixture.npz"))
    idx = maxmq_amd.TopicsIndex(0)
    fs, cs = Strings(z["filters_data"], z["filters_offs"]), Strings(z["clients_data"], z["clients_offs"])

    class W:  # the subset of tools.mqgen.Workload subscribe_workload reads
        filters, clients = fs, cs
        qos, no_local, rap, rh, ident = z["qos"], z["no_local"], z["rap"], z["rh"], z["ident"]

    idx.subscribe_workload(W)
    res = idx.match_batch(z["topics_data"], z["topics_offs"])
    g, gs = canon_gpu(res)
    dout = np.zeros(len(z["dclient"]), dtype=[("client", "<u4"), ("first_filter", "<u4"), ("first_ident", "<i4"),
                                              ("qos", "u1"), ("no_local", "u1"), ("rap", "u1"), ("rh", "u1")])
    dout["client"], dout["first_filter"], dout["first_ident"] = z["dclient"], z["dfilter"], z["dident"]
    dout["qos"], dout["no_local"], dout["rap"], dout["rh"] = z["dqos"], z["dno_local"], z["drap"], z["drh"]
    sout = np.zeros(len(z["sclient"]), dtype=[("filter", "<u4"), ("client", "<u4")])
    sout["filter"], sout["client"] = z["sfilter"], z["sclient"]
    r, rs = canon_oracle(z["doffs"], dout, z["soffs"], sout)
    assert_same(g, r, "deliveries")
    assert_same(gs, rs, "shared")


@pytest.mark.parametrize("config,overrides", [
    (1, {}),                                   # BASELINE configs[0]: 10k filters, 100k topics
    (5, dict(n_filters=200000, n_topics=200000)),  # shared subscriptions + MQTT 5 options
])
def test_config_vs_oracle(config, overrides):
    w = mqgen.generate(config, **overrides)
    idx = maxmq_amd.TopicsIndex(0)
    idx.subscribe_workload(w)
    ora = OracleIndex()
    ora.subscribe_workload(w)
    res = idx.match_batch(w.topics.data, w.topics.offs)
    g, gs = canon_gpu(res)
    r, rs = canon_oracle(*ora.match(w.topics.data, w.topics.offs, nthreads=16)[:4])
    assert len(r) > 0
    assert_same(g, r, "deliveries")
    assert_same(gs, rs, "shared")


@pytest.mark.parametrize("merge", ["fast", "resolve", "table"])
def test_edge_cases_and_fallback_paths(merge, monkeypatch):
    """every edge case through the one-launch path for small batches (fast.hip,
    the default for this batch size) and through the batch pipeline
    (MQM_NO_FAST=1) with multi entries merged by resolution (partner lists,
    MQM_RESOLVE=1) or by hash table (MQM_RESOLVE=0: the k_merge_small / k_merge /
    k_multi<1024|2048|4096> / k_multi_part tiers)"""
    if merge != "fast":
        monkeypatch.setenv("MQM_NO_FAST", "1")
    if merge != "fast":
        monkeypatch.setenv("MQM_RESOLVE", "1" if merge == "resolve" else "0")
    filters, clients, topics = [], [], []
    # heavy clients (merged by hash table even with resolution on): 70 filters
    # each (> 64 per client: no pairwise marking), all under "hv" and matching
    # "hv/a/b/c/d/e/f" (every prefix, each level after the first literal or
    # '+'), 50 clients -> 350 heavy multi entries for "hv/a/b" (a workgroup
    # tier); and a client with 20 compatible filters (> 15 partners each: heavy)
    hv = ["hv", "a", "b", "c", "d", "e", "f"]
    hvf = []
    for k in range(1, 8):
        for m in range(1 << (k - 1)):
            hvf.append("/".join(["hv"] + ["+" if (m >> (b - 1)) & 1 else hv[b] for b in range(1, k)]))
    for i in range(50):
        filters += hvf[:70]
        clients += [f"hv{i}"] * 70
    filters += hvf[100:120]
    clients += ["p20"] * 20
    # 4 compatible filters per client (3 partners: the partner list, not inline)
    for i in range(30):
        filters += ["q4/a/b", "q4/+/b", "q4/a/+", "q4/#"]
        clients += [f"q{i}"] * 4
    topics += ["hv/a/b/c/d/e/f", "hv/a/b", "hv/x/b/c/d/e/f/g", "q4/a/b", "q4/z/b", "q4"]
    # hub: 1000 clients on a/# and a/b -> S > 384 per topic (global dedupe path)
    for i in range(1000):
        filters += ["hub/#", "hub/x"]
        clients += [f"h{i}", f"h{i}"]
    topics += ["hub/x", "hub", "hub/x/y"]
    # 4000 multi entries for one topic: past the 4096-slot single-pass tier
    # (k_multi<4096> takes up to 3072) -> the partitioned workgroup merge
    for i in range(2000):
        filters += ["hub2/#", "hub2/x"]
        clients += [f"k{i}", f"k{i}"]
    topics += ["hub2/x", "hub2/x/y"]
    # 300 raw entries, all multi: the wave tier's table is too small -> workgroup tier
    for i in range(100):
        filters += ["m/#", "m/y"]
        clients += [f"m{i}", f"m{i}"]
    topics += ["m/y", "m", "m/z"]
    # a client whose filters cannot co-match (solo entries) next to one whose can
    filters += ["p/q/r", "p/s/r", "p/+/r", "p/q/#"]
    clients += ["solo", "solo", "multi", "multi"]
    topics += ["p/q/r", "p/s/r", "p/q"]
    # deep topics (> 16 levels) and deep filters (walk beyond the LDS level cache)
    deep = "/".join(f"l{i}" for i in range(40))
    filters += [deep, "/".join(["+"] * 20) + "/#", "l0/#", "/".join(f"l{i}" for i in range(25)) + "/#"]
    clients += ["d1", "d2", "d3", "d4"]
    topics += [deep, deep + "/z", "/".join(f"l{i}" for i in range(18))]
    # long tokens (>= 16 bytes: hashed key + byte verification)
    lt = "x" * 40
    filters += [f"{lt}/a", f"{lt}/+", "y" * 16, "z" * 15]
    clients += ["t1", "t2", "t3", "t4"]
    topics += [f"{lt}/a", f"{lt[:-1]}y/a", "y" * 16, "y" * 17, "z" * 15]
    # frontier blow-up: every {a, +} combination over 6 levels under w/
    for m in range(64):
        filters.append("w/" + "/".join("+" if (m >> k) & 1 else "a" for k in range(6)))
        clients.append(f"f{m % 7}")
    topics += ["w/a/a/a/a/a/a", "w/a/a/a/a/a/a/a"]
    # many shared groups on one node (> 32 shared hits is not a thing: one node
    # -> one hit; but many nodes with shared subs along a wildcard walk)
    for g in range(50):
        filters += [f"$SHARE/g{g}/s/+", f"$share/g{g}/s/#"]
        clients += [f"s{g}", f"s{g}"]
    topics += ["s/q", "s", "$SYS/s"]
    # '$' rules, empty levels, unicode
    filters += ["#", "+/+", "$SYS/#", "+", "/", "é/ü/+", "$SHARE/g/#"]
    clients += ["u1", "u2", "u3", "u4", "u5", "u6", "u7"]
    topics += ["$SYS/x", "$x", "/", "//", "", "é/ü/ß", "a", "$", "a/+", "a/#"]
    (g, gs), (r, rs), res = _gpu_and_oracle(filters, topics, clients)
    assert_same(g, r, "deliveries")
    assert_same(gs, rs, "shared")
    # the same batch through the device pipeline: the merge kernels that ran
    import torch

    s = Strings.from_list(topics)
    idx = res._index
    tb = torch.from_numpy(s.data).cuda()
    to = torch.from_numpy(s.offs.view(np.int64)).cuda()
    r = idx.match_device(tb.data_ptr(), to.data_ptr(), len(topics))
    torch.cuda.synchronize()
    assert int(r.n_deliveries) == len(g), (int(r.n_deliveries), len(g))
    if merge == "resolve":
        assert r.n_resolve > 0 and r.n_big > 0, (r.n_resolve, r.n_big)
    elif merge == "table":
        assert r.n_resolve == 0 and r.n_part > 0, (r.n_resolve, r.n_part)
    else:
        assert r.n_resolve + r.n_big > 0, (r.n_resolve, r.n_big)
    rng = random.Random(99)
    levels = ["a", "b", "", "+", "#", "$SYS", "$x", "c" * 18]
    for trial in range(8):
        idx = maxmq_amd.TopicsIndex(0)
        py = pyref.TopicsIndex()
        for step in range(400):
            f = "/".join(rng.choice(levels) for _ in range(rng.randint(1, 5)))
            c = f"k{rng.randint(0, 7)}"
            if rng.random() < 0.7:
                q = rng.randint(0, 2)
                assert idx.subscribe(c, maxmq_amd.Subscription(f, q)) == py.subscribe(c, pyref.Sub(f, q))
            else:
                assert idx.unsubscribe(f, c) == py.unsubscribe(f, c)
            if step % 50 == 49:
                topics = ["/".join(rng.choice(["a", "b", "", "$SYS", "$x", "c" * 18]) for _ in range(rng.randint(1, 6)))
                          for _ in range(50)]
                s = Strings.from_list(topics)
                res = idx.match_batch(s.data, s.offs)
                for i, t in enumerate(topics):
                    subs, shared = py.subscribers(t)
                    lo, hi = res.offsets[i], res.offsets[i + 1]
                    _, qos, _ = capi.delivery_fields(res.deliveries["packed"][lo:hi])
                    got = sorted((idx.client_name(int(cl)), int(q)) for cl, q in zip(res.deliveries["client"][lo:hi], qos))
                    assert got == sorted((k, v.qos) for k, v in subs.items()), (trial, step, t)


def test_full_size_c2_properties():
    """BASELINE configs[1] at full size (1M filters, 10M topics): exact
    agreement with the oracle on a 100k-topic sample, and size-independent
    properties over the whole batch (CSR monotone, per-topic clients unique and
    within range, QoS <= 2, deterministic across two runs)."""
    w = mqgen.generate(2)
    idx = maxmq_amd.TopicsIndex(0)
    idx.subscribe_workload(w)
    idx.commit()
    import torch

    dev = torch.device("cuda:0")
    tb = torch.from_numpy(w.topics.data).to(dev)
    to = torch.from_numpy(w.topics.offs.view(np.int64)).to(dev)
    n = len(w.topics)
    rng = np.random.default_rng(5)
    sample = np.sort(rng.choice(n, size=100000, replace=False))

    def segments(r):
        """per-topic counts (all topics) and the sample's packed deliveries
        (4 B: first sub | qos << 28 | no_local << 30), sorted within topic"""
        starts = _dev_copy(r.starts, n * 8).view(np.uint64).astype(np.int64)
        counts = _dev_copy(r.counts, n * 4).view(np.uint32).astype(np.int64)
        end = int((starts + counts).max()) if n else 0
        buf = _dev_copy(r.deliveries, end * 4).view(np.uint32)
        st, ct = starts[sample], counts[sample]
        tid = np.repeat(sample, ct)
        pos = np.repeat(st - np.concatenate([[0], np.cumsum(ct)[:-1]]), ct) + np.arange(ct.sum())
        ents = buf[pos]
        o = np.lexsort((ents, tid))
        return starts, counts, ents[o], tid[o]

    r1 = idx.match_device(tb.data_ptr(), to.data_ptr(), n)
    torch.cuda.synchronize()
    nd = int(r1.n_deliveries)
    starts, counts, ents, tid = segments(r1)
    r2 = idx.match_device(tb.data_ptr(), to.data_ptr(), n)
    torch.cuda.synchronize()
    assert int(r2.n_deliveries) == nd
    s2, c2, e2, _ = segments(r2)
    # same per-topic results run to run (DFS-path topics live in a tail whose
    # placement and internal order follow atomics: compared as sorted sets)
    assert np.array_equal(c2, counts) and np.array_equal(e2, ents)
    assert counts.sum() == nd
    # segments never overlap
    o = np.argsort(starts, kind="stable")
    assert np.all(starts[o][1:] >= (starts + counts)[o][:-1])
    sub = Strings.from_list([w.topics[int(i)] for i in sample])
    res = idx.match_batch(sub.data, sub.offs)  # same snapshot: resolves sids to clients
    first, qos, _ = capi.delivery_fields(ents)
    assert np.all(qos <= 2)
    clients = res.sub_infos(first)["client"].astype(np.uint32)
    assert clients.max() < idx.num_clients()
    key = (tid.astype(np.uint64) << np.uint64(32)) | clients.astype(np.uint64)
    assert len(np.unique(key)) == len(key), "a client appears twice in one topic"
    # the full-batch segments of the sample == the host path's rows for it
    htid = np.repeat(sample, np.diff(res.offsets).astype(np.int64))
    hp = res.deliveries["packed"]
    o2 = np.lexsort((hp, htid))
    assert np.array_equal(htid[o2], tid) and np.array_equal(hp[o2], ents), "full-batch segments != host-path rows"
    # exact agreement with the oracle on the same sample of topics
    ora = OracleIndex()
    ora.subscribe_workload(w)
    r, rs = canon_oracle(*ora.match(sub.data, sub.offs, nthreads=16)[:4])
    g, gs = canon_gpu(res)
    assert_same(g, r, "deliveries (sample)")
    assert_same(gs, rs, "shared (sample)")


def _dev_copy(ptr, nbytes):
    import ctypes

    import torch

    out = np.empty(nbytes, np.uint8)
    if nbytes:
        torch.cuda.synchronize()
        hip = ctypes.CDLL("libamdhip64.so")
        rc = hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes),
                           ctypes.c_int(2))
        assert rc == 0
    return out


# ---- Subscription.Identifiers (packets.go:250-259, rule M3) -------------------------------------

def test_kat_identifiers(kat):
    for case in kat["merge"]:
        idx = maxmq_amd.TopicsIndex(0, identifiers=True)
        for c, f, q, nl, rap, rh, ident in case["subs"]:
            idx.subscribe(c, maxmq_amd.Subscription(f, q, ident, bool(nl), bool(rap), rh))
        got = idx.subscribers(case["topic"])
        assert {c: s.identifiers for c, s in got.subscriptions.items()} == case["identifiers"], case


@pytest.mark.parametrize("config,overrides", [(1, {}), (5, dict(n_filters=200000, n_topics=100000))])
def test_identifiers_vs_oracle(config, overrides):
    w = mqgen.generate(config, **overrides)
    idx = maxmq_amd.TopicsIndex(0, identifiers=True)
    idx.subscribe_workload(w)
    ora = OracleIndex()
    ora.subscribe_workload(w)
    res = idx.match_batch(w.topics.data, w.topics.offs)
    g = canon_gpu_idents(res)
    r = canon_oracle_idents(*ora.identifiers(w.topics.data, w.topics.offs, nthreads=16))
    assert (r["ident"] > 0).sum() > 0
    assert_same(g, r, "identifiers")


def test_identifiers_dfs_topics_and_device_form(monkeypatch):
    """Hubs of identified subscriptions (9000 multi entries per topic: the
    partitioned workgroup merge) and topics deeper than the walk's 16 cached
    levels (the unbounded DFS path), with identifiers.  The host call runs the
    batch pipeline too (MQM_NO_FAST=1), so its listed sids and the device
    form's come from the same pass (k_ident lists multi entries only: a solo
    delivery's map is its first pair)."""
    filters, clients, subs = [], [], []
    for i in range(3000):  # 3 compatible filters per client: 9000 multi entries on hub/x
        filters += ["hub/#", "hub/x", "+/x"]
        clients += [f"h{i}"] * 3
        subs += [(1, 0, 0, 0, i + 1), (0, 0, 0, 0, 0), (2, 0, 0, 0, 7)]
    filters += ["a/#", "a/b", "#"]
    clients += ["k", "k", "j"]
    subs += [(0, 0, 0, 0, 3), (1, 0, 0, 0, 4), (0, 0, 0, 0, 0)]
    deep = "/".join(f"d{i}" for i in range(20))
    for i in range(50):  # a 20-level topic: DFS
        filters += ["d0/#", "d0/d1/+/d3/#", deep]
        clients += [f"p{i}"] * 3
        subs += [(i % 3, 0, 0, 0, i + 1), (1, 1, 0, 0, 0), (2, 0, 1, 2, 5)]
    topics = ["hub/x", "hub", "a/b", "a/b/c", "zz/x", "$SYS/x", deep, deep + "/e"]
    monkeypatch.setenv("MQM_NO_FAST", "1")
    idx = maxmq_amd.TopicsIndex(0, identifiers=True)
    monkeypatch.delenv("MQM_NO_FAST")
    ora = OracleIndex()
    for f, c, (q, nl, rap, rh, ident) in zip(filters, clients, subs):
        idx.subscribe(c, maxmq_amd.Subscription(f, q, ident, bool(nl), bool(rap), rh))
        ora.subscribe(c, f, q, nl, rap, rh, ident)
    s = Strings.from_list(topics)
    res = idx.match_batch(s.data, s.offs)
    assert_same(canon_gpu_idents(res), canon_oracle_idents(*ora.identifiers(s.data, s.offs)), "identifiers")
    # device form over a device-resident batch: same per-topic counts
    import torch
    tb = torch.from_numpy(s.data).cuda()
    to = torch.from_numpy(s.offs.view(np.int64)).cuda()
    r = idx.match_device(tb.data_ptr(), to.data_ptr(), len(topics))
    assert r.n_fallback > 0
    d = idx.identifiers_device()
    torch.cuda.synchronize()
    assert d.n_topics == len(topics) and d.n_idents == int(res.ident_offsets[-1])


@pytest.mark.parametrize("config,overrides", [(3, dict(n_filters=40000, n_topics=30000)),
                                              (4, dict(n_filters=30000, n_topics=20000))])
def test_identifiers_beside_the_match_equal_after(config, overrides):
    """mqm_identifiers_early: the identifiers pass forked onto a side stream
    after the walk (overlapping the merges) lists exactly what the pass run
    after the match lists — offsets and sids, byte for byte — over several
    batches (the capacity it sizes from the last call grows in between), and
    the host path of an MQM_CFG_IDENTIFIERS index (which always runs it
    beside the match) still equals the oracle's maps."""
    import torch

    from maxmq_amd.devbuf import dev_view_copy

    w = mqgen.generate(config, **overrides)
    idx = maxmq_amd.TopicsIndex(0, identifiers=True)
    idx.subscribe_workload(w)
    idx.commit()
    dev = torch.device("cuda", 0)
    s = w.topics
    tb = torch.from_numpy(s.data).to(dev)
    to = torch.from_numpy(s.offs.view(np.int64)).to(dev)
    n = len(s)

    def run(early):
        idx.identifiers_early(early)
        idx.match_device(tb.data_ptr(), to.data_ptr(), n)
        d = idx.identifiers_device()
        offs = dev_view_copy(d.offsets, n + 1, torch.int64, dev).cpu().numpy()
        sids = dev_view_copy(d.sids, max(int(d.n_idents), 1), torch.int32, dev).cpu().numpy()[:int(d.n_idents)]
        torch.cuda.synchronize()
        return int(d.n_idents), offs, sids

    late = run(False)
    for _ in range(3):
        early = run(True)
        assert early[0] == late[0] and np.array_equal(early[1], late[1]) and np.array_equal(early[2], late[2])
    idx.identifiers_early(False)
    assert late[0] > 0
    ora = OracleIndex()
    ora.subscribe_workload(w)
    k = min(n, 4000)
    res = idx.match_batch(s.data[: int(s.offs[k])], s.offs[: k + 1])
    assert_same(canon_gpu_idents(res), canon_oracle_idents(*ora.identifiers(s.data[: int(s.offs[k])], s.offs[: k + 1])),
                "identifiers")


# ---- subscriber-sharded node result: mqm_dense_device + mqm_gather_shards ----------

@pytest.mark.parametrize("n_shards", [1, 3, 4])
def test_gather_shards_equals_unsharded(n_shards):
    """S shard indexes on one device (each a contiguous client range), their
    dense CSRs laid out by mqm_gather_shards == the unsharded index's result:
    same (topic, node client, QoS, NoLocal) rows, shard order within a topic."""
    import torch

    from maxmq_amd import shard

    w = mqgen.generate(1, n_filters=20000, n_topics=30000, p_shared=0.1)
    s = w.topics
    tb = torch.from_numpy(s.data).cuda()
    to = torch.from_numpy(s.offs.view(np.int64)).cuda()
    n = len(s)
    full = maxmq_amd.TopicsIndex(0)
    full.subscribe_workload(w)
    ref = full.match_batch(s.data, s.offs)
    idxs, parts, maps, total = [], [], [], 0
    sparts, stotal, shost = [], 0, []
    for r in range(n_shards):
        ix = maxmq_amd.TopicsIndex(0)
        ix.subscribe_workload(shard.shard_workload(w, n_shards, r))
        ix.match_device(tb.data_ptr(), to.data_ptr(), n)
        d = ix.dense_device()
        total += int(d.n_deliveries)
        stotal += int(d.n_shared)
        cm = torch.from_numpy(shard.client_map(w, n_shards, r).astype(np.int32)).cuda()
        idxs.append(ix)
        maps.append(cm)
        parts.append((d.offsets, d.deliveries, cm.data_ptr(), cm.numel()))
        sparts.append((d.shared_offsets, d.shared))
        shost.append(ix.match_batch(s.data, s.offs))  # resolves the shard's shared ids
    out_o = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    out_d = torch.zeros(max(total, 1), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    maxmq_amd.gather_shards(n, parts, out_o.data_ptr(), out_d.data_ptr())
    go = out_o.cpu().numpy().view(np.uint64)
    assert np.array_equal(go, ref.offsets), "node-wide offsets"
    gd = out_d[:total].cpu().numpy().view(capi.DELIVERY_DTYPE)
    _, gq, gn = capi.delivery_fields(gd["packed"])
    _, rq, rn = capi.delivery_fields(ref.deliveries["packed"])
    topic = np.repeat(np.arange(n), np.diff(go).astype(np.int64))
    g = np.unique(np.rec.fromarrays([topic, gd["client"], gq, gn]))
    r = np.unique(np.rec.fromarrays([topic, ref.deliveries["client"], rq, rn]))
    assert len(g) == total and np.array_equal(g, r)
    # shared candidates: shard-tagged, resolved on their shard == the unsharded set
    so = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    sd = torch.zeros(max(stotal, 1), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    maxmq_amd.gather_shards_shared(n, sparts, so.data_ptr(), sd.data_ptr())
    sov = so.cpu().numpy().view(np.uint64)
    assert np.array_equal(sov, ref.shared_offsets), "node-wide shared offsets"
    sdv = sd[:stotal].cpu().numpy().view(np.uint32)
    assert stotal > 0
    got = set()
    for t in range(n):
        for v in sdv[sov[t]:sov[t + 1]]:
            r, sid = int(v) >> 28, int(v) & 0x0FFFFFFF
            info = shost[r].shared_info(sid)
            got.add((t, idxs[r].filter_name(info.filter), idxs[r].client_name(info.client)))
    want = set()
    for t in range(n):
        for sid in ref.shared[ref.shared_offsets[t]:ref.shared_offsets[t + 1]]:
            info = ref.shared_info(int(sid))
            want.add((t, full.filter_name(info.filter), full.client_name(info.client)))
    assert got == want and len(got) == stotal
    # a client id outside its shard's map is an error, never silent
    bad = [(p[0], p[1], p[2], 0) for p in parts]
    if total:
        with pytest.raises(maxmq_amd.MqmError):
            maxmq_amd.gather_shards(n, bad, out_o.data_ptr(), out_d.data_ptr())


def test_full_size_c3_headline_config():
    """BASELINE configs[2], the config the headline is quoted on (10M filters,
    40% '+', 10% '#', Zipf(1.2) topics, 10M-topic batch), through the same
    mqm_match_device call bench.py times:
      * bit-exact against the oracle on a 100k-topic sample of the batch (the
        full-batch rows of those topics are compared with the host-path rows,
        which are compared with oracle/mochi_ref.c field by field);
      * over all 10M topics: dense CSR monotone and summing to n_deliveries,
        QoS <= 2, client ids in range, per-topic client uniqueness (on a 1M
        sample), run-to-run equality of every topic's checksum of its entries;
      * the merges ran (the hash-table tiers, or with MQM_RESOLVE=1 the merge by
        resolution: every C3 multi entry is light)."""
    import torch

    from tests.gpu_util import dev_tensor, topic_checksums

    w = mqgen.generate(3)
    n = len(w.topics)
    idx = maxmq_amd.TopicsIndex(0, autocommit=False)
    idx.subscribe_workload(w)
    idx.commit()
    dev = torch.device("cuda:0")
    tb = torch.from_numpy(w.topics.data).to(dev)
    to = torch.from_numpy(w.topics.offs.view(np.int64)).to(dev)

    def run():
        r = idx.match_device(tb.data_ptr(), to.data_ptr(), n)
        d = idx.dense_device()
        torch.cuda.synchronize()
        offs = dev_tensor(d.offsets, n + 1, torch.int64)
        ents = dev_tensor(d.deliveries, int(d.n_deliveries), torch.int64)
        sh_offs = dev_tensor(d.shared_offsets, n + 1, torch.int64)
        return r, offs, ents, sh_offs

    r1, offs, ents, sh_offs = run()
    nd = int(r1.n_deliveries)
    assert nd > 50 * n, nd  # Zipf fan-out: ~230 deliveries per topic
    assert r1.n_resolve + r1.n_big > 0, "no merge kernel ran"
    assert int(offs[0]) == 0 and int(offs[-1]) == nd
    assert bool((offs[1:] >= offs[:-1]).all())
    assert int(sh_offs[-1]) == int(r1.n_shared)
    clients = ents & 0xFFFFFFFF
    packed = (ents >> 32) & 0xFFFFFFFF
    assert int(clients.max()) < idx.num_clients()
    assert int(((packed >> 28) & 3).max()) <= 2
    sums1 = topic_checksums(offs, ents)
    del clients, packed
    # run-to-run: every topic's entries, as a set, identical
    _, offs2, ents2, _ = run()
    assert torch.equal(offs2, offs)
    assert torch.equal(topic_checksums(offs2, ents2), sums1)
    del offs2, ents2
    # per-topic client uniqueness on a 1M-topic sample (host)
    rng = np.random.default_rng(3)
    sample = np.sort(rng.choice(n, size=1000000, replace=False))
    o = offs.cpu().numpy()
    cnt = (o[sample + 1] - o[sample]).astype(np.int64)
    pos = torch.from_numpy(np.repeat(o[sample] - np.concatenate([[0], np.cumsum(cnt)[:-1]]), cnt)
                           + np.arange(cnt.sum())).to(dev)
    samp = ents[pos].cpu().numpy().view(np.uint64)
    tid = np.repeat(np.arange(len(sample), dtype=np.uint64), cnt)
    key = (tid << np.uint64(32)) | (samp & np.uint64(0xFFFFFFFF))
    assert len(np.unique(key)) == len(key), "a client appears twice in one topic"
    # bit-exact on a 100k-topic sample: full-batch rows == host-path rows == oracle
    small = np.sort(rng.choice(n, size=100000, replace=False))
    sub = Strings.from_list([w.topics[int(i)] for i in small])
    res = idx.match_batch(sub.data, sub.offs)
    cnt = (o[small + 1] - o[small]).astype(np.int64)
    assert np.array_equal(cnt, np.diff(res.offsets).astype(np.int64)), "per-topic counts differ from the host path"
    pos = torch.from_numpy(np.repeat(o[small] - np.concatenate([[0], np.cumsum(cnt)[:-1]]), cnt)
                           + np.arange(cnt.sum())).to(dev)
    full_rows = ents[pos].cpu().numpy().view(np.uint64)
    tid = np.repeat(np.arange(len(small), dtype=np.uint64), cnt)
    host_rows = res.deliveries.view(np.uint64)
    assert np.array_equal(np.unique(np.stack([tid, full_rows], 1), axis=0),
                          np.unique(np.stack([tid, host_rows], 1), axis=0)), "full-batch rows != host-path rows"
    ora = OracleIndex()
    ora.subscribe_workload(w)
    r, rs = canon_oracle(*ora.match(sub.data, sub.offs, nthreads=16)[:4])
    g, gs = canon_gpu(res)
    assert_same(g, r, "C3 deliveries (sample)")
    assert_same(gs, rs, "C3 shared (sample)")
