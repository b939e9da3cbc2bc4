"""Incremental commits: the delta log, the background
builder's shadow store and double-buffered publishing.

CPU tests use host-only indexes (MQM_DEVICE_NONE), whose commits build the
host side of the snapshot: the builder's replay of the delta log must produce a
snapshot bit-identical (equal digest) to a synchronous flatten of the
authoritative store, whatever the interleaving of commits and mutations.  The
GPU tests check that matches read the front buffer while the back buffer is
built, and agree with the oracle once it is published."""

import random

import numpy as np
import pytest

import maxmq_amd
from maxmq_amd import capi
from oracle import mochi_ref as pyref

LEVELS = ["a", "b", "", "+", "#", "$SYS", "$SHARE", "$share", "g", "x" * 20]


def _random_op(rng, idx_list, step):
    f = "/".join(rng.choice(LEVELS) for _ in range(rng.randint(1, 4)))
    c = f"k{rng.randint(0, 5)}"
    r = rng.random()
    out = []
    for idx in idx_list:
        if r < 0.55:
            out.append(idx.subscribe(c, maxmq_amd.Subscription(f, qos=step % 3, identifier=step % 5)))
        elif r < 0.85:
            out.append(idx.unsubscribe(f, c))
        else:
            t = f.replace("+", "p").replace("#", "h")
            out.append(idx.retain_message(t, step, 4 if step % 3 else 0))
    return out


def test_async_requires_config():
    idx = maxmq_amd.TopicsIndex(device=None)
    with pytest.raises(maxmq_amd.MqmError) as e:
        idx.commit_async()
    assert e.value.rc == capi.MQM_EINVAL


def test_host_commit_builds_snapshot():
    idx = maxmq_amd.TopicsIndex(device=None)
    idx.subscribe("c", maxmq_amd.Subscription("a/+/c"))
    idx.commit()
    st = idx.snapshot_stats()
    assert st["subs"] == 1 and st["nodes"] == 4 and st["device_bytes"] == 0
    d0 = idx.snapshot_digest()
    idx.subscribe("d", maxmq_amd.Subscription("a/+/c"))
    assert idx.snapshot_digest() == d0  # not committed yet
    idx.commit()
    assert idx.snapshot_digest() != d0


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_builder_replay_equals_sync_flatten(seed):
    rng = random.Random(seed)
    sync = maxmq_amd.TopicsIndex(device=None, autocommit=False)
    asy = maxmq_amd.TopicsIndex(device=None, autocommit=False, async_commit=True)
    for step in range(1500):
        a, b = _random_op(rng, [sync, asy], step)
        assert a == b
        if step % 97 == 0:
            asy.commit_async()  # coalesced when builds overlap
        if step % 250 == 249:
            sync.commit()
            asy.commit_async()
            asy.commit_poll(wait=True)
            st = asy.commit_state()
            assert st["snapshot_version"] == st["store_version"] and st["pending_ops"] == 0
            assert asy.snapshot_digest() == sync.snapshot_digest(), step


def test_sync_commit_on_async_index_is_read_your_writes():
    idx = maxmq_amd.TopicsIndex(device=None, autocommit=False, async_commit=True)
    ref = maxmq_amd.TopicsIndex(device=None, autocommit=False)
    for i in range(200):
        for x in (idx, ref):
            x.subscribe(f"c{i % 7}", maxmq_amd.Subscription(f"t/{i % 13}/+"))
    idx.commit()
    ref.commit()
    assert idx.snapshot_digest() == ref.snapshot_digest()
    st = idx.commit_state()
    assert st["builds"] >= 1 and st["last_build_ms"] > 0


def test_commit_policy_auto_submits():
    idx = maxmq_amd.TopicsIndex(device=None, autocommit=False, async_commit=True)
    idx.commit_policy(max_ops=50)
    for i in range(120):
        idx.subscribe(f"c{i}", maxmq_amd.Subscription(f"p/{i}"))
    st = idx.commit_state()
    assert st["pending_ops"] == 20  # 2 logs of 50 submitted by the policy
    idx.commit_poll(wait=True)
    st = idx.commit_state()
    assert st["has_snapshot"] and st["snapshot_version"] == 100 and st["store_version"] == 120
    assert st["builds"] >= 1


def test_visibility_lag_is_reported():
    idx = maxmq_amd.TopicsIndex(device=None, autocommit=False, async_commit=True)
    idx.subscribe("c", maxmq_amd.Subscription("a"))
    idx.commit()
    d0 = idx.snapshot_digest()
    idx.subscribe("c", maxmq_amd.Subscription("b"))
    st = idx.commit_state()
    assert st["snapshot_version"] == 1 and st["store_version"] == 2 and st["pending_ops"] == 1
    assert idx.snapshot_digest() == d0
    idx.commit_async()
    idx.commit_poll(wait=True)
    assert idx.snapshot_digest() != d0


def test_unsubscribe_false_is_not_logged():
    """Unsubscribe of a missing node changes nothing (topics.go:334-336)."""
    idx = maxmq_amd.TopicsIndex(device=None, autocommit=False, async_commit=True)
    assert not idx.unsubscribe("nope/x", "c")
    assert idx.commit_state()["pending_ops"] == 0
    idx.subscribe("c", maxmq_amd.Subscription("a"))
    assert idx.unsubscribe("a", "other")  # node exists: true, logged
    assert idx.commit_state()["pending_ops"] == 2


# ---------------------------------------------------------------- GPU ------------


def _match_sets(idx, topics):
    from tools.mqgen import Strings

    s = Strings.from_list(topics)
    res = idx.match_batch(s.data, s.offs)
    out = []
    for i in range(len(topics)):
        lo, hi = res.offsets[i], res.offsets[i + 1]
        _, qos, _ = capi.delivery_fields(res.deliveries["packed"][lo:hi])
        out.append(sorted((idx.client_name(int(c)), int(q)) for c, q in zip(res.deliveries["client"][lo:hi], qos)))
    return out


def _py_sets(py, topics):
    return [sorted((k, v.qos) for k, v in py.subscribers(t)[0].items()) for t in topics]


@pytest.mark.gpu
def test_gpu_async_matches_front_buffer_then_published():
    rng = random.Random(11)
    idx = maxmq_amd.TopicsIndex(0, autocommit=False, async_commit=True)
    py_front = pyref.TopicsIndex()  # state of the published snapshot
    py_now = pyref.TopicsIndex()    # state of the store
    topics = ["/".join(rng.choice(["a", "b", "", "$SYS", "g"]) for _ in range(rng.randint(1, 5))) for _ in range(300)]
    ops = []
    for rnd in range(6):
        for step in range(150):
            f = "/".join(rng.choice(LEVELS[:5] + ["g"]) for _ in range(rng.randint(1, 4)))
            c = f"k{rng.randint(0, 9)}"
            q = rng.randint(0, 2)
            if rng.random() < 0.7:
                assert idx.subscribe(c, maxmq_amd.Subscription(f, q)) == py_now.subscribe(c, pyref.Sub(f, q))
                ops.append(("s", c, f, q))
            else:
                assert idx.unsubscribe(f, c) == py_now.unsubscribe(f, c)
                ops.append(("u", c, f, q))
        if rnd == 0:
            idx.commit()
        else:
            # a match while the back buffer is built reads the front buffer; a
            # match that finds the build finished publishes it first
            before = idx.commit_state()["builds"]
            idx.commit_async()
            got = _match_sets(idx, topics)
            published = idx.commit_state()["builds"] > before
            assert got == _py_sets(py_now if published else py_front, topics), (rnd, published)
            idx.commit_poll(wait=True)
        for op in ops:
            if op[0] == "s":
                py_front.subscribe(op[1], pyref.Sub(op[2], op[3]))
            else:
                py_front.unsubscribe(op[2], op[1])
        ops = []
        assert _match_sets(idx, topics) == _py_sets(py_now, topics), rnd


@pytest.mark.gpu
def test_gpu_async_no_publish_without_poll():
    """Without a poll or a match, a finished build is not published; without
    a commit, mutations stay invisible (the documented visibility lag)."""
    idx = maxmq_amd.TopicsIndex(0, autocommit=False, async_commit=True)
    idx.subscribe("c1", maxmq_amd.Subscription("a/+"))
    idx.commit()
    assert _match_sets(idx, ["a/b"]) == [[("c1", 0)]]
    idx.subscribe("c2", maxmq_amd.Subscription("a/b", qos=2))
    assert _match_sets(idx, ["a/b"]) == [[("c1", 0)]]  # not committed: front buffer
    idx.commit_async()
    idx.commit_poll(wait=True)
    assert _match_sets(idx, ["a/b"]) == [[("c1", 0), ("c2", 2)]]
    d = idx.snapshot_digest()
    ref = maxmq_amd.TopicsIndex(0)
    ref.subscribe("c1", maxmq_amd.Subscription("a/+"))
    ref.subscribe("c2", maxmq_amd.Subscription("a/b", qos=2))
    ref.commit()
    assert ref.snapshot_digest() == d
    assert np.uint64(d) != 0


def test_unsubscribe_many_matches_single_calls():
    from tools.mqgen import Strings

    rng = random.Random(5)
    a = maxmq_amd.TopicsIndex(device=None, autocommit=False, async_commit=True)
    b = maxmq_amd.TopicsIndex(device=None, autocommit=False)
    pairs = [("/".join(rng.choice(LEVELS) for _ in range(rng.randint(1, 3))), f"k{rng.randint(0, 3)}")
             for _ in range(300)]
    for f, c in pairs:
        a.subscribe(c, maxmq_amd.Subscription(f))
        b.subscribe(c, maxmq_amd.Subscription(f))
    rng.shuffle(pairs)
    got = a.unsubscribe_many(Strings.from_list([f for f, _ in pairs]), Strings.from_list([c for _, c in pairs]))
    want = [b.unsubscribe(f, c) for f, c in pairs]
    assert got.tolist() == [int(x) for x in want]
    a.commit()
    b.commit()
    assert a.snapshot_digest() == b.snapshot_digest()


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_failed_build_is_reported_then_rebuilt(stage):
    """a failed background build (replay part-way, flatten, upload)
    must not leave a stale snapshot published as current.  The commit that
    waits for it reports the error or repairs it at once; the following
    commit publishes a snapshot equal to a synchronous flatten of the store."""
    rng = random.Random(40 + stage)
    sync = maxmq_amd.TopicsIndex(device=None, autocommit=False)
    asy = maxmq_amd.TopicsIndex(device=None, autocommit=False, async_commit=True)
    for step in range(300):
        _random_op(rng, [sync, asy], step)
    asy.commit()
    sync.commit()
    assert asy.snapshot_digest() == sync.snapshot_digest()
    for step in range(300, 600):
        _random_op(rng, [sync, asy], step)
    sync.commit()
    check = capi.check
    check("mqm_debug_fault", capi.lib().mqm_debug_fault(asy._h, stage, 1))
    asy.commit_async()
    try:
        asy.commit()  # a replay fault is repaired inside this commit (full resync)
    except maxmq_amd.MqmError as e:
        assert stage != 1 and e.rc == capi.MQM_ENOMEM
        st = asy.commit_state()
        assert st["snapshot_version"] != st["store_version"]  # the stale snapshot is not claimed current
        asy.commit()
    st = asy.commit_state()
    assert st["snapshot_version"] == st["store_version"]
    assert asy.snapshot_digest() == sync.snapshot_digest()
    # and the shadow store stays in step afterwards
    for step in range(600, 700):
        _random_op(rng, [sync, asy], step)
    sync.commit()
    asy.commit()
    assert asy.snapshot_digest() == sync.snapshot_digest()


def test_replay_fault_while_logs_queue():
    """a replay fault with more logs submitted behind it: the stale shadow
    refuses them, and the next commit resyncs from a full copy"""
    rng = random.Random(77)
    sync = maxmq_amd.TopicsIndex(device=None, autocommit=False)
    asy = maxmq_amd.TopicsIndex(device=None, autocommit=False, async_commit=True)
    capi.check("mqm_debug_fault", capi.lib().mqm_debug_fault(asy._h, 1, 2))
    for step in range(400):
        _random_op(rng, [sync, asy], step)
        if step % 50 == 49:
            asy.commit_async()
    sync.commit()
    try:
        asy.commit()
    except maxmq_amd.MqmError:
        asy.commit()
    assert asy.snapshot_digest() == sync.snapshot_digest()


def test_solo_marking_of_hash_nodes():
    """kFlagParentLit (snapshot.h): a '#' node whose parent has a literal key is
    gathered once per topic by the walks (the parent-'#' probe, topics.go:507-509;
    its own visit is skipped), so its subscription is solo unless the client has
    a level-compatible partner.  "a/#" alone: solo; "+/#" alone: solo (no parent
    probe after '+'); "x/y" with "x/#" (one client, compatible): both multi."""
    idx = maxmq_amd.TopicsIndex(device=None)
    idx.subscribe("c1", maxmq_amd.Subscription("a/#"))
    idx.subscribe("c2", maxmq_amd.Subscription("+/#"))
    idx.subscribe("c3", maxmq_amd.Subscription("x/y"))
    idx.subscribe("c3", maxmq_amd.Subscription("x/#"))
    idx.commit()
    assert idx.snapshot_stats()["solo_subs"] == 2


def _kept_shape(idx):
    import ctypes as C
    ms = (C.c_double * 5)()
    capi.check("mqm_build_phases_ms", capi.lib().mqm_build_phases_ms(idx._h, ms))
    return bool(ms[4])


def test_rebuild_keeps_the_trie_shape_when_no_node_moves():
    """FlattenCache (flatten.h): a background build after Subscribe /
    Unsubscribe calls that create or remove no node reuses the previous
    build's preorder and edge list (refreshing the edges' inline child
    descriptors) — and must still equal a full flatten of the store, byte
    for byte; a call that creates a node (a new filter) or removes one (the
    last subscriber of a leaf) forces the full path."""
    from tools import mqgen

    w = mqgen.generate(1, n_filters=4000, n_topics=10)
    rng = random.Random(11)
    sync = maxmq_amd.TopicsIndex(device=None, autocommit=False)
    asy = maxmq_amd.TopicsIndex(device=None, autocommit=False, async_commit=True)
    for idx in (sync, asy):
        idx.subscribe_workload(w)
        idx.commit()
    filters = [w.filters[i] for i in range(len(w.filters))]
    kept = []
    for rnd in range(6):
        for k in range(200):  # existing filters, new clients (and some of them leaving again)
            f = rng.choice(filters)
            c = f"churn-{rnd}-{k % 50}"
            for idx in (sync, asy):
                if k % 3 == 2:
                    idx.unsubscribe(f, c)
                else:
                    idx.subscribe(c, maxmq_amd.Subscription(f, qos=k % 3, identifier=k % 4))
        if rnd == 3:  # a new filter: new nodes
            for idx in (sync, asy):
                idx.subscribe("newcomer", maxmq_amd.Subscription(f"zz/{rnd}/+/leaf"))
        if rnd == 4:  # its only subscriber leaves: the nodes go again
            for idx in (sync, asy):
                idx.unsubscribe(f"zz/3/+/leaf", "newcomer")
        sync.commit()
        asy.commit()
        assert asy.snapshot_digest() == sync.snapshot_digest(), rnd
        kept.append(_kept_shape(asy))
    assert kept == [True, True, True, False, False, True], kept


def test_flatten_layout_independent_of_thread_count():
    """The flatten's children lists (a binned counting sort over the node
    array), preorder, edge staging and client grouping are laid out by store
    ids and fixed chunk counts, never by thread timing: the same store state
    flattened on 1, 3 and 8 host threads gives one digest.  The op sequence
    removes nodes and re-creates others, so store ids are reused from the free
    list and are not in creation order; retained messages add the reverse
    index (its groups sorted by parent)."""
    rng = random.Random(7)
    ops = []
    for step in range(3000):
        f = "/".join(rng.choice(LEVELS[:5] + ["m", "n", "o"]) for _ in range(rng.randint(1, 5)))
        ops.append((rng.random(), f, f"c{rng.randint(0, 40)}", step))
    digests = []
    try:
        for threads in (1, 3, 8):
            capi.check("mqm_build_threads", capi.lib().mqm_build_threads(threads))
            idx = maxmq_amd.TopicsIndex(device=None, autocommit=False)
            for r, f, c, step in ops:
                if r < 0.6:
                    idx.subscribe(c, maxmq_amd.Subscription(f, qos=step % 3, identifier=step % 4))
                elif r < 0.9:
                    idx.unsubscribe(f, c)
                else:
                    idx.retain_message(f.replace("+", "p").replace("#", "h"), step, 3)
            idx.commit()
            digests.append(idx.snapshot_digest())
    finally:
        capi.lib().mqm_build_threads(0)
    assert digests[0] == digests[1] == digests[2]
