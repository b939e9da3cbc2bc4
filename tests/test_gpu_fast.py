"""The small-batch path (maxmq_amd/csrc/fast.hip): Subscribers for batches of
up to kFastMaxTopics topics in one launch — the per-publish call shape
(server.go:776).  Bit-exact against the C oracle and against the batch
pipeline (the same index built with MQM_NO_FAST=1) on the same topics:
deliveries (client, max QoS, NoLocal, first filter, its identifier, RAP, RH)
and shared candidates.  Also the cases the path handles differently from the
batch pipeline: partitioned merges (more multi entries than one LDS table
holds), result blocks regrown after an overflow, and topics past its
capacities (the batch then takes the pipeline)."""

import numpy as np
import pytest

import maxmq_amd
from oracle.binding import OracleIndex
from tests.gpu_util import assert_same, canon_gpu, canon_gpu_idents, canon_oracle, canon_oracle_idents
from tools import mqgen
from tools.mqgen import Strings

pytestmark = pytest.mark.gpu


def _pair(monkeypatch, subscribe):
    monkeypatch.setenv("MQM_NO_FAST", "1")
    pipe = maxmq_amd.TopicsIndex(0)
    monkeypatch.delenv("MQM_NO_FAST")
    fast = maxmq_amd.TopicsIndex(0)
    ora = OracleIndex()
    for idx in (pipe, fast):
        subscribe(idx, None)
    subscribe(None, ora)
    return fast, pipe, ora


def _check(fast, pipe, ora, topics, what):
    s = topics if isinstance(topics, Strings) else Strings.from_list(topics)
    g, gs = canon_gpu(fast.match_batch(s.data, s.offs))
    p, ps = canon_gpu(pipe.match_batch(s.data, s.offs))
    r, rs = canon_oracle(*ora.match(s.data, s.offs, nthreads=8)[:4])
    assert_same(g, r, f"{what}: fast vs oracle")
    assert_same(gs, rs, f"{what}: fast vs oracle (shared)")
    assert_same(p, r, f"{what}: pipeline vs oracle")
    assert_same(ps, rs, f"{what}: pipeline vs oracle (shared)")
    return len(g)


@pytest.mark.parametrize("config,overrides", [(1, {"p_shared": 0.05}), (3, {"n_filters": 300000, "n_topics": 20000})])
def test_fast_batches_vs_oracle_and_pipeline(monkeypatch, config, overrides):
    w = mqgen.generate(config, **overrides)

    def sub(idx, ora):
        if idx is not None:
            idx.subscribe_workload(w)
        else:
            ora.subscribe_workload(w)

    fast, pipe, ora = _pair(monkeypatch, sub)
    rng = np.random.default_rng(config)
    n = len(w.topics)
    total = 0
    for size in (1, 2, 7, 64, 333, 1000, 4096):
        pick = rng.choice(n, size=min(size, n), replace=False)
        total += _check(fast, pipe, ora, Strings.from_list([w.topics[int(i)] for i in pick]), f"batch of {size}")
    assert total > 1000
    # the 4-B packed form: the same rows once each client is resolved
    for size in (5, 4096, min(n, 20000)):
        pick = rng.choice(n, size=size, replace=False)
        sub = Strings.from_list([w.topics[int(i)] for i in pick])
        g, gs = canon_gpu(fast.match_batch_packed(sub.data, sub.offs))
        r, rs = canon_oracle(*ora.match(sub.data, sub.offs, nthreads=8)[:4])
        assert_same(g, r, f"packed batch of {size}")
        assert_same(gs, rs, f"packed batch of {size} (shared)")
    # single-topic calls (mqm_subscribers, the reference's per-publish shape)
    for i in rng.choice(n, size=50, replace=False):
        t = w.topics[int(i)]
        a, b = fast.subscribers(t), pipe.subscribers(t)
        assert a.subscriptions == b.subscriptions and a.shared == b.shared, t


def test_fast_partitioned_merge_and_overflow_regrowth(monkeypatch):
    """2500 clients each with 3 filters that all match "a/b/c" (7500 multi
    entries: five merge passes), 120k solo subscribers of "x/#" (past the
    first result block: the call regrows it and runs again), and QoS / NoLocal
    / identifiers that differ between a client's filters (max QoS, NoLocal OR,
    first-merged = the lowest rank)."""
    def sub(idx, ora):
        def s(c, f, q, nl=0, ident=0):
            if idx is not None:
                idx.subscribe(c, maxmq_amd.Subscription(f, q, ident, bool(nl)))
            else:
                ora.subscribe(c, f, q, nl, 0, 0, ident)
        for i in range(2500):
            s(f"m{i}", "a/+/c", i % 3, 0, i + 1)
            s(f"m{i}", "a/#", (i + 1) % 3, i % 2)
            s(f"m{i}", "+/b/#", (i + 2) % 3, 0, 7)
        for i in range(120000):
            s(f"x{i}", "x/#", i % 3)
        s("sh", "$SHARE/g/a/+/c", 1)

    fast, pipe, ora = _pair(monkeypatch, sub)
    n = _check(fast, pipe, ora, ["a/b/c", "x/y", "a/b", "x", "a/b/c/d"], "partitioned merge + overflow")
    assert n > 120000 + 2500
    # the same again on the grown blocks, then a small batch on them
    _check(fast, pipe, ora, ["x/y", "a/b/c"] * 3, "again")
    _check(fast, pipe, ora, ["a/q/c"], "small after large")


def test_fast_capacity_fallback(monkeypatch):
    """Topics past the path's capacities in a small batch — 1500 bytes, 40
    levels, a frontier wider than a level's item list (300 nodes with '+'
    children under one '+' level) — take the batch pipeline; the results stay
    exact, and the batch around them too."""
    long_tok = "t" * 1400
    deep = "/".join(["d"] * 40)

    def sub(idx, ora):
        def s(c, f, q=1):
            if idx is not None:
                idx.subscribe(c, maxmq_amd.Subscription(f, q))
            else:
                ora.subscribe(c, f, q, 0, 0, 0, 0)
        s("a", long_tok + "/#")
        s("b", "d/#")
        s("c", deep)
        for i in range(300):
            s(f"w{i}", f"k{i}/+/+/z")
            s(f"v{i}", f"k{i}/#", 2)
        s("e", "+/+/+/z")

    fast, pipe, ora = _pair(monkeypatch, sub)
    topics = [long_tok + "/x", deep, "d/e", "q/r/s/z"] + [f"k{i}/a/b/z" for i in range(0, 300, 37)]
    _check(fast, pipe, ora, topics, "capacity fallback")
    # a topic level that is '+' or '#' (a topic the broker would refuse) and "" and "$SYS/x"
    _check(fast, pipe, ora, ["", "+/a/b/z", "#", "$SYS/x", "/", "//"], "odd topics")


def test_fast_identifiers_vs_oracle(monkeypatch):
    """MQM_CFG_IDENTIFIERS (the Go shim's configuration) on the small-batch
    path: every delivery's full Identifiers map (packets.go:250-259) equals the
    oracle's, and the batch pipeline's on the same index built with
    MQM_NO_FAST=1."""
    w = mqgen.generate(1, n_filters=20000, n_topics=5000, p_shared=0.05)
    monkeypatch.setenv("MQM_NO_FAST", "1")
    pipe = maxmq_amd.TopicsIndex(0, identifiers=True)
    monkeypatch.delenv("MQM_NO_FAST")
    fast = maxmq_amd.TopicsIndex(0, identifiers=True)
    ora = OracleIndex()
    for idx in (pipe, fast):
        idx.subscribe_workload(w)
    ora.subscribe_workload(w)
    for lo, hi in ((0, 1), (1, 65), (65, 4096)):
        s = Strings.from_list([w.topics[i] for i in range(lo, hi)])
        g = canon_gpu_idents(fast.match_batch(s.data, s.offs))
        p = canon_gpu_idents(pipe.match_batch(s.data, s.offs))
        r = canon_oracle_idents(*ora.identifiers(s.data, s.offs, nthreads=8))
        assert np.array_equal(g, r), f"topics [{lo}, {hi}): fast vs oracle identifiers"
        assert np.array_equal(p, r), f"topics [{lo}, {hi}): pipeline vs oracle identifiers"
