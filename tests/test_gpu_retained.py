"""GPU parity of the retained reverse match (TopicsIndex.Messages,
vendor/github.com/mochi-co/mqtt/v2/topics.go:426-480): the HIP path through
the C ABI against the hand-derived known-answer table and the C oracle
(oracle/mochi_ref.c scan_messages) on the same seeded inputs.  Bit-exact on
the sorted set of message refs per filter (the reference returns Go map
iteration order, so order within a filter is not part of parity)."""

import random

import numpy as np
import pytest

import maxmq_amd
from oracle.binding import OracleIndex
from tools import mqgen
from tools.mqgen import Strings

pytestmark = pytest.mark.gpu


def _per_filter_sets(offs, refs):
    return [sorted(int(x) for x in refs[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1)]


def _both(retained, filters, subs=(), deletes=()):
    """retained: topics (ref = index); subs: (client, filter) also in the trie;
    deletes: topics retained then deleted again (payload 0)."""
    idx = maxmq_amd.TopicsIndex(0)
    ora = OracleIndex()
    for c, f in subs:
        idx.subscribe(c, maxmq_amd.Subscription(f, 1))
        ora.subscribe(c, f, 1)
    for i, t in enumerate(retained):
        assert idx.retain_message(t, i, 5) == ora.retain_message(t, i, 5)
    for t in deletes:
        assert idx.retain_message(t, 0, 0) == ora.retain_message(t, 0, 0)
    s = Strings.from_list(filters)
    g = _per_filter_sets(*idx.messages_batch(s.data, s.offs))
    r = _per_filter_sets(*ora.messages(s.data, s.offs))
    return g, r, idx


def test_kat_reverse(kat):
    topics = kat["retained_topics"]
    idx = maxmq_amd.TopicsIndex(0)
    for i, t in enumerate(topics):
        assert idx.retain_message(t, i, 3) == 1
    for case in kat["reverse"]:
        got = sorted(topics[i] for i in idx.messages(case["filter"]))
        assert got == sorted(case["topics"]), case


def test_quirks_vs_oracle():
    retained = ["a", "a/b", "a/b/c", "$SYS/x", "$SYS", "$foo/x", "b", "/x", "//", "a//b", "x" * 40 + "/y",
                "$SYS/a/b", "c/d/e/f/g/h/i/j/k", ""]
    filters = ["#", "+", "+/+", "+/#", "a/#", "a/+", "a/+/+", "#/b", "+/b", "$SYS/#", "$SYS/+", "$SYS", "a",
               "a/b/c/d", "a//b", "+//+", "//", "/+", "x" * 40 + "/+", "x" * 40 + "/y", "c/+/e/#", "c/#",
               "a/+/c/#", "", "zz", "zz/#", "+/zz", "a/#/c"]
    subs = [("k1", "a/+"), ("k2", "a/#"), ("k3", "+/x/#"), ("k4", "q/r")]
    g, r, _ = _both(retained, filters, subs)
    assert g == r
    # the "" quirk: literal-final wildcard filters return the message at "" for non-retained nodes
    assert any(len(x) for x in g)


def test_deletes_and_empty_topic_retained():
    retained = ["a/b", "a/c", "", "d"]
    g, r, idx = _both(retained, ["a/+", "+/b", "a/#", "d", "+", "#"], deletes=["a/c", "zzz"])
    assert g == r
    assert idx.retained_len() == 3


def test_config5_vs_oracle():
    w = mqgen.generate(5, n_filters=30000, n_topics=200000)
    idx = maxmq_amd.TopicsIndex(0)
    ora = OracleIndex()
    refs = np.arange(len(w.topics), dtype=np.uint64) * 7 + 3
    res = idx.retain_many(w.topics, refs)
    for i in range(len(w.topics)):  # the oracle store has no bulk call; same sequence
        ora.retain_message(w.topics[i], int(refs[i]), 1)
    assert (res >= 0).all()
    assert idx.retained_len() == ora.retained_len()
    f = w.filters
    go, gr = idx.messages_batch(f.data, f.offs)
    ro, rr = ora.messages(f.data, f.offs, nthreads=16)
    assert np.array_equal(go, ro), "per-filter counts differ"
    assert gr.sum() == rr.sum()
    assert _per_filter_sets(go, gr) == _per_filter_sets(ro, rr)
    assert go[-1] > 0


def test_random_retain_ops():
    rng = random.Random(7)
    lv = ["a", "b", "", "$SYS", "$x", "c" * 17]
    idx = maxmq_amd.TopicsIndex(0)
    ora = OracleIndex()
    for step in range(600):
        t = "/".join(rng.choice(lv) for _ in range(rng.randint(1, 4)))
        pl = 0 if rng.random() < 0.3 else 4
        assert idx.retain_message(t, step, pl) == ora.retain_message(t, step, pl), (step, t)
        if step % 100 == 99:
            filters = ["/".join(rng.choice(lv + ["+", "#"]) for _ in range(rng.randint(1, 4))) for _ in range(80)]
            s = Strings.from_list(filters)
            assert _per_filter_sets(*idx.messages_batch(s.data, s.offs)) == \
                _per_filter_sets(*ora.messages(s.data, s.offs)), step
