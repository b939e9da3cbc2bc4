"""MQM_CFG_FRESH: per-publish results follow every mutation at once.

The reference mutates its live trie under the root mutex and the next
Subscribers call sees the change (topics.go:303-321, 325-349, 484-518).  An
async index with MQM_CFG_FRESH matches the published snapshot and corrects
the result on the host for the clients a mutation touched since that snapshot
(maxmq_amd/csrc/fresh.h).  Here one thread interleaves random mutations —
new subscriptions, re-subscriptions with other QoS / flags / Identifiers,
unsubscriptions of live and absent pairs, shared subscriptions in both
"$SHARE" spellings, '+' / '#' filters under '$' topics, parent-'#' cases —
with calls, while the builder publishes a new snapshot every few dozen
mutations, so results are corrected against snapshots of every age the
overlay covers.  Every call must equal the oracle (oracle/mochi_ref.c) applied
to exactly the mutations made so far — rows, first filter, Identifier, RAP,
RH, the Identifiers maps and the shared pairs — and report the store's
current version."""

import random

import numpy as np
import pytest

import maxmq_amd
from oracle.binding import OracleIndex
from tests.gpu_util import assert_same, canon_gpu, canon_gpu_idents, canon_oracle, canon_oracle_idents
from tools import mqgen
from tools.mqgen import Strings

pytestmark = pytest.mark.gpu


def _records(n=3000, seed=7):
    w = mqgen.generate(1, n_filters=n, n_topics=600, n_clients=250, p_shared=0.05, seed=seed)
    recs = [(w.clients[i], w.filters[i], int(w.qos[i]), int(w.no_local[i]), int(w.rap[i]), int(w.rh[i]),
             int(w.ident[i])) for i in range(n)]
    # the corners: '$' topics against '+' / '#' first levels, both $SHARE
    # spellings of one group path, parent-'#' after a literal, empty levels
    recs += [("dollar", "+/x", 1, 0, 0, 0, 3), ("dollar", "#", 2, 1, 0, 1, 0), ("sys", "$SYS/#", 0, 0, 1, 2, 9),
             ("sh1", "$SHARE/g1/a/b", 1, 0, 0, 0, 4), ("sh1", "$share/g1/a/b", 2, 0, 0, 0, 5),
             ("sh2", "$SHARE/g2/a/+", 0, 0, 0, 0, 0), ("par", "a/b/#", 1, 0, 0, 0, 6), ("par", "a/+", 2, 1, 1, 0, 7),
             ("empty", "/x", 0, 0, 0, 0, 0), ("empty", "//", 1, 0, 0, 0, 2)]
    topics = [w.topics[i] for i in range(len(w.topics))] + ["$SYS/x", "$x", "a/b", "a/b/c", "/x", "//", "a", "x"]
    return recs, topics


def _check(idx, ora, topic, what):
    res = idx.subscribers_result(topic)
    s = Strings.from_list([topic])
    g, gs = canon_gpu(res)
    r, rs = canon_oracle(*ora.match(s.data, s.offs)[:4])
    assert_same(g, r, f"{what}: {topic!r}")
    assert_same(gs, rs, f"{what}: {topic!r} (shared)")
    assert_same(canon_gpu_idents(res), canon_oracle_idents(*ora.identifiers(s.data, s.offs)),
                f"{what}: {topic!r} (identifiers)")
    return res


@pytest.mark.parametrize("serve", [False, True])
def test_fresh_calls_follow_every_mutation(serve):
    recs, topics = _records()
    base, extra = recs[:2000], recs[2000:]
    idx = maxmq_amd.TopicsIndex(0, autocommit=False, identifiers=True, async_commit=True, serve=serve, fresh=True)
    ora = OracleIndex()
    for c, f, q, nl, rap, rh, ident in base:
        idx.subscribe(c, maxmq_amd.Subscription(f, q, ident, bool(nl), bool(rap), rh))
        ora.subscribe(c, f, q, bool(nl), bool(rap), rh, ident)
    idx.commit()
    idx.commit_policy(37, 0)  # a rebuild every 37 mutations: snapshots publish between the calls
    rnd = random.Random(0xF4E5)
    live = [(r[0], r[1]) for r in base]
    corrected = 0
    for step in range(500):
        for _ in range(rnd.randrange(1, 4)):
            x = rnd.random()
            if x < 0.35 and extra:
                c, f, q, nl, rap, rh, ident = extra.pop()
                live.append((c, f))
            elif x < 0.55 and live:
                c, f = live[rnd.randrange(len(live))]
                q, nl, rap, rh, ident = rnd.randrange(3), rnd.randrange(2), rnd.randrange(2), rnd.randrange(3), \
                    rnd.randrange(4)
            else:
                if x < 0.95 and live:
                    c, f = live.pop(rnd.randrange(len(live)))
                else:
                    c, f = "nobody", rnd.choice(["no/such/filter", "a/b", "$share/g1/a/b"])
                assert idx.unsubscribe(f, c) == ora.unsubscribe(f, c), (f, c)
                continue
            got = idx.subscribe(c, maxmq_amd.Subscription(f, q, ident, bool(nl), bool(rap), rh))
            assert got == ora.subscribe(c, f, q, bool(nl), bool(rap), rh, ident), (c, f)
        st = idx.commit_state()
        for _ in range(2):
            res = _check(idx, ora, rnd.choice(topics), f"step {step}")
            # read-your-writes: the result reflects the store as it is now
            assert res.snapshot_version == st["store_version"], (res.snapshot_version, st)
        corrected += st["snapshot_version"] < st["store_version"]
    # most calls ran ahead of the published snapshot (the overlay did the work)
    assert corrected > 250, corrected
    ora.close()


def test_fresh_off_keeps_the_snapshot_view():
    """Without the flag an async index answers from the published snapshot
    (the documented lag), so the overlay is what makes the difference."""
    recs, _ = _records(n=500, seed=3)
    idx = maxmq_amd.TopicsIndex(0, autocommit=False, async_commit=True)
    for c, f, q, nl, rap, rh, ident in recs[:400]:
        idx.subscribe(c, maxmq_amd.Subscription(f, q, ident, bool(nl), bool(rap), rh))
    idx.commit()
    v0 = idx.commit_state()["store_version"]
    idx.subscribe("late", maxmq_amd.Subscription("#", 1))
    res = idx.subscribers_result("some/topic")
    assert res.snapshot_version == v0
    clients = {idx.client_name(int(c)) for c in res.deliveries["client"]}
    assert "late" not in clients
    fresh = maxmq_amd.TopicsIndex(0, autocommit=False, async_commit=True, fresh=True)
    for c, f, q, nl, rap, rh, ident in recs[:400]:
        fresh.subscribe(c, maxmq_amd.Subscription(f, q, ident, bool(nl), bool(rap), rh))
    fresh.commit()
    fresh.subscribe("late", maxmq_amd.Subscription("#", 1))
    res = fresh.subscribers_result("some/topic")
    assert res.snapshot_version == fresh.commit_state()["store_version"]
    assert "late" in {fresh.client_name(int(c)) for c in res.deliveries["client"]}
    assert isinstance(np.asarray(res.deliveries), np.ndarray)
