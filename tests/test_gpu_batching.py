"""MQM_CFG_BATCHING: concurrent single-topic Subscribers(topic) calls — the
reference's call shape, one goroutine per connection (listeners/tcp.go:83,
server.go:776) — gathered by the collector thread into GPU batches.  Every
caller's single-topic result must equal the same topic's row of a plain
batched match (deliveries, shared candidates, Identifiers support), and the
collector must actually have batched (fewer batches than calls)."""

import ctypes as C
import threading

import numpy as np
import pytest

import maxmq_amd
from maxmq_amd import capi
from tools import mqgen


def _rows(res):
    """per topic: sorted deliveries, sorted shared candidates, and every
    delivery's Identifiers map (packets.go:250-259) — the maps, not the listed
    sids: the batch pipeline lists only the identified entries of clients with
    several gathered subscriptions (a solo delivery's map is its first pair),
    the per-publish paths list every identified entry (include/mqmatch.h)"""
    out = []
    for i in range(res.n):
        d = res.deliveries[int(res.offsets[i]):int(res.offsets[i + 1])]
        s = res.shared[int(res.shared_offsets[i]):int(res.shared_offsets[i + 1])]
        ids = () if res.idents is None else tuple(sorted(
            (c, tuple(sorted(m.items()))) for c, m in res.identifiers(i).items()))
        out.append((tuple(sorted((int(c), int(p)) for c, p in zip(d["client"], d["packed"]))),
                    tuple(sorted(int(x) for x in s)), ids))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("threads,identifiers,linger_us", [(16, True, 0), (16, False, 0), (32, False, 300)])
def test_batched_subscribers_concurrent_equal_plain(threads, identifiers, linger_us, monkeypatch):
    """identifiers=False: batches take the small-batch path (fast.hip);
    identifiers=True: mqm_match_batch.  `plain` is the batch pipeline
    (MQM_NO_FAST=1) in both cases.  linger_us > 0 with the collector's
    several workers: two workers can wait out the linger on one queue and the
    first takes it all (the other must not run an empty batch)."""
    w = mqgen.generate(1, n_filters=20000, n_topics=3200, p_shared=0.05)
    monkeypatch.setenv("MQM_NO_FAST", "1")
    plain = maxmq_amd.TopicsIndex(device=0, identifiers=identifiers)
    monkeypatch.delenv("MQM_NO_FAST")
    plain.subscribe_workload(w)
    plain.commit()
    want = _rows(plain.match_batch(w.topics.data, w.topics.offs))
    plain.close()

    idx = maxmq_amd.TopicsIndex(device=0, identifiers=identifiers, batching=True)
    if linger_us:
        idx.batching_policy(0, linger_us)
    idx.subscribe_workload(w)
    idx.commit()
    L = capi.lib()
    n = len(w.topics)
    got = [None] * n
    errors = []

    def worker(k):
        try:
            for i in range(k, n, threads):
                t = bytes(w.topics.data[int(w.topics.offs[i]):int(w.topics.offs[i + 1])])
                h = C.c_void_p()
                capi.check("mqm_subscribers", L.mqm_subscribers(idx._h, t, len(t), C.byref(h)))
                r = maxmq_amd.BatchResult(idx, h)
                try:
                    assert r.n == 1
                    got[i] = _rows(r)[0]
                finally:
                    r.close()
        except Exception as e:  # surfaced below
            errors.append(e)

    ths = [threading.Thread(target=worker, args=(k,)) for k in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[0]
    batches, topics = idx.batching_stats()
    idx.close()
    assert topics == n
    assert batches < n, "the collector never gathered more than one call"
    bad = [i for i in range(n) if got[i] != want[i]]
    assert not bad, f"{len(bad)} topics differ, first {bad[0]}: {got[bad[0]]} vs {want[bad[0]]}"


@pytest.mark.gpu
def test_batching_policy_and_single_caller():
    w = mqgen.generate(1, n_filters=2000, n_topics=50)
    idx = maxmq_amd.TopicsIndex(device=0, batching=True)
    idx.subscribe_workload(w)
    idx.commit()
    idx.batching_policy(max_batch=4, linger_us=200)
    for i in range(10):
        t = bytes(w.topics.data[int(w.topics.offs[i]):int(w.topics.offs[i + 1])]).decode()
        idx.subscribers(t)
    b, t = idx.batching_stats()
    assert (b, t) == (10, 10)  # one caller: one topic per batch, whatever the linger
    idx.close()


def test_batching_api_refused_without_flag():
    idx = maxmq_amd.TopicsIndex(device=None)
    with pytest.raises(capi.MqmError):
        idx.batching_stats()
    with pytest.raises(capi.MqmError):
        idx.batching_policy(8, 0)
    idx.close()
