"""MQM_CFG_SERVE: single-topic Subscribers(topic) calls (the reference's
per-publish call shape, server.go:776, one goroutine per connection,
listeners/tcp.go:83) answered by the persistent GPU server (fast.hip k_serve)
through a ring of pinned slots.  Every caller's result must equal the same
topic's row of a plain batched match (deliveries, shared candidates,
Identifiers support), including:
  * 16 / 64 concurrent callers (more callers than ring slots are in flight
    over the run, so slots are reused);
  * topics whose results do not fit a slot, and topics longer than a slot
    (both take the batch path: counted as fallbacks);
  * the server exiting after its idle timeout and being relaunched by the
    next call, and a snapshot published between calls (Subscribe with
    autocommit: the server is relaunched on the new snapshot).
Every server launch ends with the index (stop word) or its idle timeout, so no
grid outlives the test."""

import ctypes as C
import threading
import time

import numpy as np
import pytest

import maxmq_amd
from maxmq_amd import capi
from tests.test_gpu_batching import _rows
from tools import mqgen

pytestmark = pytest.mark.gpu


def _one(idx, topic: bytes):
    L = capi.lib()
    h = C.c_void_p()
    capi.check("mqm_subscribers", L.mqm_subscribers(idx._h, topic, len(topic), C.byref(h)))
    r = maxmq_amd.BatchResult(idx, h)
    try:
        assert r.n == 1
        return _rows(r)[0]
    finally:
        r.close()


@pytest.mark.parametrize("threads,identifiers", [(16, False), (64, True)])
def test_served_subscribers_concurrent_equal_plain(threads, identifiers, monkeypatch):
    w = mqgen.generate(1, n_filters=20000, n_topics=3000, p_shared=0.05)
    monkeypatch.setenv("MQM_NO_FAST", "1")
    plain = maxmq_amd.TopicsIndex(device=0, identifiers=identifiers)
    monkeypatch.delenv("MQM_NO_FAST")
    plain.subscribe_workload(w)
    plain.commit()
    want = _rows(plain.match_batch(w.topics.data, w.topics.offs))
    plain.close()

    idx = maxmq_amd.TopicsIndex(device=0, identifiers=identifiers, serve=True)
    idx.subscribe_workload(w)
    idx.commit()
    n = len(w.topics)
    got = [None] * n
    errors = []

    def worker(k):
        try:
            for i in range(k, n, threads):
                got[i] = _one(idx, bytes(w.topics.data[int(w.topics.offs[i]):int(w.topics.offs[i + 1])]))
        except Exception as e:  # surfaced below
            errors.append(e)

    ths = [threading.Thread(target=worker, args=(k,)) for k in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    served, fallbacks, launches = idx.serve_stats()
    cnt = idx.serve_counters()
    idx.close()
    assert not errors, errors[0]
    # no safety net fired (a forced relaunch or a timed-out slot would hide a
    # lost request behind a correct fallback result)
    assert cnt["forced"] == 0 and cnt["slot_timeouts"] == 0 and cnt["result_timeouts"] == 0, cnt
    assert served + fallbacks == n and served > 0.9 * n, (served, fallbacks)
    assert launches >= 1
    bad = [i for i in range(n) if got[i] != want[i]]
    assert not bad, f"{len(bad)} topics differ, first {bad[0]}: {got[bad[0]]} vs {want[bad[0]]}"


def test_served_fallbacks_idle_relaunch_and_new_snapshot():
    idx = maxmq_amd.TopicsIndex(device=0, serve=True)
    idx.serve_policy(8, 2000)  # 8 workgroups, exit after 2 ms idle
    ref = maxmq_amd.TopicsIndex(device=0)
    for c in range(6000):  # one topic with 6000 deliveries: past a slot (4096)
        for x in (idx, ref):
            x.subscribe(f"c{c}", maxmq_amd.Subscription("big/#", c % 3))
    for x in (idx, ref):
        x.subscribe("a", maxmq_amd.Subscription("a/+", 1))
        x.subscribe("b", maxmq_amd.Subscription("a/b", 2))
        x.subscribe("h", maxmq_amd.Subscription("#", 1))  # not for '$' topics (topics.go:527)
    long_topic = "a/" + "x" * 2000  # longer than a slot's topic bytes
    # around the 48 topic bytes that ride in the slot's polled line (ServeSlot
    # line 0): empty, 47 / 48 / 49 bytes, and a '$' topic
    edge = [b"", b"a/" + b"y" * 45, b"a/" + b"y" * 46, b"a/" + b"y" * 47, b"$SYS/a"]
    topics = [b"big/q", b"a/b", long_topic.encode(), b"zzz"] + edge

    def check_all():
        for t in topics:
            r = ref.match_batch(np.frombuffer(t, np.uint8), np.array([0, len(t)], np.uint64))
            assert _one(idx, t) == _rows(r)[0], t

    check_all()
    served, fallbacks, launches = idx.serve_stats()
    assert fallbacks == 2 and served == 2 + len(edge), (served, fallbacks)
    time.sleep(0.05)  # the server exits idle; the next call relaunches it
    check_all()
    assert idx.serve_stats()[2] >= 2, idx.serve_stats()
    # a new snapshot between calls (autocommit): the server follows it
    for x in (idx, ref):
        x.subscribe("d", maxmq_amd.Subscription("a/#", 1))
    check_all()
    cnt = idx.serve_counters()
    idx.close()
    assert cnt["forced"] == 0 and cnt["slot_timeouts"] == 0 and cnt["result_timeouts"] == 0, cnt
    ref.close()
