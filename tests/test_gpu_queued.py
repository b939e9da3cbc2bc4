"""The queued device API (mqm_match_device_async / mqm_match_ctx_wait) and the
batch pipeline's queued calls (match.hip match_enqueue: after a workspace's
first batch, no host read-back before the end; outputs sized by earlier
batches, every store checked, a batch that outgrows them re-run exactly).
Every result must equal the synchronous mqm_match_device result of the same
batch, per topic (as sets), including:
  * several contexts on two streams with batches queued back to back;
  * a context sized by a small batch then given a 50x larger one (re-run);
  * batches with topics on the unbounded DFS path after batches without
    (the DFS tables and tails are sized on the device)."""

import numpy as np
import pytest

import maxmq_amd
from tools import mqgen
from tools.mqgen import Strings

pytestmark = pytest.mark.gpu


def _dense_rows(idx, r, n):
    """per-topic sorted packed deliveries of a device result (segments)"""
    import torch

    from maxmq_amd.devbuf import dev_view_copy

    dev = torch.device("cuda:0")
    st = dev_view_copy(r.starts, n, torch.int64, dev).cpu().numpy()
    ct = dev_view_copy(r.counts, n, torch.int32, dev).cpu().numpy().astype(np.int64)
    hi = int((st + ct).max()) if n else 0
    d = dev_view_copy(r.deliveries, hi, torch.int32, dev).cpu().numpy().view(np.uint32)
    ss = dev_view_copy(r.shared_starts, n, torch.int64, dev).cpu().numpy()
    sc = dev_view_copy(r.shared_counts, n, torch.int32, dev).cpu().numpy().astype(np.int64)
    shi = int((ss + sc).max()) if n else 0
    h = dev_view_copy(r.shared, shi, torch.int32, dev).cpu().numpy().view(np.uint32)
    return [(tuple(sorted(d[st[t]:st[t] + ct[t]].tolist())), tuple(sorted(h[ss[t]:ss[t] + sc[t]].tolist())))
            for t in range(n)]


def _batches(w, sizes, seed=0):
    import torch

    rng = np.random.default_rng(seed)
    out = []
    for sz in sizes:
        pick = rng.choice(len(w.topics), size=sz, replace=False)
        s = Strings.from_list([w.topics[int(i)] for i in pick])
        out.append((torch.from_numpy(s.data).cuda(), torch.from_numpy(s.offs.view(np.int64)).cuda(), sz))
    return out


def _want(idx, batches):
    import torch

    res = []
    for tb, to, n in batches:
        r = idx.match_device(tb.data_ptr(), to.data_ptr(), n)
        torch.cuda.synchronize()
        res.append(_dense_rows(idx, r, n))
    return res


def test_queued_contexts_two_streams_equal_sync():
    import torch

    w = mqgen.generate(3, n_filters=400000, n_topics=200000)
    idx = maxmq_amd.TopicsIndex(0, autocommit=False)
    idx.subscribe_workload(w)
    idx.commit()
    batches = _batches(w, [20000, 20000, 5000, 30000, 20000, 20000, 1000, 25000])
    want = _want(idx, batches)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    ctxs = [idx.match_context(), idx.match_context()]
    # two rounds: the first sizes each context (exact), the second is queued
    for _ in range(2):
        pend = [None, None]
        for k, (tb, to, n) in enumerate(batches):
            c = k % 2
            if pend[c] is not None:  # the batch queued two steps ago on this context
                j = pend[c]
                r = ctxs[c].wait()
                assert _dense_rows(idx, r, batches[j][2]) == want[j], f"batch {j}"
            ctxs[c].submit(tb.data_ptr(), to.data_ptr(), n, streams[c].cuda_stream)
            pend[c] = k
        for c in (0, 1):
            if pend[c] is not None:
                j = pend[c]
                assert _dense_rows(idx, ctxs[c].wait(), batches[j][2]) == want[j], f"batch {j}"
    for c in ctxs:
        c.close()


def test_queued_outgrown_buffers_and_dfs_topics():
    """a context sized by a 1000-topic batch gets 50000 topics (re-run exact),
    then batches with topics past the walk's capacities (> 64 hits: the DFS
    path) after ones without — in the queued calls of match_device too"""
    import torch

    w = mqgen.generate(1, n_filters=20000, n_topics=60000, p_shared=0.05)
    idx = maxmq_amd.TopicsIndex(0, autocommit=False)
    idx.subscribe_workload(w)
    # 128 filters that all match "h/i/j/k/l/m": more hits than the walk keeps
    lv = ["h", "i", "j", "k", "l", "m"]
    for m in range(1 << 6):
        for rep in range(4):
            f = "/".join("+" if (m >> b) & 1 else lv[b] for b in range(6))
            idx.subscribe(f"dfs{rep}", maxmq_amd.Subscription(f if rep < 3 else f + "/#", rep % 3))
    idx.commit()
    plain = _batches(w, [1000, 50000, 3000])
    hot = Strings.from_list(["h/i/j/k/l/m"] * 3 + [w.topics[i] for i in range(500)])
    hot_b = (torch.from_numpy(hot.data).cuda(), torch.from_numpy(hot.offs.view(np.int64)).cuda(), len(hot))
    order = [plain[0], plain[1], plain[2], hot_b, plain[0], hot_b]
    want = _want(idx, order)  # (match_device's own queued calls and re-runs)
    ctx = idx.match_context()
    for j, (tb, to, n) in enumerate(order):
        ctx.submit(tb.data_ptr(), to.data_ptr(), n)
        r = ctx.wait()
        assert _dense_rows(idx, r, n) == want[j], f"batch {j}"
        if j == 3:
            assert r.n_fallback >= 3
    assert ctx.requeued() >= 1, "the 50x larger batch should have outgrown the context's buffers"
    ctx.close()


def test_queued_merge_lists_that_were_empty():
    """a queued call launches only the merge / shared lists the previous call
    had topics in (match.hip lists_seen); batches whose topics need a merge
    tier (or shared candidates) after batches that needed none are re-run
    exact and equal the synchronous result"""
    import torch

    w = mqgen.generate(1, n_filters=20000, n_topics=60000)
    idx = maxmq_amd.TopicsIndex(0, autocommit=False)
    idx.subscribe_workload(w)
    # clients whose filters co-match "zz/q/r": multi entries -> a merge list
    # (900 clients with 3 co-matching filters each: a workgroup tier, or the
    # merge by resolution)
    for c in range(900):
        for f in ("zz/q/r", "zz/+/r", "zz/#"):
            idx.subscribe(f"m{c}", maxmq_amd.Subscription(f, c % 3))
    idx.subscribe("s0", maxmq_amd.Subscription("$SHARE/g/zz/q/r", 1))
    idx.commit()
    solo = Strings.from_list(["nomatch/" + str(i) for i in range(2000)])
    solo_b = (torch.from_numpy(solo.data).cuda(), torch.from_numpy(solo.offs.view(np.int64)).cuda(), len(solo))
    hot = Strings.from_list(["zz/q/r"] * 5 + [w.topics[i] for i in range(2000)])
    hot_b = (torch.from_numpy(hot.data).cuda(), torch.from_numpy(hot.offs.view(np.int64)).cuda(), len(hot))
    order = [solo_b, solo_b, hot_b, solo_b, hot_b, hot_b]
    want = _want(idx, order)
    ctx = idx.match_context()
    for j, (tb, to, n) in enumerate(order):
        ctx.submit(tb.data_ptr(), to.data_ptr(), n)
        r = ctx.wait()
        assert _dense_rows(idx, r, n) == want[j], f"batch {j}"
        if j == 2:
            assert r.n_resolve + r.n_big >= 5 and r.n_shared > 0
    assert ctx.requeued() >= 2, "merge / shared lists unseen by the previous call must re-run the batch"
    ctx.close()


def test_index_destroy_refused_while_a_context_lives():
    """mqm_destroy returns MQM_EINVAL while a match context of the index is
    alive (a context reads its index) and leaves the index usable; the Python
    wrapper closes its contexts first"""
    from maxmq_amd import capi

    w = mqgen.generate(1, n_filters=2000, n_topics=100)
    idx = maxmq_amd.TopicsIndex(0)
    idx.subscribe_workload(w)
    ctx = idx.match_context()
    assert capi.lib().mqm_destroy(idx._h) == capi.MQM_EINVAL
    res = idx.match_batch(w.topics.data, w.topics.offs)  # still usable
    assert res.n == len(w.topics)
    idx.close()  # closes ctx, then the index
    assert not ctx._c
