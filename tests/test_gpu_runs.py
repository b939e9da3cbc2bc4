"""The runs form of the host path (mqm_match_batch_runs): every topic's solo
deliveries as runs of the snapshot's packed-word table (8 B per run over
PCIe), its merged winners explicit.  After expansion (mqm_result_expand) the
rows must equal the oracle's (oracle/mochi_ref.c, topics.go:484-555 +
packets.go:250-270) field by field, and the packed host path's rows, on:
  * config 1 with shared subscriptions, and a 300k-filter config 3 sample;
  * the edge cases that route topics differently: heavy clients (hash-table
    merges), topics past the walk's capacities (the DFS path: all of their
    deliveries come back as winners, no runs), '$' topics, empty levels;
  * Identifiers support on an index created with identifiers=True;
and the raw form must be consistent: runs inside the word table, run counts +
winners = the expanded counts, and the solo share reported by the device."""

import numpy as np
import pytest

import maxmq_amd
from oracle.binding import OracleIndex
from tests.gpu_util import assert_same, canon_gpu, canon_gpu_idents, canon_oracle, canon_oracle_idents
from tools import mqgen
from tools.mqgen import Strings

pytestmark = pytest.mark.gpu


def _raw_consistent(res, words_len):
    assert res.runs_form
    n = res.n
    runs = res.runs.astype(np.int64)
    assert np.all(runs[:, 0] + runs[:, 1] <= words_len), "a run past the word table"
    assert np.all(runs[:, 1] > 0), "an empty run"
    cs = np.concatenate([[0], np.cumsum(runs[:, 1])])
    ro = res.run_offsets.astype(np.int64)
    run_sum = cs[ro[1:]] - cs[ro[:-1]]
    win = np.diff(res.winner_offsets.astype(np.int64))
    assert np.array_equal(run_sum + win, np.diff(res.offsets.astype(np.int64))), "runs + winners != rows"
    return int(run_sum.sum()), int(win.sum())


@pytest.mark.parametrize("config,overrides", [(1, {"p_shared": 0.05}), (3, {"n_filters": 300000, "n_topics": 60000})])
def test_runs_form_vs_oracle_and_packed(config, overrides):
    w = mqgen.generate(config, **overrides)
    idx = maxmq_amd.TopicsIndex(0)
    idx.subscribe_workload(w)
    ora = OracleIndex()
    ora.subscribe_workload(w)
    s = w.topics
    res = idx.match_batch_runs(s.data, s.offs)
    solo, win = _raw_consistent(res, idx.snapshot_stats()["subs"])
    assert solo > win, (solo, win)  # most deliveries are solo runs
    g, gs = canon_gpu(res)
    p, ps = canon_gpu(idx.match_batch_packed(s.data, s.offs))
    r, rs = canon_oracle(*ora.match(s.data, s.offs, nthreads=16)[:4])
    assert_same(g, r, "runs form vs oracle")
    assert_same(gs, rs, "runs form vs oracle (shared)")
    assert_same(p, g, "packed vs runs form")
    assert_same(ps, gs, "packed vs runs form (shared)")


def test_runs_form_edge_cases_and_dfs_topics():
    idx = maxmq_amd.TopicsIndex(0)
    ora = OracleIndex()
    subs = []
    # a heavy client (> 64 subscriptions) and level-compatible partners
    for i in range(80):
        subs.append(("heavy", f"h/{i}/#", i % 3))
        subs.append(("heavy", f"h/+/{i}", (i + 1) % 3))
    for c in range(300):
        subs += [(f"c{c}", "a/b/c", c % 3), (f"c{c}", "a/+/c", (c + 1) % 3), (f"d{c}", "a/#", 1)]
    subs += [("x", "$SYS/#", 0), ("y", "#", 2), ("y", "+/+", 1), ("z", "/+", 0), ("z", "+//x", 1)]
    # deep filters: topics below take the DFS path (past 16 cached levels)
    deep = "/".join(f"l{k}" for k in range(22))
    for c in range(40):
        subs += [(f"p{c}", deep, c % 3), (f"p{c}", "l0/#", 1), (f"p{c}", "l0/+/l2/#", 2)]
    for cl, f, q in subs:
        idx.subscribe(cl, maxmq_amd.Subscription(f, q))
        ora.subscribe(cl, f, q)
    topics = ["h/3/3", "h/7/x", "a/b/c", "a/z/c", "$SYS/x", "/x", "//x", "x//x", "", "a", deep, deep + "/more",
              "l0/l1/l2/l3"] + [f"h/{i}/{i}" for i in range(80)]
    s = Strings.from_list(topics)
    res = idx.match_batch_runs(s.data, s.offs)
    _raw_consistent(res, idx.snapshot_stats()["subs"])
    dfs_topic = topics.index(deep)
    assert res.run_offsets[dfs_topic + 1] == res.run_offsets[dfs_topic], "a DFS topic has no runs"
    g, gs = canon_gpu(res)
    r, rs = canon_oracle(*ora.match(s.data, s.offs)[:4])
    assert_same(g, r, "runs form edge cases vs oracle")
    assert_same(gs, rs, "runs form edge cases vs oracle (shared)")


def test_runs_form_identifiers():
    w = mqgen.generate(1, n_filters=20000, n_topics=20000, p_shared=0.05)
    idx = maxmq_amd.TopicsIndex(0, identifiers=True)
    idx.subscribe_workload(w)
    ora = OracleIndex()
    ora.subscribe_workload(w)
    s = w.topics
    res = idx.match_batch_runs(s.data, s.offs)
    assert res.runs_form
    g, _ = canon_gpu(res)
    r, _ = canon_oracle(*ora.match(s.data, s.offs, nthreads=8)[:4])
    assert_same(g, r, "runs form (identifiers index) vs oracle")
    assert_same(canon_gpu_idents(res), canon_oracle_idents(*ora.identifiers(s.data, s.offs, nthreads=8)),
                "runs form identifiers")


@pytest.mark.parametrize("form", ["runs", "packed", "plain"])
def test_kernel_copy_out_matches_dma(form, monkeypatch):
    """MQM_D2H_KERNEL=1 (the result parts stored into the pinned block by one
    kernel, match.hip k_copy_out) returns what the DMA copies return, and the
    oracle's sets — shared subscriptions and Identifiers included."""
    w = mqgen.generate(1, n_filters=20000, n_topics=30000, p_shared=0.05)
    idx = maxmq_amd.TopicsIndex(0, identifiers=True)
    idx.subscribe_workload(w)
    s = w.topics
    call = {"runs": idx.match_batch_runs, "packed": idx.match_batch_packed, "plain": idx.match_batch}[form]
    got = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("MQM_D2H_KERNEL", mode)
        res = call(s.data, s.offs)
        got[mode] = (canon_gpu(res), canon_gpu_idents(res))
    (g0, gs0), i0 = got["0"]
    (g1, gs1), i1 = got["1"]
    assert_same(g1, g0, f"{form}: kernel copy-out vs DMA")
    assert_same(gs1, gs0, f"{form}: kernel copy-out vs DMA (shared)")
    assert_same(i1, i0, f"{form}: kernel copy-out vs DMA (identifiers)")
    ora = OracleIndex()
    ora.subscribe_workload(w)
    r, rs = canon_oracle(*ora.match(s.data, s.offs, nthreads=8)[:4])
    assert_same(g1, r, f"{form}: kernel copy-out vs oracle")
    assert_same(gs1, rs, f"{form}: kernel copy-out vs oracle (shared)")
