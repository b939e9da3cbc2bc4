"""CPU tests: pin the two oracle restatements (C and Python) against the
hand-derived known-answer table and the reference's system-test routing
fixtures, then against each other on generated workloads."""

import random

import numpy as np
import pytest

from oracle import mochi_ref as pyref
from oracle.binding import OracleIndex, isolate_particle
from tools import mqgen
from tools.mqgen import Strings


def _c_match_filters(idx: OracleIndex, topic: str):
    s = Strings.from_list([topic])
    doffs, dout, soffs, sout, _ = idx.match(s.data, s.offs)
    subs = sorted(idx.filter_name(int(r["first_filter"])) for r in dout)
    shared = sorted(idx.filter_name(int(r["filter"])) for r in sout)
    return subs, shared


def test_isolate_particle_kat(kat):
    for row in kat["isolate"]:
        exp = (row["particle"], row["has_next"])
        assert pyref.isolate_particle(row["s"], row["d"]) == exp, row
        assert isolate_particle(row["s"], row["d"]) == exp, row


@pytest.mark.parametrize("impl", ["c", "py"])
def test_forward_kat(kat, impl):
    for case in kat["forward"]:
        # one client per filter so the matched set names the filters
        if impl == "c":
            idx = OracleIndex()
            for i, f in enumerate(case["filters"]):
                idx.subscribe(f"c{i}", f, qos=1)
            subs, shared = _c_match_filters(idx, case["topic"])
        else:
            idx = pyref.TopicsIndex()
            for i, f in enumerate(case["filters"]):
                idx.subscribe(f"c{i}", pyref.Sub(f, 1))
            s, sh = idx.subscribers(case["topic"])
            subs = sorted(v.filter for v in s.values())
            shared = sorted(sh)
        assert subs == sorted(case["subs"]), case
        assert shared == sorted(case["shared"]), case


@pytest.mark.parametrize("impl", ["c", "py"])
def test_merge_kat(kat, impl):
    for case in kat["merge"]:
        if impl == "c":
            idx = OracleIndex()
            for c, f, q, nl, rap, rh, ident in case["subs"]:
                idx.subscribe(c, f, q, nl, rap, rh, ident)
            s = Strings.from_list([case["topic"]])
            _, dout, _, _, _ = idx.match(s.data, s.offs)
            got = {idx.client_name(int(r["client"])): dict(qos=int(r["qos"]), no_local=int(r["no_local"]),
                                                              first=idx.filter_name(int(r["first_filter"])),
                                                              first_ident=int(r["first_ident"]), rap=int(r["rap"]),
                                                              rh=int(r["rh"])) for r in dout}
            ioffs, iout = idx.identifiers(s.data, s.offs)
            ids = {}
            for r in iout:
                ids.setdefault(idx.client_name(int(r["client"])), {})[idx.filter_name(int(r["filter"]))] = int(r["ident"])
        else:
            idx = pyref.TopicsIndex()
            for c, f, q, nl, rap, rh, ident in case["subs"]:
                idx.subscribe(c, pyref.Sub(f, q, ident, nl, rap, rh))
            subs, _ = idx.subscribers(case["topic"])
            got = {c: dict(qos=v.qos, no_local=int(v.no_local), first=v.filter, first_ident=v.identifier,
                           rap=int(v.rap), rh=v.rh) for c, v in subs.items()}
            ids = {c: dict(v.identifiers) for c, v in subs.items()}
        assert got == case["expect"], case
        assert ids == case["identifiers"], case


@pytest.mark.parametrize("impl", ["c", "py"])
def test_reverse_kat(kat, impl):
    topics = kat["retained_topics"]
    idx = OracleIndex() if impl == "c" else pyref.TopicsIndex()
    for i, t in enumerate(topics):
        idx.retain_message(t, i + 1, 10, True)
    for case in kat["reverse"]:
        if impl == "c":
            s = Strings.from_list([case["filter"]])
            _, out = idx.messages(s.data, s.offs)
            got = sorted(topics[int(r) - 1] for r in out)
        else:
            got = sorted(topics[r - 1] for r in idx.messages(case["filter"]))
        assert got == sorted(case["topics"]), case


@pytest.mark.parametrize("impl", ["c", "py"])
def test_mutation_kat(kat, impl):
    idx = OracleIndex() if impl == "c" else pyref.TopicsIndex()
    for op in kat["mutations"]:
        if op[0] == "sub":
            r = idx.subscribe(op[1], op[2]) if impl == "c" else idx.subscribe(op[1], pyref.Sub(op[2]))
        elif op[0] == "unsub":
            r = idx.unsubscribe(op[1], op[2])
        else:
            r = idx.retain_message(op[1], 1, op[2], True)
        assert r == op[3], op


def test_valid_filter_kat(kat):
    for row in kat["valid"]:
        assert pyref.is_valid_filter(row["filter"], row["for_publish"]) == row["valid"], row


def _py_from_workload(w):
    idx = pyref.TopicsIndex()
    for i in range(len(w.filters)):
        idx.subscribe(w.clients[i], pyref.Sub(w.filters[i], int(w.qos[i]), int(w.ident[i]), bool(w.no_local[i]),
                                              bool(w.rap[i]), int(w.rh[i])))
    return idx


@pytest.mark.parametrize("config,nf,nt", [(1, 3000, 3000), (5, 3000, 2000)])
def test_c_vs_python_restatements(config, nf, nt):
    """The two independent restatements agree on every field of every result."""
    w = mqgen.generate(config, n_filters=nf, n_topics=nt)
    c = OracleIndex()
    c.subscribe_workload(w)
    py = _py_from_workload(w)
    doffs, dout, soffs, sout, st = c.match(w.topics.data, w.topics.offs, nthreads=4)
    ioffs, iout = c.identifiers(w.topics.data, w.topics.offs, nthreads=4)
    assert st["deliveries"] > 0
    for i in range(nt):
        subs, shared = py.subscribers(w.topics[i])
        exp = sorted((k, v.qos, int(v.no_local), v.filter, v.identifier, int(v.rap), v.rh) for k, v in subs.items())
        got = sorted((c.client_name(int(r["client"])), int(r["qos"]), int(r["no_local"]),
                      c.filter_name(int(r["first_filter"])), int(r["first_ident"]), int(r["rap"]), int(r["rh"]))
                     for r in dout[doffs[i]:doffs[i + 1]])
        assert got == exp, w.topics[i]
        exp_sh = sorted((f, k) for f, m in shared.items() for k in m)
        got_sh = sorted((c.filter_name(int(r["filter"])), c.client_name(int(r["client"])))
                        for r in sout[soffs[i]:soffs[i + 1]])
        assert got_sh == exp_sh, w.topics[i]
        exp_id = sorted((k, f, v) for k, s in subs.items() for f, v in s.identifiers.items())
        got_id = sorted((c.client_name(int(r["client"])), c.filter_name(int(r["filter"])), int(r["ident"]))
                        for r in iout[ioffs[i]:ioffs[i + 1]])
        assert got_id == exp_id, w.topics[i]


def _rand_level(rng):
    return rng.choice(["a", "b", "", "+", "#", "$SYS", "$x", "$share", "$SHARE", "cſ", "long-token-" * 2])


def test_c_vs_python_random_ops():
    """Random Subscribe/Unsubscribe/RetainMessage sequences over a tiny,
    collision-heavy alphabet (invalid filters included: TopicsIndex itself
    validates nothing): return values and match results agree."""
    rng = random.Random(1234)
    for trial in range(30):
        c, py = OracleIndex(), pyref.TopicsIndex()
        for step in range(150):
            lv = [_rand_level(rng) for _ in range(rng.randint(1, 4))]
            f = "/".join(lv)
            client = f"k{rng.randint(0, 5)}"
            op = rng.random()
            if op < 0.6:
                q = rng.randint(0, 2)
                r1 = c.subscribe(client, f, qos=q, ident=rng.randint(0, 3))
                r2 = py.subscribe(client, pyref.Sub(f, q))
            elif op < 0.85:
                r1, r2 = c.unsubscribe(f, client), py.unsubscribe(f, client)
            else:
                t = "/".join(x for x in lv if x not in ("+", "#")) or "a"
                pl = rng.choice([0, 3])
                r1, r2 = c.retain_message(t, step + 1, pl), py.retain_message(t, step + 1, pl)
            assert r1 == r2, (trial, step, op, f, client)
        topics = ["/".join(rng.choice(["a", "b", "", "$SYS", "$x", "c"]) for _ in range(rng.randint(1, 5)))
                  for _ in range(60)]
        s = Strings.from_list(topics)
        doffs, dout, soffs, sout, _ = c.match(s.data, s.offs)
        for i, t in enumerate(topics):
            subs, shared = py.subscribers(t)
            exp = sorted((k, v.qos) for k, v in subs.items())
            got = sorted((c.client_name(int(r["client"])), int(r["qos"])) for r in dout[doffs[i]:doffs[i + 1]])
            assert got == exp, (trial, t)
            exp_sh = sorted((f, k) for f, m in shared.items() for k in m)
            got_sh = sorted((c.filter_name(int(r["filter"])), c.client_name(int(r["client"])))
                            for r in sout[soffs[i]:soffs[i + 1]])
            assert got_sh == exp_sh, (trial, t)
        filters = ["/".join(_rand_level(rng) for _ in range(rng.randint(1, 3))) for _ in range(40)]
        fs = Strings.from_list(filters)
        moffs, mout = c.messages(fs.data, fs.offs)
        for i, f in enumerate(filters):
            assert sorted(py.messages(f)) == sorted(int(x) for x in mout[moffs[i]:moffs[i + 1]]), (trial, f)
