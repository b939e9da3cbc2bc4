"""The Go shim's call sequence as a C program issuing
Subscribe, then Subscribers / batched matches from 4 threads at once against
one index (tests/harness/shim_harness.c, C ABI only), checked against the
oracle restatement rendered the same way: the full `*Subscribers` value
(topics.go:247-252) — every merged subscription with its Identifiers map
(packets.go:250-270) and the `Shared` map's (filter, client) pairs
(topics.go:541-555) — plus Subscribe's return values (topics.go:303-321).
Reference callers: server.go:776-783 (publish), listeners/tcp.go:83 (one
goroutine per connection, so Subscribers runs concurrently)."""

import os
import subprocess

import numpy as np
import pytest

from oracle.binding import OracleIndex
from tools import mqgen

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tests", "harness", "_build", "shim_harness")


def _harness():
    if not os.path.exists(HARNESS):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "harness")])
    return HARNESS


def _write_input(path, w):
    with open(path, "w", encoding="utf-8", newline="\n") as fh:
        fh.write(f"{len(w.filters)} {len(w.topics)}\n")
        for i in range(len(w.filters)):
            fh.write(f"{w.clients[i]}\t{w.filters[i]}\t{w.qos[i]}\t{w.no_local[i]}\t{w.rap[i]}\t{w.rh[i]}\t"
                     f"{w.ident[i]}\n")
        for i in range(len(w.topics)):
            fh.write(w.topics[i] + "\n")


def _expected(w):
    ora = OracleIndex()
    is_new = [ora.subscribe(w.clients[i], w.filters[i], int(w.qos[i]), bool(w.no_local[i]), bool(w.rap[i]),
                            int(w.rh[i]), int(w.ident[i])) for i in range(len(w.filters))]
    doffs, dout, soffs, sout, _ = ora.match(w.topics.data, w.topics.offs, nthreads=4)
    ioffs, iout = ora.identifiers(w.topics.data, w.topics.offs, nthreads=4)
    cname = {}
    fname = {}

    def cn(i):
        if i not in cname:
            cname[i] = ora.client_name(int(i))
        return cname[i]

    def fn(i):
        if i not in fname:
            fname[i] = ora.filter_name(int(i))
        return fname[i]

    lines = [f"N {i} {int(v)}" for i, v in enumerate(is_new)]
    for t in range(len(w.topics)):
        ids = {}
        for e in iout[int(ioffs[t]):int(ioffs[t + 1])]:
            ids.setdefault(int(e["client"]), []).append((fn(e["filter"]), int(e["ident"])))
        for d in dout[int(doffs[t]):int(doffs[t + 1])]:
            m = ",".join(f"{f}={i}" for f, i in sorted(ids[int(d["client"])]))
            lines.append(f"D {t} {cn(d['client'])} {d['qos']} {d['no_local']} {fn(d['first_filter'])} "
                         f"{d['first_ident']} {d['rap']} {d['rh']} {m}")
        for s in sout[int(soffs[t]):int(soffs[t + 1])]:
            lines.append(f"H {t} {fn(s['filter'])} {cn(s['client'])}")
    ora.close()
    return sorted(lines)


@pytest.mark.gpu
@pytest.mark.parametrize("threads,mode", [(4, "direct"), (16, "batching")])
def test_shim_call_sequence_concurrent_readers(tmp_path, threads, mode):
    """mode "batching": the same call sequence with MQM_CFG_BATCHING, so the
    16 threads' single-topic calls are gathered by the collector"""
    w = mqgen.generate(1, n_filters=4000, n_topics=6000, n_clients=400, p_shared=0.05, seed=0x5A17)
    inp, out = tmp_path / "in.txt", tmp_path / "out.txt"
    _write_input(inp, w)
    args = [_harness(), str(inp), str(out), str(threads)] + (["batching"] if mode == "batching" else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    got = sorted(out.read_text(encoding="utf-8").splitlines())
    want = _expected(w)
    assert len(got) == len(want), (len(got), len(want))
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert not bad, f"first difference: got {got[bad[0]]!r} want {want[bad[0]]!r}"
    assert any(ln.startswith("H ") for ln in want) and any("," in ln.split()[-1] for ln in want if ln[0] == "D")
