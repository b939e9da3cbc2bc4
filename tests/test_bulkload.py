"""Bulk reload of persisted subscriptions:
mqm_load_subscriptions_json decodes storage.Subscription JSON records
(vendor/github.com/mochi-co/mqtt/v2/hooks/storage/storage.go:151-161) with
encoding/json's rules and replays them like Server.loadSubscriptions
(server.go:1377-1393): one Subscribe per record, in order.  Checked against
the same records applied through mqm_subscribe (equal snapshot digests and
per-record return values), and against hand cases for the decoder rules.
Host-only indexes: no GPU needed."""

import json
import random

import pytest

import maxmq_amd
from maxmq_amd import capi

LEVELS = ["a", "b", "", "+", "#", "$SYS", "$SHARE", "$share", "g", "é", "日本", "x" * 20]


def _record(rng, i):
    f = "/".join(rng.choice(LEVELS) for _ in range(rng.randint(1, 4)))
    return {"t": "subscription", "id": f"SUB_c{i}:{f}", "client": f"c{rng.randint(0, 20)}", "filter": f,
            "identifier": rng.choice([0, 0, 7, 268435455]), "retain_handling": rng.randint(0, 2),
            "qos": rng.randint(0, 2), "retain_as_pub": rng.random() < 0.3, "no_local": rng.random() < 0.2}


def _apply(idx, recs):
    out = []
    for r in recs:
        out.append(idx.subscribe(r["client"], maxmq_amd.Subscription(
            r["filter"], r["qos"], r["identifier"], r["no_local"], r["retain_as_pub"], r["retain_handling"])))
    return out


@pytest.mark.parametrize("form", ["array", "lines", "ascii"])
def test_json_load_equals_subscribe_calls(form):
    rng = random.Random(3)
    recs = [_record(rng, i) for i in range(2000)]
    if form == "array":
        blob = json.dumps(recs, ensure_ascii=False).encode()
    elif form == "lines":
        blob = "\n".join(json.dumps(r, ensure_ascii=False) for r in recs).encode()
    else:
        blob = json.dumps(recs, ensure_ascii=True, indent=1).encode()
    a = maxmq_amd.TopicsIndex(device=None, autocommit=False)
    b = maxmq_amd.TopicsIndex(device=None, autocommit=False)
    n, fresh = a.load_subscriptions_json(blob)
    want = _apply(b, recs)
    assert n == len(recs) and fresh == sum(want)
    a.commit()
    b.commit()
    assert a.snapshot_digest() == b.snapshot_digest()


def test_json_load_through_async_index_journal():
    rng = random.Random(4)
    recs = [_record(rng, i) for i in range(500)]
    a = maxmq_amd.TopicsIndex(device=None, autocommit=False, async_commit=True)
    b = maxmq_amd.TopicsIndex(device=None, autocommit=False)
    a.load_subscriptions_json(json.dumps(recs).encode())
    _apply(b, recs)
    a.commit_async()
    a.commit_poll(wait=True)
    b.commit()
    assert a.snapshot_digest() == b.snapshot_digest()


def _load_one(obj_text: str):
    idx = maxmq_amd.TopicsIndex(device=None, autocommit=False)
    idx.load_subscriptions_json(obj_text.encode("utf-8", "surrogatepass"))
    return idx


def test_decoder_rules():
    # case-insensitive keys (Go's fold incl. U+017F and U+212A), unknown keys, last duplicate wins
    idx = _load_one('{"CLIENT":"c1","Filter":"a/b","QOS":1,"xtra":{"n":[1,2,{"z":null}]},"filter":"a/c",'
                    '"no_local":true,"ſtray":1}')
    assert idx.client_name(0) == "c1" and idx.filter_name(0) == "a/c"
    idx = _load_one('{"client":"c","filter":"x","Key":1,"qoſ":2}')  # "qoſ" folds to "qos"
    idx.commit()
    assert idx.snapshot_stats()["subs"] == 1
    # escapes: surrogate pair, lone surrogate -> U+FFFD, \/ and é
    idx = _load_one('{"client":"c","filter":"\\ud83d\\ude00/\\ud800/\\/\\u00e9"}')
    assert idx.filter_name(0) == "\U0001F600/�//é"
    # null record / null fields: zero values (Subscribe("", {Filter:""}))
    idx = maxmq_amd.TopicsIndex(device=None, autocommit=False)
    assert idx.load_subscriptions_json(b'[null, {"client":null,"filter":"a","qos":null}]') == (2, 2)
    assert idx.filter_name(0) == "" and idx.client_name(0) == ""
    # empty inputs
    assert maxmq_amd.TopicsIndex(device=None).load_subscriptions_json(b"") == (0, 0)
    assert maxmq_amd.TopicsIndex(device=None).load_subscriptions_json(b" [ ] ") == (0, 0)


def test_invalid_bytes_become_replacement_char():
    idx = maxmq_amd.TopicsIndex(device=None, autocommit=False)
    idx.load_subscriptions_json(b'{"client":"c","filter":"a\xff/b\xc3"}')
    assert idx.filter_name(0) == "a�/b�"


@pytest.mark.parametrize("bad", [
    '{"client":"c","filter":"a","qos":1.0}',       # not an integer literal
    '{"client":"c","filter":"a","qos":"1"}',       # string into a byte
    '{"client":"c","filter":"a","qos":256}',       # out of byte range
    '{"client":"c","filter":"a","qos":-1}',
    '{"client":"c","filter":"a","no_local":1}',    # number into a bool
    '{"client":"c","filter":"a"',                  # truncated
    '{"client":"c","filter":"a\x01"}',             # raw control character
    '[{"client":"c","filter":"a"} {"client":"d","filter":"b"}]',  # missing comma
    '{"client":"c","filter":"a","qos":01}',        # leading zero
])
def test_rejected_records_stop_the_load(bad):
    idx = maxmq_amd.TopicsIndex(device=None, autocommit=False)
    blob = ('{"client":"ok","filter":"z"}\n' + bad).encode()
    with pytest.raises(maxmq_amd.MqmError) as e:
        idx.load_subscriptions_json(blob)
    assert e.value.rc == capi.MQM_EINVAL
    assert e.value.n_loaded in (1, 0 if bad.startswith("[") else 1)
    assert idx.filter_name(0) == "z"


@pytest.mark.parametrize("rec", ['{"client":"c","filter":"a","qos":3}',
                                 '{"client":"c","filter":"a","retain_handling":4}',
                                 '{"client":"c","filter":"a","identifier":4294967296}'])
def test_records_outside_snapshot_ranges(rec):
    idx = maxmq_amd.TopicsIndex(device=None, autocommit=False)
    with pytest.raises(maxmq_amd.MqmError) as e:
        idx.load_subscriptions_json(rec.encode())
    assert e.value.rc == capi.MQM_ELIMIT and e.value.n_loaded == 0
