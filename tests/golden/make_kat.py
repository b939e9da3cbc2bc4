"""Writes tests/golden/kat.json: the known-answer table for the reference matcher.

Every expectation below was derived BY HAND from the reference source
(vendor/github.com/mochi-co/mqtt/v2/topics.go as vendored by gsalomao/maxmq),
not computed by any restatement, so the oracles and the GPU path are all
checked against it.  Rows marked "quirk" are where the
reference differs from the MQTT spec:
  * scanSubscribers gathers at EVERY visited depth (topics.go:505), so a
    filter matches every topic it is a level-prefix of;
  * the parent-'#' rule (topics.go:507-509) fires only after a literal level;
  * the '$' rule (topics.go:527) tests Filter[0] and skips shared subs;
  * '$SHARE' is case-insensitive on Subscribe (:309) but Unsubscribe uses a
    case-sensitive HasPrefix (:330).
Also pinned: the routing cases of the reference's own system tests
(tests/system/mqtt_test.go:84-110 subscribe set, :136-253 data/# <- data/1).

Run:  python tests/golden/make_kat.py   (rewrites kat.json)
"""

import json
import os

# (filters, topic, expected matched filters (non-shared), expected shared filters, note)
FORWARD = [
    (["a"], "a/b", ["a"], [], "quirk: gather at every depth"),
    (["a/+"], "a/b/c", ["a/+"], [], "quirk: gather at every depth"),
    (["+"], "/x", ["+"], [], "quirk: '+' gathered at depth 0 of a 2-level topic"),
    (["a/+/#"], "a/b", [], [], "quirk: no parent-# after a '+' level"),
    (["+/#"], "a", [], [], "quirk: no parent-# after a '+' level"),
    (["a/b/#"], "a/b", ["a/b/#"], [], "parent-# after literal"),
    (["a/#"], "a", ["a/#"], [], "parent-# after literal"),
    (["a/+/#"], "a/b/c", ["a/+/#"], [], ""),
    (["#"], "a", ["#"], [], ""),
    (["#"], "$SYS/x", [], [], "$ rule"),
    (["+/x"], "$a/x", [], [], "$ rule"),
    (["$SYS/#"], "$SYS/x", ["$SYS/#"], [], ""),
    (["$SHARE/g/#"], "$SYS/x", [], ["$SHARE/g/#"], "quirk: shared subs skip the $ rule"),
    (["$share/g/a"], "a", [], ["$share/g/a"], "EqualFold on $SHARE"),
    (["a/b"], "a", [], [], ""),
    (["+/+"], "a", [], [], ""),
    (["a//b"], "a//b", ["a//b"], [], "empty levels"),
    (["a", "a/b", "a/+", "+/b", "#", "a/#", "a/b/#", "+/+/+", "b"], "a/b",
     ["a", "a/b", "a/+", "+/b", "#", "a/#", "a/b/#"], [], "mixed"),
    (["/", "+/", "/+", "#"], "/", ["/", "+/", "/+", "#"], [], "empty first/last levels"),
    ([""], "a", [], [], "empty filter stored at root child ''"),
    (["+"], "a/b/c/d", ["+"], [], "quirk: '+' prefix-matches deep topics"),
    (["a/+/c/#"], "a/b/c", ["a/+/c/#"], [], "parent-# after literal 'c'"),
    (["a/+/+/#"], "a/b/c", [], [], "no parent-# after '+'"),
    (["$SHARE/g1/a/+", "$SHARE/g2/a/+", "a/+"], "a/b", ["a/+"], ["$SHARE/g1/a/+", "$SHARE/g2/a/+"], "shared"),
    (["+abc/x"], "$foo/x", [], [], "unreachable literal"),
    (["$foo/+"], "$foo/x", ["$foo/+"], [], "$ topic with literal root filter"),
    (["#"], "$", [], [], "$ rule on 1-char topic"),
    (["$SHARE/g"], "g", [], ["$SHARE/g"], "invalid 2-level share filter stored at the last level (isolateParticle)"),
]

# system-test pins: R/tests/system/mqtt_test.go:84-110 and :136-253
SYSTEM = [
    (["temp", "sensor/#", "data/+/raw"], "data/1", [], [], "subscribe set does not route data/1"),
    (["data/#"], "data/1", ["data/#"], [], "mqtt_test.go:136-253 data/# receives data/1"),
]

# Merge (packets.go:250-270): one client, several matching filters
MERGE = [
    {
        "subs": [["c1", "a/#", 0, 0, 0, 0, 7], ["c1", "a/b", 2, 1, 1, 2, 0], ["c1", "+/b", 1, 0, 0, 1, 9]],
        "topic": "a/b",
        # DFS order: 'a' literal -> parent probe a/# first, then a/b, then +/b
        "expect": {"c1": {"qos": 2, "no_local": 1, "first": "a/#", "first_ident": 7, "rap": 0, "rh": 0}},
        # Identifiers (packets.go:251-259): {first: 7}, a/b has id 0 (not added), +/b adds 9
        "identifiers": {"c1": {"a/#": 7, "+/b": 9}},
    },
    {
        "subs": [["c1", "+/b", 1, 0, 1, 1, 3], ["c1", "a/b", 0, 0, 0, 2, 0]],
        "topic": "a/b",
        "expect": {"c1": {"qos": 1, "no_local": 0, "first": "a/b", "first_ident": 0, "rap": 0, "rh": 2}},
        # the first pair is kept even with Identifier 0
        "identifiers": {"c1": {"a/b": 0, "+/b": 3}},
    },
    {
        # a/+ reached through the '+' child of a; a/b/# parent probe happens
        # under literal 'b' before the '+' subtree
        "subs": [["c1", "a/+", 0, 0, 1, 0, 1], ["c1", "a/b/#", 1, 0, 0, 0, 2]],
        "topic": "a/b",
        "expect": {"c1": {"qos": 1, "no_local": 0, "first": "a/b/#", "first_ident": 2, "rap": 0, "rh": 0}},
        "identifiers": {"c1": {"a/b/#": 2, "a/+": 1}},
    },
    {
        # a/# and a/b/# are each gathered twice (parent probe, then the '#'
        # child itself); c2's root '#' comes last at level 0, after a/b/#
        "subs": [["c1", "a/#", 0, 0, 0, 0, 5], ["c1", "a/b/c", 2, 0, 0, 0, 0], ["c2", "#", 1, 0, 0, 0, 0],
                 ["c2", "a/b/#", 0, 0, 0, 0, 4]],
        "topic": "a/b/c",
        "expect": {"c1": {"qos": 2, "no_local": 0, "first": "a/#", "first_ident": 5, "rap": 0, "rh": 0},
                   "c2": {"qos": 1, "no_local": 0, "first": "a/b/#", "first_ident": 4, "rap": 0, "rh": 0}},
        "identifiers": {"c1": {"a/#": 5}, "c2": {"a/b/#": 4}},
    },
]

# retained reverse match (topics.go:426-480)
RETAINED_TOPICS = ["a", "a/b", "a/b/c", "$SYS/x", "$foo/x", "b", "/x"]
REVERSE = [
    ("a/#", ["a/b", "a/b/c"]),
    ("#", ["a", "a/b", "a/b/c", "$foo/x", "b", "/x"]),
    ("+", ["a", "b"]),
    ("+/+", ["$foo/x", "/x", "a/b"]),
    ("+/#", ["$foo/x", "/x", "a/b", "a/b/c"]),
    ("a/+/c", ["a/b/c"]),
    ("a/b", ["a/b"]),
    ("zz", []),
    ("", []),
]

ISOLATE = [
    ("a/b", 0, "a", True),
    ("a/b", 1, "b", False),
    ("a/b", 5, "b", False),
    ("a/", 1, "", False),
    ("", 0, "", False),
    ("a/b", -1, "", False),
    ("/x", 0, "", True),
]

# mutation return values (Subscribe / Unsubscribe / RetainMessage)
MUTATIONS = [
    ["sub", "c1", "a/b", True],
    ["sub", "c1", "a/b", False],
    ["sub", "c2", "a/b", True],
    ["unsub", "a/b", "c3", True],
    ["unsub", "x/y", "c1", False],
    ["sub", "c1", "$share/g/a", True],
    ["unsub", "$share/g/a", "c1", False],
    ["sub", "c1", "$share/g/a", False],
    ["unsub", "$SHARE/g/a", "c1", True],
    ["sub", "c1", "$SHARE/g/a", True],
    ["unsub", "a/b", "c1", True],
    ["unsub", "a/b", "c2", True],
    ["unsub", "a/b", "c2", False],
    ["retain", "r/t", 5, 1],
    ["retain", "r/t", 0, -1],
    ["retain", "r/t", 0, 0],
]

VALID = [
    ("a/b", False, True), ("", False, False), ("#", False, True), ("a/#/b", False, False), ("a/b#", False, True),
    ("$SHARE/g/a", False, True), ("$SHARE/g", False, False), ("$SHARE/+/a", False, False), ("$share", False, False),
    ("a/+", True, False), ("$SYS/x", True, False), ("$sys", True, False), ("a/b", True, True), ("", True, True),
    ("a+", False, True),
]


def main():
    out = {
        "source": "hand-derived from vendor/github.com/mochi-co/mqtt/v2/topics.go (mochi v2.2.12)",
        "forward": [dict(filters=f, topic=t, subs=s, shared=sh, note=n) for f, t, s, sh, n in FORWARD + SYSTEM],
        "merge": MERGE,
        "retained_topics": RETAINED_TOPICS,
        "reverse": [dict(filter=f, topics=t) for f, t in REVERSE],
        "isolate": [dict(s=s, d=d, particle=p, has_next=h) for s, d, p, h in ISOLATE],
        "mutations": MUTATIONS,
        "valid": [dict(filter=f, for_publish=p, valid=v) for f, p, v in VALID],
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
