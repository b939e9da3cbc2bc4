"""oracle/mochi_ref.py — TEST INFRASTRUCTURE ONLY.

A second, independent restatement of mochi-co/mqtt v2.2.12 ``TopicsIndex``
(vendor/github.com/mochi-co/mqtt/v2/topics.go:284-699) and
``Subscription.Merge`` (vendor/.../packets/packets.go:248-270), written with
plain Python dicts for small cases.  It exists to pin ``oracle/mochi_ref.c``
(the C restatement the GPU parity tests check against) from a second
direction, and to produce the golden fixtures under ``tests/golden``.

Only tests/ and fixture scripts import it; the product never does.
No Go toolchain is available, so neither restatement is checked against an
executed reference: the known-answer table and the
reference's own system-test routing cases are the external pins.
"""

from __future__ import annotations

SHARE_PREFIX = "$SHARE"  # topics.go:16
SYS_PREFIX = "$SYS"  # topics.go:17


def isolate_particle(s: str, d: int):
    """isolateParticle (topics.go:558-577): level d of s and hasNext.

    Past the last level it returns the last level and False; d == -1 gives
    ("", False).  Empty levels are kept.
    """
    if d < 0:
        return "", False
    parts = s.split("/")
    if d < len(parts) - 1:
        return parts[d], True
    return parts[-1], False


def equal_fold(a: str, b: str) -> bool:
    """strings.EqualFold for the ASCII words the index compares against.

    Go uses Unicode simple folding; for the letters of "$SHARE"/"$SYS" the only
    non-ASCII rune in a fold orbit is U+017F (long s) ~ 's'.
    """
    if len(a) != len(b):
        return False
    for x, y in zip(a, b):
        if x == "\u017f":
            x = "s"
        if y == "\u017f":
            y = "s"
        if x.isascii() and y.isascii():
            if x.lower() != y.lower():
                return False
        elif x != y:
            return False
    return True


class Sub:
    """packets.Subscription (packets.go:168-178), the fields the index reads."""

    __slots__ = ("filter", "qos", "identifier", "no_local", "rap", "rh", "identifiers")

    def __init__(self, filter, qos=0, identifier=0, no_local=False, rap=False, rh=0):
        self.filter = filter
        self.qos = qos
        self.identifier = identifier
        self.no_local = bool(no_local)
        self.rap = bool(rap)
        self.rh = rh
        self.identifiers = None

    def copy(self):
        s = Sub(self.filter, self.qos, self.identifier, self.no_local, self.rap, self.rh)
        s.identifiers = None if self.identifiers is None else dict(self.identifiers)
        return s

    def merge(self, n: "Sub") -> "Sub":
        """Subscription.Merge (packets.go:250-270)."""
        s = self.copy()
        if s.identifiers is None:
            s.identifiers = {s.filter: s.identifier}
        if n.identifier > 0:
            s.identifiers[n.filter] = n.identifier
        if n.qos > s.qos:
            s.qos = n.qos
        if n.no_local:
            s.no_local = True
        return s


class Particle:
    """particle (topics.go:627-646)."""

    __slots__ = ("key", "parent", "particles", "subscriptions", "shared", "retain_path")

    def __init__(self, key, parent):
        self.key = key
        self.parent = parent
        self.particles = {}
        self.subscriptions = {}  # client -> Sub
        self.shared = {}  # group -> {client -> Sub}
        self.retain_path = ""

    def shared_len(self):
        return sum(len(g) for g in self.shared.values())


class TopicsIndex:
    """TopicsIndex (topics.go:285-299)."""

    def __init__(self):
        self.root = Particle("", None)
        self.retained = {}  # topic -> (msg_ref, payload_len, retain_flag)

    # -- mutation -----------------------------------------------------------
    def _set(self, topic, d):
        n = self.root
        has_next = True
        while has_next:
            key, has_next = isolate_particle(topic, d)
            d += 1
            p = n.particles.get(key)
            if p is None:
                p = Particle(key, n)
                n.particles[key] = p
            n = p
        return n

    def _seek(self, filt, d):
        n = self.root
        has_next = True
        while has_next:
            key, has_next = isolate_particle(filt, d)
            n = n.particles.get(key)
            d += 1
            if n is None:
                return None
        return n

    def _trim(self, n):
        while (
            n.parent is not None
            and n.retain_path == ""
            and len(n.particles) + len(n.subscriptions) + n.shared_len() == 0
        ):
            key = n.key
            n = n.parent
            del n.particles[key]

    def subscribe(self, client, sub: Sub) -> bool:
        """Subscribe (topics.go:303-321)."""
        prefix, _ = isolate_particle(sub.filter, 0)
        if equal_fold(prefix, SHARE_PREFIX):
            group, _ = isolate_particle(sub.filter, 1)
            n = self._set(sub.filter, 2)
            existed = client in n.shared.get(group, {})
            n.shared.setdefault(group, {})[client] = sub
        else:
            n = self._set(sub.filter, 0)
            existed = client in n.subscriptions
            n.subscriptions[client] = sub
        return not existed

    def unsubscribe(self, filt, client) -> bool:
        """Unsubscribe (topics.go:325-349)."""
        d = 2 if filt.startswith(SHARE_PREFIX) else 0
        p = self._seek(filt, d)
        if p is None:
            return False
        prefix, _ = isolate_particle(filt, 0)
        if equal_fold(prefix, SHARE_PREFIX):
            group, _ = isolate_particle(filt, 1)
            g = p.shared.get(group)
            if g is not None:
                g.pop(client, None)
                if not g:
                    del p.shared[group]
        else:
            p.subscriptions.pop(client, None)
        self._trim(p)
        return True

    def retain_message(self, topic, msg_ref, payload_len, retain_flag=True) -> int:
        """RetainMessage (topics.go:354-377)."""
        n = self._set(topic, 0)
        if payload_len > 0:
            n.retain_path = topic
            self.retained[topic] = (msg_ref, payload_len, bool(retain_flag))
            return 1
        out = 0
        pke = self.retained.get(topic)
        if pke is not None and pke[1] > 0 and pke[2]:
            out = -1
        n.retain_path = ""
        self.retained.pop(topic, None)
        self._trim(n)
        return out

    # -- forward match ------------------------------------------------------
    def subscribers(self, topic):
        """Subscribers (topics.go:484-490) -> (subscriptions, shared)."""
        subs = {}
        shared = {}
        self._scan(topic, 0, self.root, subs, shared)
        return subs, shared

    def _scan(self, topic, d, n, subs, shared):
        """scanSubscribers (topics.go:493-518)."""
        if len(topic) == 0:
            return
        key, has_next = isolate_particle(topic, d)
        for part in (key, "+", "#"):
            p = n.particles.get(part)
            if p is None:
                continue
            self._gather(topic, p, subs)
            for g in p.shared.values():  # gatherSharedSubscriptions (topics.go:541-555)
                for client, sub in g.items():
                    shared.setdefault(sub.filter, {})[client] = sub
            wild = p.particles.get("#")
            if wild is not None and part != "#" and part != "+":
                self._gather(topic, wild, subs)
            if has_next:
                self._scan(topic, d + 1, p, subs, shared)

    @staticmethod
    def _gather(topic, p, subs):
        """gatherSubscriptions (topics.go:521-538)."""
        for client, sub in p.subscriptions.items():
            if len(sub.filter) > 0 and topic[0] == "$" and sub.filter[0] in "+#":
                continue
            cls = subs.get(client, sub)
            subs[client] = cls.merge(sub)

    # -- reverse match ------------------------------------------------------
    def messages(self, filt):
        """Messages / scanMessages (topics.go:426-480) -> list of msg_refs."""
        out = []
        self._scan_messages(filt, 0, None, out)
        return out

    def _scan_messages(self, filt, d, n, out):
        if n is None:
            n = self.root
        if len(filt) == 0 or len(self.retained) == 0:
            return
        if "#" not in filt and "+" not in filt:
            if filt in self.retained:
                out.append(self.retained[filt][0])
            return
        key, has_next = isolate_particle(filt, d)
        if key in ("+", "#") or d == -1:
            for adj in list(n.particles.values()):
                if d == 0 and adj.key == SYS_PREFIX:
                    continue
                if not has_next and adj.retain_path != "":
                    if adj.retain_path in self.retained:
                        out.append(self.retained[adj.retain_path][0])
                if has_next or (d >= 0 and key == "#"):
                    self._scan_messages(filt, d + 1, adj, out)
            return
        p = n.particles.get(key)
        if p is not None:
            if has_next:
                self._scan_messages(filt, d + 1, p, out)
                return
            if p.retain_path in self.retained:
                out.append(self.retained[p.retain_path][0])


def is_shared_filter(filt: str) -> bool:
    """IsSharedFilter (topics.go:580-583)."""
    prefix, _ = isolate_particle(filt, 0)
    return equal_fold(prefix, SHARE_PREFIX)


def is_valid_filter(filt: str, for_publish: bool) -> bool:
    """IsValidFilter (topics.go:586-624)."""
    if not for_publish and len(filt) == 0:
        return False
    if for_publish:
        if len(filt) >= len(SYS_PREFIX) and equal_fold(filt[: len(SYS_PREFIX)], SYS_PREFIX):
            return False
        if "+" in filt or "#" in filt:
            return False
    wildhash = filt.find("#")
    if wildhash >= 0 and wildhash != len(filt) - 1:
        return False
    prefix, has_next = isolate_particle(filt, 0)
    if not has_next and equal_fold(prefix, SHARE_PREFIX):
        return False
    if has_next and equal_fold(prefix, SHARE_PREFIX):
        group, has_next2 = isolate_particle(filt, 1)
        if not has_next2:
            return False
        if "+" in group or "#" in group:
            return False
    return True
