"""maxmq_amd — MI355X-native MQTT publish-routing matcher.

Python host mirror of the reference's ``TopicsIndex`` API
(vendor/github.com/mochi-co/mqtt/v2/topics.go:284-624 in gsalomao/maxmq) over
the C ABI in include/mqmatch.h.  Method names, argument meaning and return
values follow the reference:

    idx = TopicsIndex()                       # NewTopicsIndex  (topics.go:291)
    idx.subscribe("cl1", Subscription("a/+", qos=1))   -> bool (topics.go:303)
    idx.unsubscribe("a/+", "cl1")             -> bool           (topics.go:325)
    idx.retain_message(topic, ref, payload_len, retain=True) -> 1/0/-1 (:354)
    idx.subscribers("a/b")                    -> Subscribers    (topics.go:484)
    idx.match_batch(bytes, offsets)           -> BatchResult    (GPU batch)
    idx.messages("a/#")                       -> [message refs] (topics.go:426)
    idx.messages_batch(bytes, offsets)        -> (offsets, refs) (GPU batch)

Matching runs only on the GPU (libmqmatch.so); there is no Python or CPU
match path.  Without a device, ``TopicsIndex(device=None)`` still offers the
host store (mutation semantics) and raises on matching.
"""

from __future__ import annotations

import ctypes as C
import weakref
from dataclasses import dataclass, field

import numpy as np

from . import capi
from .capi import MqmError, b, check, lib

__all__ = ["TopicsIndex", "Subscription", "Subscribers", "BatchResult", "MqmError", "is_valid_filter",
           "is_shared_filter"]


@dataclass
class Subscription:
    """packets.Subscription (packets/packets.go:168-178)."""

    filter: str
    qos: int = 0
    identifier: int = 0
    no_local: bool = False
    retain_as_published: bool = False
    retain_handling: int = 0
    identifiers: dict | None = None

    def _c(self):
        return capi.Subscription(self.qos, int(self.no_local), int(self.retain_as_published),
                                 self.retain_handling, self.identifier)


@dataclass
class Subscribers:
    """Subscribers (topics.go:248-252): merged non-shared subscriptions keyed by
    client, and shared subscriptions keyed by filter then client."""

    subscriptions: dict = field(default_factory=dict)
    shared: dict = field(default_factory=dict)
    shared_selected: dict = field(default_factory=dict)

    def select_shared(self):
        """SelectShared (topics.go:255-268) with a deterministic policy: the
        lowest client id of each shared filter (the reference picks the first
        Go-map iteration entry, i.e. an arbitrary one)."""
        self.shared_selected = {}
        for filt in sorted(self.shared):
            subs = self.shared[filt]
            client = min(subs)
            sub = subs[client]
            cur = self.shared_selected.get(client, sub)
            self.shared_selected[client] = _merge(cur, sub)

    def merge_shared_selected(self):
        """MergeSharedSelected (topics.go:273-282)."""
        for client, sub in self.shared_selected.items():
            cur = self.subscriptions.get(client, sub)
            self.subscriptions[client] = _merge(cur, sub)


def _merge(s: Subscription, n: Subscription) -> Subscription:
    """Subscription.Merge (packets/packets.go:250-270)."""
    out = Subscription(s.filter, s.qos, s.identifier, s.no_local, s.retain_as_published, s.retain_handling,
                       dict(s.identifiers) if s.identifiers is not None else {s.filter: s.identifier})
    if n.identifier > 0:
        out.identifiers[n.filter] = n.identifier
    out.qos = max(out.qos, n.qos)
    out.no_local = out.no_local or n.no_local
    return out


class BatchResult:
    """Host copy of one batch's CSR result (mqm_result)."""

    def __init__(self, index: "TopicsIndex", handle):
        L = lib()
        self._index = index
        self._h = handle
        n = L.mqm_result_num_topics(handle)
        self.n = n
        # the store version of the snapshot it was matched on (mqm_result_snapshot_version)
        self.snapshot_version = int(L.mqm_result_snapshot_version(handle))

        def arr(ptr, count, dtype):
            if count == 0 or not ptr:
                return np.zeros(0, dtype)
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)),
                                         shape=(count * np.dtype(dtype).itemsize,)).view(dtype).copy()

        self.offsets = arr(L.mqm_result_offsets(handle), n + 1, np.uint64)
        self.shared_offsets = arr(L.mqm_result_shared_offsets(handle), n + 1, np.uint64)
        # the runs form (mqm_match_batch_runs): solo runs of the snapshot's words
        # + merged winners, expanded here (mqm_result_expand) into plain rows
        self.runs_form = False
        ro, rr, rw, nw = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_uint64()
        expanded = None
        if n and L.mqm_result_runs(handle, C.byref(ro), C.byref(rr), C.byref(rw), C.byref(nw)) == 0:
            self.runs_form = True
            self.run_offsets = arr(ro.value, n + 1, np.uint64)
            self.runs = arr(rr.value, 2 * int(self.run_offsets[-1]), np.uint32).reshape(-1, 2)  # (off, count)
            self.winner_offsets = self.offsets
            eo = np.zeros(n + 1, np.uint64)
            check("mqm_result_expand", L.mqm_result_expand(handle, 0, n, eo.ctypes.data_as(C.c_void_p), None))
            expanded = np.zeros(int(eo[-1]), np.uint32)
            check("mqm_result_expand", L.mqm_result_expand(handle, 0, n, eo.ctypes.data_as(C.c_void_p),
                                                           expanded.ctypes.data_as(C.c_void_p)))
            self.offsets = eo
        nd = int(self.offsets[-1]) if n else 0
        ns = int(self.shared_offsets[-1]) if n else 0
        self.shared = arr(L.mqm_result_shared(handle), ns, np.uint32)
        self.packed_only = bool(nd) and not L.mqm_result_deliveries(handle) and bool(L.mqm_result_packed(handle))
        if self.packed_only:  # mqm_match_batch_packed: the client is the first-merged subscription's
            packed = expanded if expanded is not None else arr(L.mqm_result_packed(handle), nd, np.uint32)
            self.deliveries = np.zeros(nd, capi.DELIVERY_DTYPE)
            self.deliveries["packed"] = packed
            self.deliveries["client"] = self.sub_infos(packed & 0x0FFFFFFF)["client"]
        else:
            self.deliveries = arr(L.mqm_result_deliveries(handle), nd, capi.DELIVERY_DTYPE)
        # Identifiers support (MQM_CFG_IDENTIFIERS): per topic, the sids of the
        # gathered subscriptions with Identifier > 0
        self.ident_offsets = self.idents = None
        io, ids = C.c_void_p(), C.c_void_p()
        if n and L.mqm_result_identifiers(handle, C.byref(io), C.byref(ids)) == 0:
            self.ident_offsets = arr(io.value, n + 1, np.uint64)
            self.idents = arr(ids.value, int(self.ident_offsets[-1]), np.uint32)

    def close(self):
        if self._h:
            lib().mqm_result_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sub_info(self, sub: int) -> capi.SubInfo:
        info = capi.SubInfo()
        check("mqm_result_sub_info", lib().mqm_result_sub_info(self._h, sub, C.byref(info)))
        return info

    def shared_info(self, sub: int) -> capi.SubInfo:
        info = capi.SubInfo()
        check("mqm_result_shared_info", lib().mqm_result_shared_info(self._h, sub, C.byref(info)))
        return info

    def sub_infos(self, subs: np.ndarray, shared: bool = False) -> np.ndarray:
        """Vectorised sub_info: -> structured array (capi.SUB_INFO_DTYPE)."""
        subs = np.ascontiguousarray(subs, dtype=np.uint32)
        out = np.zeros(len(subs), capi.SUB_INFO_DTYPE)
        check("mqm_result_sub_infos", lib().mqm_result_sub_infos(
            self._h, int(shared), subs.ctypes.data_as(C.c_void_p), len(subs), out.ctypes.data_as(C.c_void_p)))
        return out

    def identifiers(self, i: int) -> dict:
        """Topic i's Identifiers maps (packets.go:250-259) by client id:
        {client: {filter id: identifier}}, the first-merged pair included.
        Needs an index created with identifiers=True."""
        if self.idents is None:
            raise MqmError("mqm_result_identifiers", capi.MQM_EINVAL)
        first, _, _ = capi.delivery_fields(self.deliveries["packed"][self.offsets[i]:self.offsets[i + 1]])
        out = {}
        if len(first):
            for c, r in zip(self.deliveries["client"][self.offsets[i]:self.offsets[i + 1]], self.sub_infos(first)):
                out[int(c)] = {int(r["filter"]): int(r["identifier"])}
        sids = self.idents[self.ident_offsets[i]:self.ident_offsets[i + 1]]
        if len(sids):
            for r in self.sub_infos(sids):
                out[int(r["client"])][int(r["filter"])] = int(r["identifier"])
        return out

    def subscribers(self, i: int) -> Subscribers:
        """Topic i's result in the reference's Subscribers shape (names
        resolved).  Identifiers is the full map when the index was created
        with identifiers=True, else the first-merged filter's pair only."""
        out = Subscribers()
        first, qos, nl = capi.delivery_fields(self.deliveries["packed"][self.offsets[i]:self.offsets[i + 1]])
        clients = self.deliveries["client"][self.offsets[i]:self.offsets[i + 1]]
        ids = self.identifiers(i) if self.idents is not None else None
        for c, f, q, n in zip(clients, first, qos, nl):
            info = self.sub_info(int(f))
            fname = self._index.filter_name(info.filter)
            idmap = ({self._index.filter_name(k): v for k, v in ids[int(c)].items()} if ids is not None
                     else {fname: info.identifier})
            out.subscriptions[self._index.client_name(int(c))] = Subscription(
                fname, int(q), info.identifier, bool(n), bool(info.retain_as_published), info.retain_handling,
                idmap)
        for sid in self.shared[self.shared_offsets[i]:self.shared_offsets[i + 1]]:
            info = self.shared_info(int(sid))
            fname = self._index.filter_name(info.filter)
            out.shared.setdefault(fname, {})[self._index.client_name(info.client)] = Subscription(
                fname, info.qos, info.identifier, bool(info.no_local), bool(info.retain_as_published),
                info.retain_handling)
        return out


class TopicsIndex:
    """TopicsIndex (topics.go:285) backed by the MI355X matcher."""

    def __init__(self, device: int | None = 0, autocommit: bool = True, identifiers: bool = False,
                 async_commit: bool = False, batching: bool = False, serve: bool = False, fresh: bool = False):
        """identifiers=True: match_batch / subscribers also return the full
        Subscription.Identifiers maps (an extra GPU pass per batch).
        async_commit=True: mutations are logged and snapshots are rebuilt by a
        background builder (commit_async / commit_poll / commit_policy).
        batching=True: concurrent subscribers() calls are gathered into GPU
        batches by a collector thread (MQM_CFG_BATCHING).
        serve=True: subscribers() calls go to a persistent GPU server through
        a ring of pinned slots (MQM_CFG_SERVE; no launch per call).
        fresh=True (with async_commit): subscribers() returns the store's
        current subscriptions without waiting for a rebuild (MQM_CFG_FRESH)."""
        L = lib()
        cfg = capi.Config(capi.MQM_DEVICE_NONE if device is None else device,
                          (capi.MQM_CFG_AUTOCOMMIT if autocommit else 0) |
                          (capi.MQM_CFG_IDENTIFIERS if identifiers else 0) |
                          (capi.MQM_CFG_ASYNC_COMMIT if async_commit else 0) |
                          (capi.MQM_CFG_BATCHING if batching else 0) |
                          (capi.MQM_CFG_SERVE if serve else 0) |
                          (capi.MQM_CFG_FRESH if fresh else 0))
        h = C.c_void_p()
        check("mqm_create", L.mqm_create(C.byref(cfg), C.byref(h)))
        self._h = h
        self.device = device
        self._fresh = bool(fresh)
        self._ctxs = weakref.WeakSet()  # live MatchContexts (destroyed before the index)

    @property
    def fresh(self) -> bool:
        """created with fresh=True (MQM_CFG_FRESH)"""
        return self._fresh

    def fresh_policy(self, correct_calls: bool):
        """MQM_CFG_FRESH: subscribers() corrected for every mutation (True,
        the default) or the published snapshot's view (False).  Switched on
        again, the corrections start with a published snapshot that holds
        every mutation made while off (at once when the published one does;
        commit_async() then commit_poll(wait=True) publishes one)."""
        check("mqm_fresh_policy", lib().mqm_fresh_policy(self._h, int(bool(correct_calls))))

    def fresh_stats(self) -> dict:
        """the fresh overlay: clients held (touched since the previous
        snapshot), operations applied per copy, applier rounds, calls
        corrected and the time in their read sections"""
        v = (C.c_uint64 * 9)()
        check("mqm_fresh_stats", lib().mqm_fresh_stats(self._h, C.byref(v)))
        return {"held_clients": v[0], "ops_applied": v[1], "rounds": v[2], "calls_corrected": v[3],
                "read_ns": v[4], "scan_ns": v[5], "max_batch_age_ns": v[6], "max_round_ns": v[7],
                "max_copy_wait_ns": v[8]}

    def batching_policy(self, max_batch: int = 0, linger_us: int = 0):
        check("mqm_batching_policy", lib().mqm_batching_policy(self._h, max_batch, linger_us))

    def serve_policy(self, grid: int = 0, idle_us: int = 0):
        check("mqm_serve_policy", lib().mqm_serve_policy(self._h, grid, idle_us))

    def serve_stats(self):
        """(calls served in the ring, calls that took the batch path, server launches)"""
        a, b_, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        check("mqm_serve_stats", lib().mqm_serve_stats(self._h, C.byref(a), C.byref(b_), C.byref(c)))
        return a.value, b_.value, c.value

    def serve_counters(self) -> dict:
        """the served path's counters (mqm_serve_counters): served, fallbacks,
        launches, stale decodes, forced relaunches, slot / result timeouts,
        ring slots handed on past a caller that gave up before posting"""
        v = (C.c_uint64 * 8)()
        check("mqm_serve_counters_get", lib().mqm_serve_counters_get(self._h, C.byref(v)))
        keys = ("served", "fallbacks", "launches", "stale", "forced", "slot_timeouts", "result_timeouts",
                "skipped_slots")
        return dict(zip(keys, (int(x) for x in v)))

    def serve_device_us(self) -> float:
        """mean device time per served call, claim to published result (us)"""
        v = (C.c_double * 4)()
        check("mqm_serve_device_us", lib().mqm_serve_device_us(self._h, v))
        return {"total": v[0], "stage_keys": v[1], "walk": v[2], "emit_publish": v[3]}

    def serve_host_us(self):
        """mean host time per served call since the previous read (us): entry
        -> posted, posted -> result seen, seen -> returned; share that slept"""
        v = (C.c_double * 4)()
        check("mqm_serve_host_us", lib().mqm_serve_host_us(self._h, v))
        return {"post": v[0], "wait": v[1], "collect": v[2], "slept_share": v[3]}

    def identifiers_early(self, on: bool = True):
        """device matches compute the Identifiers lists beside their merges
        (mqm_identifiers_early); identifiers_device then only collects"""
        check("mqm_identifiers_early", lib().mqm_identifiers_early(self._h, 1 if on else 0))

    def serve_host_max_us(self):
        """the longest served call per host phase since the previous read (us),
        and the number of calls over 10 ms"""
        v = (C.c_double * 8)()
        check("mqm_serve_host_max_us", lib().mqm_serve_host_max_us(self._h, v))
        names = ("front", "server_check", "slot_post", "result_wait", "result_block", "fallback")
        return {"max": dict(zip(names, v[0:6])), "calls_over_10ms": int(v[6])}

    def direct_host_us(self):
        """single-topic calls on the direct path since the previous read (us):
        mean and max per phase (front buffer, context, launch + wait, result)"""
        v = (C.c_double * 9)()
        check("mqm_direct_host_us", lib().mqm_direct_host_us(self._h, v))
        names = ("front", "context", "kernel", "result")
        return {"mean": dict(zip(names, v[0:4])), "max": dict(zip(names, v[4:8])), "calls": int(v[8])}

    def batching_stats(self):
        """(batches run, topics they carried) of the MQM_CFG_BATCHING collector"""
        b, t = C.c_uint64(), C.c_uint64()
        check("mqm_batching_stats", lib().mqm_batching_stats(self._h, C.byref(b), C.byref(t)))
        return b.value, t.value

    def close(self):
        if getattr(self, "_h", None):
            for c in list(getattr(self, "_ctxs", ())):  # mqm_destroy refuses while a context lives
                c.close()
            check("mqm_destroy", lib().mqm_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- mutation -------------------------------------------------------------
    def subscribe(self, client: str, sub: Subscription) -> bool:
        c, f = b(client), b(sub.filter)
        out = C.c_int()
        cs = sub._c()
        check("mqm_subscribe", lib().mqm_subscribe(self._h, c, len(c), f, len(f), C.byref(cs), C.byref(out)))
        return bool(out.value)

    def subscribe_workload(self, w) -> np.ndarray:
        """Bulk Subscribe of a tools.mqgen.Workload in filter order; -> is_new[]."""
        return self.subscribe_many(w.clients, w.filters, w.qos, w.no_local, w.rap, w.rh, w.ident)

    def subscribe_many(self, clients, filters, qos, no_local=0, rap=0, rh=0, ident=0) -> np.ndarray:
        """Bulk Subscribe of (clients[i], filters[i]) (tools.mqgen.Strings) in order; -> is_new[]."""
        n = len(filters)
        subs = np.zeros(n, dtype=np.dtype([("qos", "u1"), ("nl", "u1"), ("rap", "u1"), ("rh", "u1"),
                                           ("ident", "<i4")]))
        subs["qos"], subs["nl"], subs["rap"], subs["rh"], subs["ident"] = qos, no_local, rap, rh, ident
        is_new = np.zeros(n, np.uint8)
        p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
        check("mqm_subscribe_many", lib().mqm_subscribe_many(
            self._h, n, p(clients.data), p(clients.offs), p(filters.data), p(filters.offs), p(subs), p(is_new)))
        return is_new

    def unsubscribe(self, filt: str, client: str) -> bool:
        f, c = b(filt), b(client)
        out = C.c_int()
        check("mqm_unsubscribe", lib().mqm_unsubscribe(self._h, f, len(f), c, len(c), C.byref(out)))
        return bool(out.value)

    def load_subscriptions_json(self, blob: bytes) -> tuple:
        """Server.loadSubscriptions over persisted storage.Subscription JSON
        records (array or one object per line); -> (n_loaded, n_new)."""
        n, fresh = C.c_uint64(), C.c_uint64()
        rc = lib().mqm_load_subscriptions_json(self._h, blob, len(blob), C.byref(n), C.byref(fresh))
        if rc != capi.MQM_OK:
            err = MqmError("mqm_load_subscriptions_json", rc)
            err.n_loaded = int(n.value)
            raise err
        return int(n.value), int(fresh.value)

    def unsubscribe_many(self, filters, clients) -> np.ndarray:
        """Bulk Unsubscribe of (filters[i], clients[i]) (tools.mqgen.Strings) in order; -> existed[]."""
        n = len(filters)
        out = np.zeros(n, np.uint8)
        p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
        check("mqm_unsubscribe_many", lib().mqm_unsubscribe_many(
            self._h, n, p(filters.data), p(filters.offs), p(clients.data), p(clients.offs), p(out)))
        return out

    def retain_message(self, topic: str, message_ref: int, payload_len: int, retain: bool = True) -> int:
        t = b(topic)
        out = C.c_int64()
        check("mqm_retain_message",
              lib().mqm_retain_message(self._h, t, len(t), message_ref, payload_len, int(retain), C.byref(out)))
        return int(out.value)

    def retain_many(self, topics, refs: np.ndarray, payload_lens: np.ndarray | None = None,
                    retain_flags: np.ndarray | None = None) -> np.ndarray:
        """Bulk RetainMessage of topics (a tools.mqgen.Strings) in order; -> results[]."""
        n = len(topics)
        refs = np.ascontiguousarray(refs, dtype=np.uint64)
        pl = np.ones(n, np.uint32) if payload_lens is None else np.ascontiguousarray(payload_lens, dtype=np.uint32)
        rf = None if retain_flags is None else np.ascontiguousarray(retain_flags, dtype=np.uint8)
        out = np.zeros(n, np.int64)
        p = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)  # noqa: E731
        check("mqm_retain_many", lib().mqm_retain_many(
            self._h, n, p(topics.data), p(topics.offs), p(refs), p(pl), p(rf), p(out)))
        return out

    def retained_len(self) -> int:
        out = C.c_uint64()
        check("mqm_retained_len", lib().mqm_retained_len(self._h, C.byref(out)))
        return int(out.value)

    def commit(self):
        check("mqm_commit", lib().mqm_commit(self._h))

    # -- incremental commits (async_commit=True) ---------------------------------
    def commit_async(self):
        """Hand the logged mutations to the background builder; returns at once."""
        check("mqm_commit_async", lib().mqm_commit_async(self._h))

    def commit_poll(self, wait: bool = False) -> bool:
        """Publish the newest finished snapshot (wait: for every submitted log)."""
        out = C.c_int()
        check("mqm_commit_poll", lib().mqm_commit_poll(self._h, int(wait), C.byref(out)))
        return bool(out.value)

    def commit_policy(self, max_ops: int = 0, max_ms: int = 0):
        """Periodic rebuild: auto-submit after max_ops logged mutations or max_ms."""
        check("mqm_commit_policy", lib().mqm_commit_policy(self._h, max_ops, max_ms))

    def commit_state(self) -> dict:
        st = capi.CommitState()
        check("mqm_commit_state_get", lib().mqm_commit_state_get(self._h, C.byref(st)))
        return {n: getattr(st, n) for n, _ in capi.CommitState._fields_}

    def snapshot_digest(self) -> int:
        out = C.c_uint64()
        check("mqm_snapshot_digest", lib().mqm_snapshot_digest(self._h, C.byref(out)))
        return int(out.value)

    # -- names ------------------------------------------------------------------
    def _name(self, fn, i):
        n = C.c_size_t()
        check(fn, getattr(lib(), fn)(self._h, i, None, 0, C.byref(n)))
        buf = C.create_string_buffer(max(n.value, 1))
        check(fn, getattr(lib(), fn)(self._h, i, buf, n.value, C.byref(n)))
        return buf.raw[: n.value].decode("utf-8", "surrogateescape")

    def client_name(self, i: int) -> str:
        return self._name("mqm_client_name", i)

    def filter_name(self, i: int) -> str:
        return self._name("mqm_filter_name", i)

    def num_clients(self) -> int:
        out = C.c_uint32()
        check("mqm_num_clients", lib().mqm_num_clients(self._h, C.byref(out)))
        return out.value

    def profile(self, on: bool):
        check("mqm_profile_enable", lib().mqm_profile_enable(self._h, int(on)))

    def profile_read(self) -> dict:
        p = capi.Profile()
        check("mqm_profile_read", lib().mqm_profile_read(self._h, C.byref(p)))
        return {n: getattr(p, n) for n, _ in capi.Profile._fields_}

    def snapshot_stats(self) -> dict:
        st = capi.SnapshotStats()
        check("mqm_snapshot_stats_get", lib().mqm_snapshot_stats_get(self._h, C.byref(st)))
        return {n: int(getattr(st, n)) for n, _ in capi.SnapshotStats._fields_}

    # -- matching -------------------------------------------------------------------
    def match_batch(self, data: np.ndarray, offs: np.ndarray) -> BatchResult:
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        h = C.c_void_p()
        check("mqm_match_batch", lib().mqm_match_batch(
            self._h, data.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(C.c_void_p), len(offs) - 1,
            C.byref(h)))
        return BatchResult(self, h)

    def match_batch_packed(self, data: np.ndarray, offs: np.ndarray) -> BatchResult:
        """mqm_match_batch_packed (4-B deliveries); the BatchResult resolves
        each delivery's client through its first-merged subscription."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        h = C.c_void_p()
        check("mqm_match_batch_packed", lib().mqm_match_batch_packed(
            self._h, data.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(C.c_void_p), len(offs) - 1,
            C.byref(h)))
        return BatchResult(self, h)

    def match_batch_runs(self, data: np.ndarray, offs: np.ndarray) -> BatchResult:
        """mqm_match_batch_runs (solo deliveries as runs of the snapshot's
        packed words, merged winners explicit); the BatchResult expands them
        into plain rows and keeps the raw form (run_offsets, runs,
        winner_offsets)."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        h = C.c_void_p()
        check("mqm_match_batch_runs", lib().mqm_match_batch_runs(
            self._h, data.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(C.c_void_p), len(offs) - 1,
            C.byref(h)))
        return BatchResult(self, h)

    def subscribers_result(self, topic: str) -> BatchResult:
        """mqm_subscribers' raw single-topic result (ids, not names)"""
        t = b(topic)
        h = C.c_void_p()
        check("mqm_subscribers", lib().mqm_subscribers(self._h, t, len(t), C.byref(h)))
        return BatchResult(self, h)

    def subscribers(self, topic: str) -> Subscribers:
        t = b(topic)
        h = C.c_void_p()
        check("mqm_subscribers", lib().mqm_subscribers(self._h, t, len(t), C.byref(h)))
        r = BatchResult(self, h)
        try:
            return r.subscribers(0)
        finally:
            r.close()

    def messages_batch(self, data: np.ndarray, offs: np.ndarray):
        """Messages (topics.go:426-480) for a batch of filters on the GPU ->
        (offsets[n+1], refs): filter i's retained message refs are
        refs[offsets[i]:offsets[i+1]] (order within a filter unspecified)."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        h = C.c_void_p()
        L = lib()
        check("mqm_messages_batch", L.mqm_messages_batch(
            self._h, data.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(C.c_void_p), len(offs) - 1, C.byref(h)))
        try:
            n = L.mqm_messages_num_filters(h)

            def arr(ptr, count):
                if count == 0 or not ptr:
                    return np.zeros(0, np.uint64)
                return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint64)), shape=(count,)).copy()

            o = arr(L.mqm_messages_offsets(h), n + 1)
            r = arr(L.mqm_messages_refs(h), int(o[-1]) if n else 0)
            return o, r
        finally:
            L.mqm_messages_free(h)

    def messages(self, filt: str) -> list:
        """Messages(filter) (topics.go:426): the retained message refs, sorted."""
        f = b(filt)
        o, r = self.messages_batch(np.frombuffer(f, np.uint8) if f else np.zeros(0, np.uint8),
                                   np.array([0, len(f)], np.uint64))
        return sorted(int(x) for x in r)

    def messages_device(self, d_bytes_ptr: int, d_offs_ptr: int, n: int, stream_ptr: int = 0) -> capi.DeviceMessages:
        out = capi.DeviceMessages()
        check("mqm_messages_device", lib().mqm_messages_device(
            self._h, C.c_void_p(d_bytes_ptr), C.c_void_p(d_offs_ptr), n, C.c_void_p(stream_ptr), C.byref(out)))
        return out

    def identifiers_device(self, stream_ptr: int = 0) -> capi.DeviceIdentifiers:
        """Identifiers support for the last match_device batch (its topic
        buffers must still hold it): per-topic sids with Identifier > 0."""
        out = capi.DeviceIdentifiers()
        check("mqm_identifiers_device", lib().mqm_identifiers_device(self._h, C.c_void_p(stream_ptr), C.byref(out)))
        return out

    def dense_device(self, stream_ptr: int = 0) -> capi.DeviceDense:
        """Dense CSR (no gaps) of the last match_device result, on the device."""
        out = capi.DeviceDense()
        check("mqm_dense_device", lib().mqm_dense_device(self._h, C.c_void_p(stream_ptr), C.byref(out)))
        return out

    def match_context(self) -> "MatchContext":
        """A context of the queued device API (several batches in flight)."""
        c = MatchContext(self)
        self._ctxs.add(c)
        return c

    def match_device(self, d_bytes_ptr: int, d_offs_ptr: int, n: int, stream_ptr: int = 0) -> capi.DeviceResult:
        """Device-resident batch (pointers from e.g. torch tensors); the result's
        device buffers are owned by the index and valid until the next match."""
        out = capi.DeviceResult()
        check("mqm_match_device", lib().mqm_match_device(self._h, C.c_void_p(d_bytes_ptr), C.c_void_p(d_offs_ptr),
                                                         n, C.c_void_p(stream_ptr), C.byref(out)))
        return out


class MatchContext:
    """A caller-owned context of the queued device API (mqm_match_device_async
    / mqm_match_ctx_wait): one batch in flight at a time; contexts on
    different streams overlap.  The result's device buffers belong to the
    context and stay valid until its next submit."""

    def __init__(self, index: "TopicsIndex"):
        self._index = index  # keeps the index alive
        self._c = C.c_void_p()
        check("mqm_match_ctx_create", lib().mqm_match_ctx_create(index._h, C.byref(self._c)))

    def submit(self, d_bytes_ptr: int, d_offs_ptr: int, n: int, stream_ptr: int = 0):
        check("mqm_match_device_async", lib().mqm_match_device_async(
            self._c, C.c_void_p(d_bytes_ptr), C.c_void_p(d_offs_ptr), n, C.c_void_p(stream_ptr)))

    def wait(self) -> capi.DeviceResult:
        out = capi.DeviceResult()
        check("mqm_match_ctx_wait", lib().mqm_match_ctx_wait(self._c, C.byref(out)))
        return out

    def requeued(self) -> int:
        v = C.c_uint64()
        check("mqm_match_ctx_stats", lib().mqm_match_ctx_stats(self._c, C.byref(v)))
        return int(v.value)

    def close(self):
        if self._c:
            lib().mqm_match_ctx_destroy(self._c)
            self._c = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def gather_shards(n_topics: int, parts, d_out_offsets_ptr: int, d_out_ptr: int, stream_ptr: int = 0):
    """mqm_gather_shards: node-wide dense CSR of a subscriber-sharded match.
    parts: (offsets_ptr, deliveries_ptr, client_map_ptr or 0, n_map) per shard,
    all device pointers on the current device.  Synchronises the stream."""
    arr = (capi.ShardPart * max(1, len(parts)))()
    for i, (o, d, m, nm) in enumerate(parts):
        arr[i] = capi.ShardPart(o, d, m or None, nm)
    check("mqm_gather_shards", lib().mqm_gather_shards(n_topics, len(parts), arr, C.c_void_p(stream_ptr),
                                                       C.c_void_p(d_out_offsets_ptr), C.c_void_p(d_out_ptr)))


def gather_shards_shared(n_topics: int, parts, d_out_offsets_ptr: int, d_out_ptr: int, stream_ptr: int = 0):
    """mqm_gather_shards_shared: node-wide shared candidates of a
    subscriber-sharded match.  parts: (shared_offsets_ptr, shared_ids_ptr) per
    shard (device pointers); entries come out as shard << 28 | shard-local id."""
    arr = (capi.ShardSharedPart * max(1, len(parts)))()
    for i, (o, d) in enumerate(parts):
        arr[i] = capi.ShardSharedPart(o, d)
    check("mqm_gather_shards_shared", lib().mqm_gather_shards_shared(
        n_topics, len(parts), arr, C.c_void_p(stream_ptr), C.c_void_p(d_out_offsets_ptr), C.c_void_p(d_out_ptr)))


def is_valid_filter(filt: str, for_publish: bool) -> bool:
    """IsValidFilter (topics.go:586-624)."""
    f = b(filt)
    return bool(lib().mqm_is_valid_filter(f, len(f), int(for_publish)))


def is_shared_filter(filt: str) -> bool:
    """IsSharedFilter (topics.go:580-583)."""
    f = b(filt)
    return bool(lib().mqm_is_shared_filter(f, len(f)))
