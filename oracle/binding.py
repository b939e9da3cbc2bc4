"""oracle/binding.py — TEST INFRASTRUCTURE ONLY.

ctypes wrapper over oracle/_build/libmochi_ref.so (the C restatement of the
reference ``TopicsIndex``).  Importable only from tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg: it is the checker, never the product.
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

DELIVERY_DTYPE = np.dtype(
    [("client", "<u4"), ("first_filter", "<u4"), ("first_ident", "<i4"), ("qos", "u1"), ("no_local", "u1"),
     ("rap", "u1"), ("rh", "u1")]
)
SHARED_DTYPE = np.dtype([("filter", "<u4"), ("client", "<u4"), ("qos", "u1"), ("pad", "u1", (3,))])
IDENT_DTYPE = np.dtype([("client", "<u4"), ("filter", "<u4"), ("ident", "<i4")])


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("topics", "topic_bytes", "probes", "visits", "gathered",
                                          "deliveries", "shared")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "_build", "libmochi_ref.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = C.CDLL(path)
        vp, u32, u64, cp = C.c_void_p, C.c_uint32, C.c_uint64, C.c_char_p
        L.oref_new.restype = vp
        L.oref_free.argtypes = [vp]
        L.oref_subscribe.argtypes = [vp, cp, u32, cp, u32, C.c_uint8, C.c_uint8, C.c_uint8, C.c_uint8, C.c_int32]
        L.oref_subscribe.restype = C.c_int
        L.oref_subscribe_many.argtypes = [vp, u64] + [vp] * 9
        L.oref_unsubscribe.argtypes = [vp, cp, u32, cp, u32]
        L.oref_unsubscribe.restype = C.c_int
        L.oref_retain.argtypes = [vp, cp, u32, u64, u32, C.c_uint8]
        L.oref_retain.restype = C.c_int64
        L.oref_num_clients.argtypes = [vp]
        L.oref_num_clients.restype = u32
        L.oref_num_filters.argtypes = [vp]
        L.oref_num_filters.restype = u32
        L.oref_filter_name.argtypes = [vp, u32, C.c_char_p, u32]
        L.oref_filter_name.restype = u32
        L.oref_client_name.argtypes = [vp, u32, C.c_char_p, u32]
        L.oref_client_name.restype = u32
        L.oref_retain_many.argtypes = [vp, u64, vp, vp, vp, u32]
        L.oref_retain_many.restype = None
        L.oref_retained_len.argtypes = [vp]
        L.oref_retained_len.restype = u64
        L.oref_match_counts.argtypes = [vp, vp, vp, u32, C.c_int, vp, vp, C.POINTER(Stats)]
        L.oref_match_fill.argtypes = [vp, vp, vp, u32, C.c_int, vp, vp, vp, vp]
        L.oref_match_ident_counts.argtypes = [vp, vp, vp, u32, C.c_int, vp]
        L.oref_match_ident_fill.argtypes = [vp, vp, vp, u32, C.c_int, vp, vp]
        L.oref_messages_counts.argtypes = [vp, vp, vp, u32, C.c_int, vp]
        L.oref_messages_fill.argtypes = [vp, vp, vp, u32, C.c_int, vp, vp]
        L.oref_isolate_particle.argtypes = [cp, u32, C.c_int, C.POINTER(u32), C.POINTER(u32)]
        L.oref_isolate_particle.restype = C.c_int
        _LIB = L
    return _LIB


def _b(s) -> bytes:
    return s.encode("utf-8", "surrogateescape") if isinstance(s, str) else bytes(s)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def isolate_particle(s, d):
    b = _b(s)
    st, ln = C.c_uint32(), C.c_uint32()
    hn = lib().oref_isolate_particle(b, len(b), d, C.byref(st), C.byref(ln))
    return b[st.value : st.value + ln.value].decode("utf-8", "surrogateescape"), bool(hn)


class OracleIndex:
    """The C restatement of TopicsIndex (topics.go:284-699)."""

    def __init__(self):
        self._L = lib()
        self._h = self._L.oref_new()

    def close(self):
        if self._h:
            self._L.oref_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def subscribe(self, client, filt, qos=0, no_local=False, rap=False, rh=0, ident=0) -> bool:
        c, f = _b(client), _b(filt)
        return bool(self._L.oref_subscribe(self._h, c, len(c), f, len(f), qos, int(no_local), int(rap), rh, ident))

    def subscribe_workload(self, w):
        """Bulk Subscribe of a tools.mqgen.Workload, in filter order."""
        arrs = [np.ascontiguousarray(a) for a in (w.clients.data, w.clients.offs, w.filters.data, w.filters.offs,
                                                  w.qos, w.no_local, w.rap, w.rh, w.ident)]
        self._L.oref_subscribe_many(self._h, len(w.filters.offs) - 1, *[_ptr(a) for a in arrs])

    def unsubscribe(self, filt, client) -> bool:
        c, f = _b(client), _b(filt)
        return bool(self._L.oref_unsubscribe(self._h, f, len(f), c, len(c)))

    def retain_message(self, topic, msg_ref, payload_len, retain_flag=True) -> int:
        t = _b(topic)
        return int(self._L.oref_retain(self._h, t, len(t), msg_ref, payload_len, int(retain_flag)))

    def retain_many(self, topics, refs: np.ndarray, payload_len: int = 1):
        """RetainMessage of every topic of a tools.mqgen.Strings, in order."""
        refs = np.ascontiguousarray(refs, dtype=np.uint64)
        self._L.oref_retain_many(self._h, len(topics), _ptr(topics.data), _ptr(topics.offs), _ptr(refs), payload_len)

    def retained_len(self) -> int:
        return int(self._L.oref_retained_len(self._h))

    def num_clients(self):
        return int(self._L.oref_num_clients(self._h))

    def num_filters(self):
        return int(self._L.oref_num_filters(self._h))

    def filter_name(self, i):
        n = self._L.oref_filter_name(self._h, i, None, 0)
        buf = C.create_string_buffer(max(n, 1))
        self._L.oref_filter_name(self._h, i, buf, n)
        return buf.raw[:n].decode("utf-8", "surrogateescape")

    def client_name(self, i):
        n = self._L.oref_client_name(self._h, i, None, 0)
        buf = C.create_string_buffer(max(n, 1))
        self._L.oref_client_name(self._h, i, buf, n)
        return buf.raw[:n].decode("utf-8", "surrogateescape")

    def match_counts(self, data: np.ndarray, offs: np.ndarray, nthreads=1):
        n = len(offs) - 1
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        dc = np.zeros(n, np.uint32)
        sc = np.zeros(n, np.uint32)
        st = Stats()
        self._L.oref_match_counts(self._h, _ptr(data), _ptr(offs), n, nthreads, _ptr(dc), _ptr(sc), C.byref(st))
        return dc, sc, st.as_dict()

    def match(self, data: np.ndarray, offs: np.ndarray, nthreads=1):
        """-> (doffs, deliveries, soffs, shared, stats): CSR over topics."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        dc, sc, st = self.match_counts(data, offs, nthreads)
        n = len(offs) - 1
        doffs = np.zeros(n + 1, np.uint64)
        soffs = np.zeros(n + 1, np.uint64)
        doffs[1:] = np.cumsum(dc, dtype=np.uint64)
        soffs[1:] = np.cumsum(sc, dtype=np.uint64)
        dout = np.zeros(int(doffs[-1]), DELIVERY_DTYPE)
        sout = np.zeros(int(soffs[-1]), SHARED_DTYPE)
        self._L.oref_match_fill(self._h, _ptr(data), _ptr(offs), n, nthreads, _ptr(doffs), _ptr(dout),
                                _ptr(soffs), _ptr(sout))
        return doffs, dout, soffs, sout, st

    def identifiers(self, data: np.ndarray, offs: np.ndarray, nthreads=1):
        """Subscription.Identifiers of every delivery (packets.go:250-258) ->
        (ioffs, entries IDENT_DTYPE): per topic, (client, filter, ident) sorted
        by (client, filter)."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        n = len(offs) - 1
        cnt = np.zeros(n, np.uint32)
        self._L.oref_match_ident_counts(self._h, _ptr(data), _ptr(offs), n, nthreads, _ptr(cnt))
        ioffs = np.zeros(n + 1, np.uint64)
        ioffs[1:] = np.cumsum(cnt, dtype=np.uint64)
        out = np.zeros(int(ioffs[-1]), IDENT_DTYPE)
        self._L.oref_match_ident_fill(self._h, _ptr(data), _ptr(offs), n, nthreads, _ptr(ioffs), _ptr(out))
        return ioffs, out

    def messages(self, data: np.ndarray, offs: np.ndarray, nthreads=1):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        n = len(offs) - 1
        cnt = np.zeros(n, np.uint32)
        self._L.oref_messages_counts(self._h, _ptr(data), _ptr(offs), n, nthreads, _ptr(cnt))
        moffs = np.zeros(n + 1, np.uint64)
        moffs[1:] = np.cumsum(cnt, dtype=np.uint64)
        out = np.zeros(int(moffs[-1]), np.uint64)
        self._L.oref_messages_fill(self._h, _ptr(data), _ptr(offs), n, nthreads, _ptr(moffs), _ptr(out))
        return moffs, out
