"""ctypes wrapper over tools/_build/libmqgen.so (synthetic workload generator).

Bench/test infrastructure.  ``generate(config, **overrides)`` returns a
``Workload`` of numpy arrays; strings are (bytes, offsets) pairs so they can be
handed to both the product C-ABI and the oracle without re-encoding.
"""

from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class _Params(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64),
        ("n_filters", C.c_uint64),
        ("n_topics", C.c_uint64),
        ("max_depth", C.c_uint32),
        ("n_clients", C.c_uint32),
        ("p_plus", C.c_double),
        ("p_hash", C.c_double),
        ("p_shared", C.c_double),
        ("p_dollar_topic", C.c_double),
        ("p_instantiate", C.c_double),
        ("topic_zipf_s", C.c_double),
        ("token_zipf_s", C.c_double),
        ("vocab", C.c_uint32 * 8),
        ("depth_w", C.c_double * 32),
        ("n_root_hash", C.c_uint32),
        ("pad_", C.c_uint32),
        ("client_lo", C.c_uint64),
        ("client_hi", C.c_uint64),
    ]


class _Strings(C.Structure):
    _fields_ = [("n", C.c_uint64), ("bytes", C.POINTER(C.c_char)), ("offs", C.POINTER(C.c_uint64))]


class _Workload(C.Structure):
    _fields_ = [
        ("filters", _Strings),
        ("clients", _Strings),
        ("client_ids", C.POINTER(C.c_uint32)),
        ("qos", C.POINTER(C.c_uint8)),
        ("no_local", C.POINTER(C.c_uint8)),
        ("rap", C.POINTER(C.c_uint8)),
        ("rh", C.POINTER(C.c_uint8)),
        ("ident", C.POINTER(C.c_int32)),
        ("topics", _Strings),
    ]


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "_build", "libmqgen.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C tools` (or __graft_entry__.build())")
        _LIB = C.CDLL(path)
        _LIB.mqgen_default_params.argtypes = [C.c_int, C.POINTER(_Params)]
        _LIB.mqgen_generate.argtypes = [C.POINTER(_Params), C.POINTER(_Workload)]
        _LIB.mqgen_generate.restype = C.c_int
        _LIB.mqgen_free.argtypes = [C.POINTER(_Workload)]
    return _LIB


@dataclass
class Strings:
    data: np.ndarray  # uint8
    offs: np.ndarray  # uint64, n+1

    def __len__(self):
        return len(self.offs) - 1

    def __getitem__(self, i) -> str:
        return bytes(self.data[self.offs[i] : self.offs[i + 1]]).decode("utf-8", "surrogateescape")

    @staticmethod
    def from_list(items) -> "Strings":
        enc = [s.encode("utf-8", "surrogateescape") if isinstance(s, str) else bytes(s) for s in items]
        offs = np.zeros(len(enc) + 1, dtype=np.uint64)
        if enc:
            offs[1:] = np.cumsum([len(e) for e in enc], dtype=np.uint64)
        data = np.frombuffer(b"".join(enc), dtype=np.uint8).copy() if enc else np.zeros(0, np.uint8)
        return Strings(data, offs)


@dataclass
class Workload:
    params: dict
    filters: Strings
    clients: Strings
    client_ids: np.ndarray
    qos: np.ndarray
    no_local: np.ndarray
    rap: np.ndarray
    rh: np.ndarray
    ident: np.ndarray
    topics: Strings


def _copy_strings(s: _Strings) -> Strings:
    n = int(s.n)
    offs = np.ctypeslib.as_array(s.offs, shape=(n + 1,)).copy()
    nb = int(offs[-1])
    data = np.ctypeslib.as_array(C.cast(s.bytes, C.POINTER(C.c_uint8)), shape=(max(nb, 1),))[:nb].copy()
    return Strings(data, offs)


def default_params(config: int) -> dict:
    p = _Params()
    _lib().mqgen_default_params(config, C.byref(p))
    return {name: (list(getattr(p, name)) if name in ("vocab", "depth_w") else getattr(p, name))
            for name, _ in _Params._fields_}


def generate(config: int, **overrides) -> Workload:
    lib = _lib()
    p = _Params()
    lib.mqgen_default_params(config, C.byref(p))
    for k, v in overrides.items():
        if k in ("vocab", "depth_w"):
            arr = getattr(p, k)
            for i, x in enumerate(v):
                arr[i] = x
        else:
            setattr(p, k, v)
    w = _Workload()
    rc = lib.mqgen_generate(C.byref(p), C.byref(w))
    if rc != 0:
        raise ValueError(f"mqgen_generate failed: {rc}")
    try:
        nf = int(w.filters.n)

        def arr(ptr, n):
            return np.ctypeslib.as_array(ptr, shape=(max(n, 1),))[:n].copy()

        params = {name: (list(getattr(p, name)) if name in ("vocab", "depth_w") else getattr(p, name))
                  for name, _ in _Params._fields_}
        return Workload(
            params=params,
            filters=_copy_strings(w.filters),
            clients=_copy_strings(w.clients),
            client_ids=arr(w.client_ids, nf),
            qos=arr(w.qos, nf),
            no_local=arr(w.no_local, nf),
            rap=arr(w.rap, nf),
            rh=arr(w.rh, nf),
            ident=arr(w.ident, nf),
            topics=_copy_strings(w.topics),
        )
    finally:
        lib.mqgen_free(C.byref(w))
