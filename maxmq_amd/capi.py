"""ctypes binding of the C ABI in include/mqmatch.h (maxmq_amd/_lib/libmqmatch.so).

This is the binding a Python host would add (the Go host would use the cgo
stub in INTEGRATION.md).  It loads the in-tree library and fails loudly if it
is missing: there is no Python or CPU implementation of the match path.
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MQM_LIB: an alternative build of the same library (e.g. `make sanitize`'s
# host-ASan one for CPU tests); default: the in-tree gfx950 build
LIB_PATH = os.environ.get("MQM_LIB") or os.path.join(_HERE, "_lib", "libmqmatch.so")

MQM_OK = 0
MQM_EINVAL = -1
MQM_ENOMEM = -2
MQM_EHIP = -3
MQM_ELIMIT = -4
MQM_ENODEV = -5
MQM_CFG_AUTOCOMMIT = 1
MQM_CFG_IDENTIFIERS = 2
MQM_CFG_ASYNC_COMMIT = 4
MQM_CFG_BATCHING = 8
MQM_CFG_SERVE = 16
MQM_CFG_FRESH = 32
MQM_DEVICE_NONE = -1

ERRORS = {MQM_EINVAL: "EINVAL", MQM_ENOMEM: "ENOMEM", MQM_EHIP: "EHIP", MQM_ELIMIT: "ELIMIT",
          MQM_ENODEV: "ENODEV"}

# every function include/mqmatch.h declares (checked by tests/test_capi_symbols.py)
EXPORTED = [
    "mqm_create", "mqm_destroy", "mqm_subscribe", "mqm_subscribe_many", "mqm_unsubscribe",
    "mqm_retain_message", "mqm_retained_len", "mqm_commit", "mqm_match_batch", "mqm_subscribers",
    "mqm_batching_policy", "mqm_batching_stats",
    "mqm_match_device", "mqm_result_num_topics", "mqm_result_offsets", "mqm_result_deliveries",
    "mqm_result_shared_offsets", "mqm_result_shared", "mqm_result_sub_info", "mqm_result_shared_info",
    "mqm_result_sub_infos", "mqm_result_free", "mqm_client_name", "mqm_filter_name", "mqm_num_clients", "mqm_is_valid_filter",
    "mqm_is_shared_filter", "mqm_snapshot_stats_get", "mqm_profile_enable", "mqm_profile_read", "mqm_version",
    "mqm_retain_many", "mqm_messages_batch", "mqm_messages_one", "mqm_messages_num_filters", "mqm_messages_offsets",
    "mqm_messages_refs", "mqm_messages_free", "mqm_messages_device", "mqm_identifiers_device",
    "mqm_result_identifiers", "mqm_dense_device", "mqm_gather_shards", "mqm_commit_async", "mqm_commit_poll",
    "mqm_commit_policy", "mqm_commit_state_get", "mqm_snapshot_digest", "mqm_unsubscribe_many", "mqm_load_subscriptions_json",
    "mqm_debug_fault", "mqm_gather_shards_shared", "mqm_match_ctx_create", "mqm_match_ctx_destroy",
    "mqm_match_device_async", "mqm_match_ctx_wait", "mqm_match_ctx_stats", "mqm_match_batch_packed",
    "mqm_result_packed", "mqm_match_batch_runs", "mqm_result_runs", "mqm_result_expand",
    "mqm_serve_policy", "mqm_serve_stats", "mqm_serve_device_us", "mqm_serve_host_us", "mqm_serve_host_max_us",
    "mqm_build_phases_ms", "mqm_build_threads", "mqm_identifiers_early",
    "mqm_result_snapshot_version", "mqm_direct_host_us", "mqm_serve_counters_get", "mqm_fresh_policy",
    "mqm_fresh_stats",
    "mqm_debug_stamp_counts", "mqm_batch_host_us",
]


class MqmError(RuntimeError):
    def __init__(self, fn, rc):
        super().__init__(f"{fn} failed: {ERRORS.get(rc, rc)}")
        self.rc = rc


class Config(C.Structure):
    _fields_ = [("device", C.c_int), ("flags", C.c_uint32)]


class CommitState(C.Structure):
    _fields_ = [("store_version", C.c_uint64), ("snapshot_version", C.c_uint64), ("pending_ops", C.c_uint64),
                ("builds", C.c_uint64), ("last_build_ops", C.c_uint64), ("last_build_ms", C.c_double),
                ("has_snapshot", C.c_int32), ("building", C.c_int32)]


class Subscription(C.Structure):
    _fields_ = [("qos", C.c_uint8), ("no_local", C.c_uint8), ("retain_as_published", C.c_uint8),
                ("retain_handling", C.c_uint8), ("identifier", C.c_int32)]


class SubInfo(C.Structure):
    _fields_ = [("filter", C.c_uint32), ("client", C.c_uint32), ("identifier", C.c_int32), ("qos", C.c_uint8),
                ("no_local", C.c_uint8), ("retain_as_published", C.c_uint8), ("retain_handling", C.c_uint8)]


class DeviceResult(C.Structure):
    _fields_ = [("n_topics", C.c_uint32), ("n_deliveries", C.c_uint64), ("n_shared", C.c_uint64),
                ("starts", C.c_void_p), ("counts", C.c_void_p), ("deliveries", C.c_void_p),
                ("shared_starts", C.c_void_p), ("shared_counts", C.c_void_p),
                ("shared", C.c_void_p), ("n_fallback", C.c_uint32), ("n_big", C.c_uint32),
                ("fallback_why", C.c_uint32 * 5), ("n_merge_small", C.c_uint32), ("n_merge_wave", C.c_uint32),
                ("n_solo_ranges", C.c_uint64), ("n_tier2", C.c_uint32), ("n_tier3", C.c_uint32),
                ("multi_entries", C.c_uint64 * 3), ("n_part", C.c_uint32), ("n_resolve", C.c_uint32),
                ("n_solo", C.c_uint64)]


class DeviceMessages(C.Structure):
    _fields_ = [("n_filters", C.c_uint32), ("n_refs", C.c_uint64), ("offsets", C.c_void_p), ("refs", C.c_void_p),
                ("n_ranges", C.c_uint64), ("n_items", C.c_uint64),
                ("n_skipped", C.c_uint64)]


class DeviceIdentifiers(C.Structure):
    _fields_ = [("n_topics", C.c_uint32), ("n_idents", C.c_uint64), ("offsets", C.c_void_p), ("sids", C.c_void_p)]


class DeviceDense(C.Structure):
    _fields_ = [("n_topics", C.c_uint32), ("n_deliveries", C.c_uint64), ("n_shared", C.c_uint64),
                ("offsets", C.c_void_p), ("deliveries", C.c_void_p), ("shared_offsets", C.c_void_p),
                ("shared", C.c_void_p)]


class ShardPart(C.Structure):
    _fields_ = [("offsets", C.c_void_p), ("deliveries", C.c_void_p), ("client_map", C.c_void_p),
                ("n_map", C.c_uint32)]


class ShardSharedPart(C.Structure):
    _fields_ = [("offsets", C.c_void_p), ("shared", C.c_void_p)]


class SnapshotStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("nodes", "edges", "edge_buckets", "subs", "shared", "height",
                                          "device_bytes", "solo_subs")]


class Profile(C.Structure):
    _fields_ = [("calls", C.c_uint64), ("fallback_topics", C.c_uint64), ("walk_ms", C.c_double),
                ("dedupe_ms", C.c_double), ("total_ms", C.c_double)]


_LIB = None


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                           "(there is no non-HIP implementation of the match path)")
    # One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64 /
    # libhsa-runtime64 (same SONAMEs as /opt/rocm's).  If libmqmatch loaded
    # /opt/rocm's copy first, a later `import torch` would map a second HSA
    # runtime and torch would see no GPU.  Importing torch first makes the
    # dynamic linker bind libmqmatch to torch's copy (SONAME match), so torch
    # tensors, streams and torch.distributed/RCCL share the device with us.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, sz, u32, u64, i32, cp = C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint64, C.c_int32, C.c_char_p
    sigs = {
        "mqm_create": ([C.POINTER(Config), C.POINTER(vp)], C.c_int),
        "mqm_destroy": ([vp], C.c_int),
        "mqm_subscribe": ([vp, cp, sz, cp, sz, C.POINTER(Subscription), C.POINTER(C.c_int)], C.c_int),
        "mqm_subscribe_many": ([vp, sz, vp, vp, vp, vp, vp, vp], C.c_int),
        "mqm_unsubscribe": ([vp, cp, sz, cp, sz, C.POINTER(C.c_int)], C.c_int),
        "mqm_retain_message": ([vp, cp, sz, u64, u32, C.c_int, C.POINTER(C.c_int64)], C.c_int),
        "mqm_retained_len": ([vp, C.POINTER(u64)], C.c_int),
        "mqm_commit": ([vp], C.c_int),
        "mqm_match_batch": ([vp, vp, vp, u32, C.POINTER(vp)], C.c_int),
        "mqm_subscribers": ([vp, cp, sz, C.POINTER(vp)], C.c_int),
        "mqm_batching_policy": ([vp, u32, u32], C.c_int),
        "mqm_batching_stats": ([vp, C.POINTER(u64), C.POINTER(u64)], C.c_int),
        "mqm_match_device": ([vp, vp, vp, u32, vp, C.POINTER(DeviceResult)], C.c_int),
        "mqm_result_num_topics": ([vp], u32),
        "mqm_result_snapshot_version": ([vp], u64),
        "mqm_direct_host_us": ([vp, C.POINTER(C.c_double)], C.c_int),
        "mqm_result_offsets": ([vp], vp),
        "mqm_result_deliveries": ([vp], vp),
        "mqm_result_shared_offsets": ([vp], vp),
        "mqm_result_shared": ([vp], vp),
        "mqm_result_sub_info": ([vp, u32, C.POINTER(SubInfo)], C.c_int),
        "mqm_result_shared_info": ([vp, u32, C.POINTER(SubInfo)], C.c_int),
        "mqm_result_sub_infos": ([vp, C.c_int, vp, sz, vp], C.c_int),
        "mqm_result_free": ([vp], None),
        "mqm_client_name": ([vp, u32, C.c_char_p, sz, C.POINTER(sz)], C.c_int),
        "mqm_filter_name": ([vp, u32, C.c_char_p, sz, C.POINTER(sz)], C.c_int),
        "mqm_num_clients": ([vp, C.POINTER(u32)], C.c_int),
        "mqm_is_valid_filter": ([cp, sz, C.c_int], C.c_int),
        "mqm_is_shared_filter": ([cp, sz], C.c_int),
        "mqm_snapshot_stats_get": ([vp, C.POINTER(SnapshotStats)], C.c_int),
        "mqm_profile_enable": ([vp, C.c_int], C.c_int),
        "mqm_profile_read": ([vp, C.POINTER(Profile)], C.c_int),
        "mqm_version": ([], C.c_char_p),
        "mqm_retain_many": ([vp, sz, vp, vp, vp, vp, vp, vp], C.c_int),
        "mqm_messages_batch": ([vp, vp, vp, u32, C.POINTER(vp)], C.c_int),
        "mqm_messages_one": ([vp, cp, sz, C.POINTER(vp)], C.c_int),
        "mqm_messages_num_filters": ([vp], u32),
        "mqm_messages_offsets": ([vp], vp),
        "mqm_messages_refs": ([vp], vp),
        "mqm_messages_free": ([vp], None),
        "mqm_messages_device": ([vp, vp, vp, u32, vp, C.POINTER(DeviceMessages)], C.c_int),
        "mqm_identifiers_device": ([vp, vp, C.POINTER(DeviceIdentifiers)], C.c_int),
        "mqm_result_identifiers": ([vp, C.POINTER(vp), C.POINTER(vp)], C.c_int),
        "mqm_dense_device": ([vp, vp, C.POINTER(DeviceDense)], C.c_int),
        "mqm_gather_shards": ([u32, u32, C.POINTER(ShardPart), vp, vp, vp], C.c_int),
        "mqm_unsubscribe_many": ([vp, sz, vp, vp, vp, vp, vp], C.c_int),
        "mqm_load_subscriptions_json": ([vp, C.c_char_p, sz, C.POINTER(u64), C.POINTER(u64)], C.c_int),
        "mqm_commit_async": ([vp], C.c_int),
        "mqm_commit_poll": ([vp, C.c_int, C.POINTER(C.c_int)], C.c_int),
        "mqm_commit_policy": ([vp, u64, u32], C.c_int),
        "mqm_commit_state_get": ([vp, C.POINTER(CommitState)], C.c_int),
        "mqm_snapshot_digest": ([vp, C.POINTER(u64)], C.c_int),
        "mqm_debug_fault": ([vp, C.c_int, C.c_int], C.c_int),
        "mqm_gather_shards_shared": ([u32, u32, C.POINTER(ShardSharedPart), vp, vp, vp], C.c_int),
        "mqm_match_ctx_create": ([vp, C.POINTER(vp)], C.c_int),
        "mqm_match_ctx_destroy": ([vp], C.c_int),
        "mqm_match_device_async": ([vp, vp, vp, u32, vp], C.c_int),
        "mqm_match_ctx_wait": ([vp, C.POINTER(DeviceResult)], C.c_int),
        "mqm_match_ctx_stats": ([vp, C.POINTER(u64)], C.c_int),
        "mqm_match_batch_packed": ([vp, vp, vp, u32, C.POINTER(vp)], C.c_int),
        "mqm_result_packed": ([vp], vp),
        "mqm_match_batch_runs": ([vp, vp, vp, u32, C.POINTER(vp)], C.c_int),
        "mqm_result_runs": ([vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), C.POINTER(u64)], C.c_int),
        "mqm_result_expand": ([vp, u32, u32, vp, vp], C.c_int),
        "mqm_serve_policy": ([vp, u32, u32], C.c_int),
        "mqm_serve_stats": ([vp, C.POINTER(u64), C.POINTER(u64), C.POINTER(u64)], C.c_int),
        "mqm_serve_counters_get": ([vp, C.POINTER(u64 * 8)], C.c_int),
        "mqm_fresh_policy": ([vp, C.c_int], C.c_int),
        "mqm_fresh_stats": ([vp, C.POINTER(C.c_uint64 * 9)], C.c_int),
        "mqm_debug_stamp_counts": ([C.POINTER(u64), C.POINTER(u64), C.POINTER(u64)], C.c_int),
        "mqm_batch_host_us": ([vp, C.POINTER(C.c_double)], C.c_int),
        "mqm_serve_device_us": ([vp, vp], C.c_int),
        "mqm_serve_host_us": ([vp, vp], C.c_int),
        "mqm_serve_host_max_us": ([vp, vp], C.c_int),
        "mqm_build_phases_ms": ([vp, vp], C.c_int),
        "mqm_build_threads": ([C.c_uint32], C.c_int),
        "mqm_identifiers_early": ([vp, C.c_int], C.c_int),
    }
    missing = [name for name in sigs if getattr(L, name, None) is None]
    if missing:  # a library older than this file: fail here, not with an AttributeError mid-call
        raise RuntimeError(f"{LIB_PATH} lacks {', '.join(missing)}: a stale build — "
                           f"rebuild it with `make -C maxmq_amd/csrc`")
    for name, (args, res) in sigs.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _LIB = L
    return L


def check(fn, rc):
    if rc != MQM_OK:
        raise MqmError(fn, rc)
    return rc


def b(s) -> bytes:
    return s.encode("utf-8", "surrogateescape") if isinstance(s, str) else bytes(s)


DELIVERY_DTYPE = np.dtype([("client", "<u4"), ("packed", "<u4")])
SUB_INFO_DTYPE = np.dtype([("filter", "<u4"), ("client", "<u4"), ("identifier", "<i4"), ("qos", "u1"),
                           ("no_local", "u1"), ("rap", "u1"), ("rh", "u1")])


def delivery_fields(packed: np.ndarray):
    """-> (first_sub, qos, no_local) arrays from the packed word (mqmatch.h)."""
    packed = packed.astype(np.uint32, copy=False)
    return packed & 0x0FFFFFFF, (packed >> 28) & 3, (packed >> 30) & 1
