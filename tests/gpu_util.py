"""Helpers shared by the GPU parity tests: canonical (sorted) forms of the
product's and the oracle's batch results so they compare bit-for-bit."""

import numpy as np

from maxmq_amd import capi

CANON = np.dtype([("topic", "<u4"), ("client", "<u4"), ("qos", "u1"), ("no_local", "u1"), ("filter", "<u4"),
                  ("ident", "<i4"), ("rap", "u1"), ("rh", "u1")])
SHARED = np.dtype([("topic", "<u4"), ("filter", "<u4"), ("client", "<u4")])


def _sort(a, keys):
    return a[np.lexsort(tuple(a[k] for k in reversed(keys)))]


def canon_gpu(res):
    n = res.n
    cnt = np.diff(res.offsets).astype(np.int64)
    out = np.zeros(int(cnt.sum()), CANON)
    out["topic"] = np.repeat(np.arange(n, dtype=np.uint32), cnt)
    out["client"] = res.deliveries["client"]
    first, qos, nl = capi.delivery_fields(res.deliveries["packed"])
    out["qos"], out["no_local"] = qos, nl
    info = res.sub_infos(first)
    out["filter"], out["ident"], out["rap"], out["rh"] = info["filter"], info["identifier"], info["rap"], info["rh"]
    scnt = np.diff(res.shared_offsets).astype(np.int64)
    sh = np.zeros(int(scnt.sum()), SHARED)
    sh["topic"] = np.repeat(np.arange(n, dtype=np.uint32), scnt)
    sinfo = res.sub_infos(res.shared, shared=True)
    sh["filter"], sh["client"] = sinfo["filter"], sinfo["client"]
    return _sort(out, ["topic", "client"]), _sort(sh, ["topic", "filter", "client"])


def canon_oracle(doffs, dout, soffs, sout):
    n = len(doffs) - 1
    cnt = np.diff(doffs).astype(np.int64)
    out = np.zeros(int(cnt.sum()), CANON)
    out["topic"] = np.repeat(np.arange(n, dtype=np.uint32), cnt)
    out["client"] = dout["client"]
    out["qos"], out["no_local"] = dout["qos"], dout["no_local"]
    out["filter"], out["ident"], out["rap"], out["rh"] = dout["first_filter"], dout["first_ident"], dout["rap"], dout["rh"]
    scnt = np.diff(soffs).astype(np.int64)
    sh = np.zeros(int(scnt.sum()), SHARED)
    sh["topic"] = np.repeat(np.arange(n, dtype=np.uint32), scnt)
    sh["filter"], sh["client"] = sout["filter"], sout["client"]
    return _sort(out, ["topic", "client"]), _sort(sh, ["topic", "filter", "client"])


def assert_same(gpu, ref, what=""):
    g, r = gpu, ref
    if len(g) != len(r) or not np.array_equal(g, r):
        # locate the first differing topic for a readable failure
        n = min(len(g), len(r))
        bad = np.nonzero(g[:n] != r[:n])[0]
        i = int(bad[0]) if len(bad) else n
        raise AssertionError(f"{what}: {len(g)} vs {len(r)} rows; first difference at row {i}: "
                             f"gpu={g[i] if i < len(g) else None} ref={r[i] if i < len(r) else None}")


IDENT = np.dtype([("topic", "<u4"), ("client", "<u4"), ("filter", "<u4"), ("ident", "<i4")])


def canon_gpu_idents(res):
    """Every delivery's Identifiers map as (topic, client, filter, ident) rows:
    the first-merged pair plus the pairs of the topic's listed sids
    (mqm_result_identifiers), one row per (topic, client, filter)."""
    n = res.n
    cnt = np.diff(res.offsets).astype(np.int64)
    first, _, _ = capi.delivery_fields(res.deliveries["packed"])
    a = np.zeros(int(cnt.sum()), IDENT)
    a["topic"] = np.repeat(np.arange(n, dtype=np.uint32), cnt)
    a["client"] = res.deliveries["client"]
    info = res.sub_infos(first)
    a["filter"], a["ident"] = info["filter"], info["identifier"]
    icnt = np.diff(res.ident_offsets).astype(np.int64)
    b = np.zeros(int(icnt.sum()), IDENT)
    b["topic"] = np.repeat(np.arange(n, dtype=np.uint32), icnt)
    binfo = res.sub_infos(res.idents)
    b["client"], b["filter"], b["ident"] = binfo["client"], binfo["filter"], binfo["identifier"]
    assert (binfo["identifier"] > 0).all()
    return np.unique(np.concatenate([a, b]))


def canon_oracle_idents(ioffs, iout):
    n = len(ioffs) - 1
    cnt = np.diff(ioffs).astype(np.int64)
    a = np.zeros(int(cnt.sum()), IDENT)
    a["topic"] = np.repeat(np.arange(n, dtype=np.uint32), cnt)
    a["client"], a["filter"], a["ident"] = iout["client"], iout["filter"], iout["ident"]
    return np.unique(a)


def dev_tensor(ptr, count, dtype):
    """A copy (device to device) of `count` elements of a library-owned device
    buffer, as a torch tensor on cuda:0."""
    import ctypes

    import torch

    t = torch.empty(max(int(count), 1), dtype=dtype, device="cuda")[: int(count)]
    nbytes = int(count) * t.element_size()
    if nbytes:
        torch.cuda.synchronize()
        hip = ctypes.CDLL("libamdhip64.so")
        rc = hip.hipMemcpy(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes),
                           ctypes.c_int(3))
        assert rc == 0, rc
    return t


def mix64(x):
    """splitmix64 finaliser on an int64 torch tensor (wrapping arithmetic)."""
    import torch

    x = x ^ ((x >> 30) & 0x3FFFFFFFF)
    x = x * torch.tensor(-4658895280553007687, dtype=torch.int64, device=x.device)  # 0xBF58476D1CE4E5B9
    x = x ^ ((x >> 27) & 0x1FFFFFFFFF)
    x = x * torch.tensor(-7723592293110705685, dtype=torch.int64, device=x.device)  # 0x94D049BB133111EB
    return x ^ ((x >> 31) & 0x1FFFFFFFF)


def topic_checksums(offs, ents, chunk=1 << 20):
    """Per-topic order-independent checksum (sum of mix64 of every entry, with
    the topic id folded in) of a dense device CSR: int64 tensor [n]."""
    import torch

    n = offs.numel() - 1
    out = torch.zeros(n, dtype=torch.int64, device=offs.device)
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        a, b = int(offs[lo]), int(offs[hi])
        if a == b:
            continue
        cnt = (offs[lo + 1:hi + 1] - offs[lo:hi])
        tid = torch.repeat_interleave(torch.arange(lo, hi, device=offs.device), cnt)
        h = mix64(ents[a:b] ^ mix64(tid))
        out.index_add_(0, tid, h)
    return out
