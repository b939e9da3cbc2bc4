"""Device-buffer helpers for the host side (bench, sharded node step, tests):
copies out of library-owned device buffers on a stream, and order-independent
per-segment checksums of a CSR held on the device.

The library's device results (mqm_device_result, mqm_device_dense,
mqm_device_messages) are raw device pointers owned by the index; these helpers
copy them into torch tensors with hipMemcpyAsync on the caller's stream (never
the null stream, which would serialise against every other stream)."""

from __future__ import annotations

import ctypes

_HIP = None


def _hip():
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
        _HIP.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                        ctypes.c_void_p]
        _HIP.hipMemcpyAsync.restype = ctypes.c_int
    return _HIP


def _cur(dev):
    import torch

    return torch.cuda.current_stream(dev).cuda_stream


def copy_from_ptr(dst, ptr: int, stream_ptr: int | None = None, count: int | None = None, offset: int = 0):
    """dst[:count] <- the device buffer at ptr (elements of dst's dtype,
    starting `offset` elements in), device to device, queued on stream_ptr
    (default: torch's current stream on dst's device, so torch work queued
    after it is ordered after the copy)."""
    if stream_ptr is None:
        stream_ptr = _cur(dst.device)
    n = dst.numel() if count is None else int(count)
    nbytes = n * dst.element_size()
    if nbytes == 0:
        return dst
    rc = _hip().hipMemcpyAsync(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(ptr + offset * dst.element_size()),
                               ctypes.c_size_t(nbytes), ctypes.c_int(3), ctypes.c_void_p(stream_ptr))
    if rc != 0:
        raise RuntimeError(f"hipMemcpyAsync D2D failed: {rc}")
    return dst


def dev_view_copy(ptr: int, count: int, dtype, device, stream_ptr: int | None = None):
    """A new tensor holding `count` elements of the device buffer at ptr."""
    import torch

    t = torch.empty(max(int(count), 1), dtype=dtype, device=device)[: int(count)]
    return copy_from_ptr(t, ptr, stream_ptr, count)


def mix64(x):
    """splitmix64 finaliser on an int64 torch tensor (wrapping arithmetic)."""
    import torch

    x = x ^ ((x >> 30) & 0x3FFFFFFFF)
    x = x * torch.tensor(-4658895280553007687, dtype=torch.int64, device=x.device)  # 0xBF58476D1CE4E5B9
    x = x ^ ((x >> 27) & 0x1FFFFFFFFF)
    x = x * torch.tensor(-7723592293110705685, dtype=torch.int64, device=x.device)  # 0x94D049BB133111EB
    return x ^ ((x >> 31) & 0x1FFFFFFFF)


def iter_csr_chunks(offs, ents_ptr: int, elem_dtype, max_entries: int = 1 << 28):
    """Walk a CSR whose offsets (int64 tensor [n+1]) are on the device and
    whose entries are a library-owned device buffer, in chunks of whole
    segments of at most max_entries entries (a longer segment is a chunk of
    its own), copying each chunk on torch's current stream into one reused
    buffer.  Yields (lo, hi, a, ents, sid): segments [lo, hi), entries
    [a, a + len(ents)) as int64, and each entry's segment index."""
    import torch

    n = offs.numel() - 1
    dev = offs.device
    o = offs.cpu()
    lo = 0
    buf = None
    while lo < n:
        # the largest hi with o[hi] - o[lo] <= max_entries (at least one segment)
        hi = int(torch.searchsorted(o, o[lo] + max_entries, right=True)) - 1
        hi = min(n, max(hi, lo + 1))
        a, b = int(o[lo]), int(o[hi])
        if b > a:
            if buf is None or buf.numel() < b - a:
                buf = None
                buf = torch.empty(b - a, dtype=elem_dtype, device=dev)
            seg = copy_from_ptr(buf, ents_ptr, None, b - a, offset=a)[: b - a].to(torch.int64)
            cnt = offs[lo + 1:hi + 1] - offs[lo:hi]
            sid = torch.repeat_interleave(torch.arange(lo, hi, device=dev), cnt)
            yield lo, hi, a, seg, sid
        lo = hi


def segment_checksums(offs, ents_ptr: int, elem_dtype, max_entries: int = 1 << 28, fold_index: bool = True):
    """Per-segment order-independent checksum (sum of mix64 of every entry,
    the segment index folded in) of a device CSR (see iter_csr_chunks): the
    temporaries stay bounded whatever the result size.  -> int64 tensor [n]."""
    import torch

    out = torch.zeros(offs.numel() - 1, dtype=torch.int64, device=offs.device)
    for _, _, _, seg, sid in iter_csr_chunks(offs, ents_ptr, elem_dtype, max_entries):
        out.index_add_(0, sid, mix64(seg ^ mix64(sid)) if fold_index else mix64(seg))
    return out
