"""Host buffers for the direct host path (include/mpcqp.h mpcqp_host_register): a caller's
array copied into its own page-aligned, page-padded numpy buffer, which mpcqp_host_register
accepts (it refuses unaligned starts: pinning works on whole pages, and a page shared by two
registrations left the HIP runtime a stale mapping that faulted a later copy)."""
from __future__ import annotations

import mmap

import numpy as np


def page_aligned(a: np.ndarray) -> np.ndarray:
    """a C-contiguous copy of `a` whose buffer starts on a page and owns every page it touches
    (padded to the next page boundary; the padding bytes belong to nothing else)"""
    page = mmap.PAGESIZE
    a = np.ascontiguousarray(a)
    span = max(1, -(-a.nbytes // page)) * page
    raw = np.zeros(span + page, np.uint8)
    off = (-raw.ctypes.data) % page
    out = raw[off:off + a.nbytes].view(a.dtype).reshape(a.shape)
    out[...] = a
    return out


def page_aligned_empty(shape, dtype) -> np.ndarray:
    """page_aligned(np.zeros(shape, dtype))"""
    return page_aligned(np.zeros(shape, dtype))
