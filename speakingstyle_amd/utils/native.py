"""ctypes bindings of the native host-runtime library (``csrc/host_*.cpp`` ->
``speakingstyle_amd/_lib/libssamd_host.so``, built by ``csrc/build.py``).

Pure host code (no GPU): used by the data pipeline.  When the library is absent
the callers fall back to numpy (same results; ``tests/test_native_host.py``).
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional

import numpy as np

_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib", "libssamd_host.so")
_lib = None
_tried = False


def lib() -> Optional[ctypes.CDLL]:
    global _lib, _tried
    if not _tried:
        _tried = True
        if os.path.exists(_PATH):
            h = ctypes.CDLL(_PATH)
            h.ssamd_pad_rows.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int64), ctypes.c_int,
                                         ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int]
            h.ssamd_pad_rows.restype = ctypes.c_int
            _lib = h
    return _lib


def pad_rows(arrays: List[np.ndarray], max_rows: Optional[int] = None, nthreads: int = 8) -> Optional[np.ndarray]:
    """Stack ``arrays`` (same dtype and trailing shape) along a new axis 0, zero-padding
    axis 0 of each to ``max_rows``.  Returns None if the native library is unavailable."""
    h = lib()
    if h is None or not arrays:
        return None
    first = np.asarray(arrays[0])
    tail, dt = first.shape[1:], first.dtype
    arrs = [np.ascontiguousarray(a, dtype=dt) for a in arrays]
    if any(a.shape[1:] != tail for a in arrs):
        return None
    rows = np.array([a.shape[0] for a in arrs], dtype=np.int64)
    max_rows = int(rows.max()) if max_rows is None else int(max_rows)
    out = np.empty((len(arrs), max_rows) + tail, dtype=dt)
    row_bytes = int(np.prod(tail, dtype=np.int64)) * dt.itemsize if tail else dt.itemsize
    ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    rc = h.ssamd_pad_rows(ptrs, rows.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), len(arrs), row_bytes, max_rows,
                          out.ctypes.data, int(nthreads))
    if rc != 0:
        raise ValueError("sequence longer than max_len")
    return out
