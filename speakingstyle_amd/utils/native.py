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
            dp = ctypes.POINTER(ctypes.c_double)
            d, i64 = ctypes.c_double, ctypes.c_int64
            h.ssamd_dio_frames.argtypes = [i64, d, d]
            h.ssamd_dio_frames.restype = i64
            h.ssamd_dio.argtypes = [dp, i64, d, d, d, d, d, d, dp, dp]
            h.ssamd_dio.restype = ctypes.c_int
            h.ssamd_stonemask.argtypes = [dp, i64, d, dp, dp, i64, dp]
            h.ssamd_stonemask.restype = ctypes.c_int
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


def _require():
    h = lib()
    if h is None:
        raise RuntimeError(f"native host library missing ({_PATH}); build it with `python csrc/build.py`")
    return h


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def dio(x: np.ndarray, fs: int, f0_floor: float = 71.0, f0_ceil: float = 800.0, channels_in_octave: float = 2.0,
        frame_period: float = 5.0, allowed_range: float = 0.1):
    """DIO F0 estimation (csrc/host_f0.cpp), pyworld ``dio`` call contract:
    returns ``(f0 [Hz, 0 = unvoiced], temporal_positions [s])`` as float64 arrays."""
    h = _require()
    x = np.ascontiguousarray(x, dtype=np.float64)
    nf = int(h.ssamd_dio_frames(len(x), float(fs), float(frame_period)))
    f0 = np.zeros(nf, np.float64)
    t = np.zeros(nf, np.float64)
    rc = h.ssamd_dio(_dptr(x), len(x), float(fs), float(frame_period), float(f0_floor), float(f0_ceil),
                     float(channels_in_octave), float(allowed_range), _dptr(f0), _dptr(t))
    if rc != 0:
        raise ValueError("dio: invalid arguments")
    return f0, t


def stonemask(x: np.ndarray, f0: np.ndarray, temporal_positions: np.ndarray, fs: int) -> np.ndarray:
    """StoneMask F0 refinement (csrc/host_f0.cpp), pyworld ``stonemask`` call contract."""
    h = _require()
    x = np.ascontiguousarray(x, dtype=np.float64)
    f0 = np.ascontiguousarray(f0, dtype=np.float64)
    t = np.ascontiguousarray(temporal_positions, dtype=np.float64)
    if f0.shape != t.shape:
        raise ValueError("stonemask: f0 and temporal_positions must have the same length")
    out = np.zeros_like(f0)
    rc = h.ssamd_stonemask(_dptr(x), len(x), float(fs), _dptr(t), _dptr(f0), len(f0), _dptr(out))
    if rc != 0:
        raise ValueError("stonemask: invalid arguments")
    return out
