"""Slaney-style mel filterbank (what ``librosa.filters.mel`` returns with its
defaults: htk=False, norm='slaney'), computed once in numpy."""
from __future__ import annotations

import numpy as np

_F_SP = 200.0 / 3
_MIN_LOG_HZ = 1000.0
_MIN_LOG_MEL = _MIN_LOG_HZ / _F_SP
_LOGSTEP = np.log(6.4) / 27.0


def hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    mel = f / _F_SP
    return np.where(f >= _MIN_LOG_HZ, _MIN_LOG_MEL + np.log(np.maximum(f, 1e-10) / _MIN_LOG_HZ) / _LOGSTEP, mel)


def mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f = _F_SP * m
    return np.where(m >= _MIN_LOG_MEL, _MIN_LOG_HZ * np.exp(_LOGSTEP * (m - _MIN_LOG_MEL)), f)


def mel_filterbank(sr: int, n_fft: int, n_mels: int = 80, fmin: float = 0.0, fmax: float | None = None) -> np.ndarray:
    fmax = sr / 2.0 if fmax is None else float(fmax)
    n_freq = 1 + n_fft // 2
    fft_freqs = np.linspace(0, sr / 2.0, n_freq)
    mel_pts = mel_to_hz(np.linspace(hz_to_mel(fmin), hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_pts)
    ramps = mel_pts[:, None] - fft_freqs[None, :]
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    w = np.maximum(0.0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_pts[2: n_mels + 2] - mel_pts[:n_mels])
    return (w * enorm[:, None]).astype(np.float32)
