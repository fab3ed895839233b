"""WAV I/O + resampling without librosa/soundfile (scipy only)."""
from __future__ import annotations

from math import gcd

import numpy as np
from scipy.io import wavfile
from scipy.signal import resample_poly


def read_wav(path: str, target_sr: int | None = None):
    """-> (float32 mono in [-1, 1], sr); resamples with a polyphase filter if asked."""
    sr, data = wavfile.read(path)
    if data.dtype == np.int16:
        x = data.astype(np.float32) / 32768.0
    elif data.dtype == np.int32:
        x = data.astype(np.float32) / 2147483648.0
    elif data.dtype == np.uint8:
        x = (data.astype(np.float32) - 128.0) / 128.0
    else:
        x = data.astype(np.float32)
    if x.ndim == 2:
        x = x.mean(axis=1)
    if target_sr and target_sr != sr:
        g = gcd(int(sr), int(target_sr))
        x = resample_poly(x, target_sr // g, sr // g).astype(np.float32)
        sr = target_sr
    return x, sr


def write_wav(path: str, sr: int, wav):
    wav = np.asarray(wav)
    if wav.dtype != np.int16:
        peak = max(1e-8, float(np.abs(wav).max())) if wav.size else 1.0
        wav = (np.clip(wav / max(peak, 1.0), -1, 1) * 32767).astype(np.int16)
    wavfile.write(path, int(sr), wav)
