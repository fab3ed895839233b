"""HiFi-GAN's mel front-end (reference ``hifigan/meldataset.py:49-72``).

Differs from the FastSpeech2 ``TacotronSTFT`` framing on purpose, like the reference:
reflect padding of (n_fft - hop) / 2 on each side and an *uncentred* STFT, so a
segment of N samples gives exactly N / hop frames; |X| = sqrt(re^2 + im^2 + 1e-9);
log(clamp(mel, 1e-5)).  The loss mel may use a different ``fmax`` (``fmax_for_loss``,
None = Nyquist).  Mel bases and windows are cached per (fmax, device).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

from ..audio.mel import mel_filterbank

_cache: Dict[Tuple, Tuple[torch.Tensor, torch.Tensor]] = {}


def _basis_window(sr, n_fft, n_mels, fmin, fmax, win, device):
    key = (sr, n_fft, n_mels, fmin, fmax, win, str(device))
    hit = _cache.get(key)
    if hit is None:
        basis = torch.from_numpy(mel_filterbank(sr, n_fft, n_mels, fmin, fmax)).float().to(device)
        hit = (basis, torch.hann_window(win, device=device))
        _cache[key] = hit
    return hit


def mel_spectrogram(y: torch.Tensor, n_fft: int, num_mels: int, sampling_rate: int, hop_size: int, win_size: int,
                    fmin: float, fmax: Optional[float]) -> torch.Tensor:
    """y [B, N] (or [N]) in [-1, 1] -> log-mel [B, num_mels, N // hop]."""
    if y.dim() == 1:
        y = y.unsqueeze(0)
    basis, window = _basis_window(sampling_rate, n_fft, num_mels, fmin, fmax, win_size, y.device)
    p = (n_fft - hop_size) // 2
    yp = torch.nn.functional.pad(y.float().unsqueeze(1), (p, p), mode="reflect").squeeze(1)
    spec = torch.stft(yp, n_fft, hop_length=hop_size, win_length=win_size, window=window, center=False,
                      normalized=False, onesided=True, return_complex=True)
    mag = torch.sqrt(spec.real.pow(2) + spec.imag.pow(2) + 1e-9)
    return torch.log(torch.clamp(torch.matmul(basis, mag), min=1e-5))


def mel_for(h, y: torch.Tensor, loss: bool = False) -> torch.Tensor:
    """Mel of ``y`` with the vocoder config ``h`` (``loss``: the ``fmax_for_loss`` variant)."""
    fmax = h.get("fmax_for_loss") if loss else h.fmax
    return mel_spectrogram(y, h.n_fft, h.num_mels, h.sampling_rate, h.hop_size, h.win_size, h.fmin, fmax)
