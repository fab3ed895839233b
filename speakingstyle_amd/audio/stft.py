"""STFT / mel front-end (reference ``audio/stft.py``, ``audio/audio_processing.py``,
``audio/tools.py``).

``TacotronSTFT.mel_spectrogram`` reproduces the reference's conv-basis STFT
(hann window, reflect padding of n_fft/2, hop 256) -> |X| -> mel_basis @ |X| ->
log(clamp(., 1e-5)), plus energy = ||X||_2 over frequency.  The transform runs
on whatever device the input lives on (the reference forces a CUDA round trip,
SURVEY D17).  Griffin-Lim inversion is provided for vocoder-free previews.
"""
from __future__ import annotations

import numpy as np
import torch

from .mel import mel_filterbank


def dynamic_range_compression(x, C=1, clip_val=1e-5):
    return torch.log(torch.clamp(x, min=clip_val) * C)


def dynamic_range_decompression(x, C=1):
    return torch.exp(x) / C


class TacotronSTFT(torch.nn.Module):
    def __init__(self, filter_length=1024, hop_length=256, win_length=1024, n_mel_channels=80,
                 sampling_rate=22050, mel_fmin=0.0, mel_fmax=8000.0):
        super().__init__()
        self.n_fft, self.hop, self.win = filter_length, hop_length, win_length
        self.sampling_rate = sampling_rate
        fb = mel_filterbank(sampling_rate, filter_length, n_mel_channels, mel_fmin, mel_fmax)
        self.register_buffer("mel_basis", torch.from_numpy(fb))
        self.register_buffer("window", torch.hann_window(win_length, periodic=True))

    def magnitudes(self, y: torch.Tensor) -> torch.Tensor:
        spec = torch.stft(y.float(), self.n_fft, self.hop, self.win, window=self.window.to(y.device), center=True,
                          pad_mode="reflect", return_complex=True)
        return spec.abs()  # [B, n_fft/2+1, frames]

    def fft_window(self, device) -> torch.Tensor:
        """The win_length window centred in n_fft (torch.stft's convention), fp32 on ``device``."""
        w = self.window.to(device=device, dtype=torch.float32)
        if self.win < self.n_fft:
            left = (self.n_fft - self.win) // 2
            w = torch.nn.functional.pad(w, (left, self.n_fft - self.win - left))
        return w.contiguous()

    def mel_spectrogram(self, y: torch.Tensor):
        """y [B, N] in [-1, 1] -> (mel [B, n_mel, frames], energy [B, frames]).

        On the GPU (no autograd) one fused HIP kernel does framing + FFT + |X| + mel + log +
        energy (``csrc/k_audio.hip``); the differentiable / CPU path is torch.stft."""
        if not y.requires_grad and not y.is_cuda:  # reference range check (audio/stft.py:169-170), host tensors only
            assert float(y.min()) >= -1 and float(y.max()) <= 1
        from .. import ops

        if y.is_cuda and ops.use_hip(y) and not (torch.is_grad_enabled() and y.requires_grad) \
                and y.shape[-1] > self.n_fft // 2:
            from ..ops import hip

            return hip.logmel(y.float().contiguous(), self.n_fft, self.hop, self.fft_window(y.device),
                              self.mel_basis.to(y.device).contiguous(), 1e-5)
        mag = self.magnitudes(y)
        mel = dynamic_range_compression(torch.matmul(self.mel_basis.to(y.device), mag))
        energy = torch.norm(mag, dim=1)
        return mel, energy


def get_mel_from_wav(audio: np.ndarray, stft: TacotronSTFT):
    """-> (mel [n_mel, T] float32, energy [T] float32) like ``audio/tools.py:8-15``."""
    y = torch.clip(torch.from_numpy(np.asarray(audio, dtype=np.float32)).unsqueeze(0), -1, 1)
    mel, energy = stft.mel_spectrogram(y)
    return mel[0].numpy().astype(np.float32), energy[0].numpy().astype(np.float32)


def griffin_lim(magnitudes: torch.Tensor, stft: TacotronSTFT, n_iters: int = 30) -> torch.Tensor:
    angles = torch.exp(2j * np.pi * torch.rand_like(magnitudes))
    spec = magnitudes * angles
    win = stft.window.to(magnitudes.device)
    y = torch.istft(spec, stft.n_fft, stft.hop, stft.win, window=win)
    for _ in range(n_iters):
        s = torch.stft(y, stft.n_fft, stft.hop, stft.win, window=win, return_complex=True)
        spec = magnitudes * torch.exp(1j * torch.angle(s))
        y = torch.istft(spec, stft.n_fft, stft.hop, stft.win, window=win)
    return y


def inv_mel_spec(mel: torch.Tensor, stft: TacotronSTFT, n_iters: int = 30) -> torch.Tensor:
    """log-mel [n_mel, T] -> waveform via pseudo-inverse mel basis + Griffin-Lim."""
    m = dynamic_range_decompression(mel)
    basis = stft.mel_basis.to(mel.device)
    mag = torch.clamp(torch.linalg.pinv(basis) @ m, min=0.0).unsqueeze(0)
    return griffin_lim(mag, stft, n_iters)[0]
