"""Fused log-mel kernel (csrc/k_audio.hip) vs the torch.stft TacotronSTFT path in fp32."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from speakingstyle_amd.audio.stft import TacotronSTFT  # noqa: E402
from speakingstyle_amd.ops import hip  # noqa: E402


@pytest.mark.parametrize("n_fft,hop,win,N", [(1024, 256, 1024, 22050), (1024, 256, 800, 5001), (512, 128, 512, 3000),
                                             (2048, 300, 1200, 9999)])
def test_logmel_matches_torch(n_fft, hop, win, N):
    torch.manual_seed(0)
    stft = TacotronSTFT(n_fft, hop, win, 80, 22050, 0.0, 8000.0)
    t = torch.arange(N) / 22050.0
    y = (0.5 * torch.sin(2 * torch.pi * 220 * t) + 0.1 * torch.randn(2, N)).clamp(-1, 1)
    mel_ref, en_ref = stft.mel_spectrogram(y)  # CPU: torch.stft
    stft_g = TacotronSTFT(n_fft, hop, win, 80, 22050, 0.0, 8000.0).to("cuda")
    mel, en = stft_g.mel_spectrogram(y.to("cuda"))  # GPU: fused HIP kernel
    assert mel.shape == mel_ref.shape and en.shape == en_ref.shape
    assert (mel.cpu() - mel_ref).abs().max().item() < 2e-3
    assert ((en.cpu() - en_ref).abs() / en_ref.clamp_min(1e-3)).max().item() < 1e-3


def test_logmel_kernel_is_used():
    stft = TacotronSTFT().to("cuda")
    y = torch.randn(1, 4000, device="cuda").clamp(-1, 1)
    mel, en = hip.logmel(y, 1024, 256, stft.fft_window(y.device), stft.mel_basis.contiguous())
    mel2, en2 = stft.mel_spectrogram(y)
    assert torch.equal(mel, mel2) and torch.equal(en, en2)
