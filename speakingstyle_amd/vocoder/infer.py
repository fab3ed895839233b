"""HiFi-GAN inference entry points (reference ``hifigan/inference.py:37-90`` and
``hifigan/inference_e2e.py:34-85``).

* ``from_wavs``: every wav in a directory -> HiFi-GAN mel (``vocoder/mel.py``) -> waveform,
  written as ``{name}_generated.wav`` (copy-synthesis / vocoder check);
* ``from_mels``: every ``.npy`` mel ([n_mels, T] or [1, n_mels, T], e.g. FastSpeech2 output)
  -> ``{name}_generated_e2e.wav``.

On the GPU the generator runs channel-last through the HIP kernels (``Generator.infer``:
3-tap upsampler GEMMs, fused ResBlock layers, int16 written by the conv_post kernel); a
directory is processed in length-sorted batches of ``batch_size`` utterances (padded to the
batch's longest mel, outputs trimmed per utterance) instead of one utterance at a time.
Checkpoints load with ``weights_only=True``; the config is ``config.json`` next to the
checkpoint (reference behaviour) unless given.
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import numpy as np
import torch

from ..audio.io import read_wav, write_wav
from ..models import hifigan as H
from ..utils.model import vocoder_config
from .mel import mel_for


def load_generator(checkpoint_file: str, device, config: Optional[str] = None):
    cfg = config or os.path.join(os.path.dirname(checkpoint_file), "config.json")
    h = vocoder_config(cfg if os.path.exists(cfg) else None)
    g = H.Generator(h)
    state = torch.load(checkpoint_file, map_location="cpu", weights_only=True)
    g.load_state_dict(state["generator"])
    g.eval().fold_weight_norm().to(device)
    g.requires_grad_(False)
    return g, h


@torch.no_grad()
def vocode(g, h, mels: List[torch.Tensor], device, batch_size: int = 16) -> List[np.ndarray]:
    """[n_mels, T_i] fp32 mels -> int16 waveforms of T_i * hop samples each."""
    hop = h.hop_size
    order = sorted(range(len(mels)), key=lambda i: -mels[i].shape[-1])
    out: List[Optional[np.ndarray]] = [None] * len(mels)
    for s in range(0, len(order), batch_size):
        idx = order[s:s + batch_size]
        T = max(mels[i].shape[-1] for i in idx)
        batch = torch.full((len(idx), T, mels[idx[0]].shape[0]), float(np.log(1e-5)), dtype=torch.float32)
        for k, i in enumerate(idx):
            batch[k, : mels[i].shape[-1]] = mels[i].t()
        x = batch.to(device)
        if x.is_cuda:
            pcm = g.infer(x.to(torch.bfloat16).contiguous(), int16_scale=32768.0,
                          lengths=[mels[i].shape[-1] for i in idx]).cpu().numpy()
        else:
            w = g(x.transpose(1, 2)).squeeze(1)
            pcm = (w * 32768.0).clamp(-32768, 32767).to(torch.int16).numpy()
        for k, i in enumerate(idx):
            out[i] = pcm[k, : mels[i].shape[-1] * hop].astype(np.int16)
    return out  # type: ignore[return-value]


def _listdir(d: str, ext: str) -> List[str]:
    return sorted(f for f in os.listdir(d) if f.endswith(ext))


def from_wavs(input_wavs_dir: str, output_dir: str, checkpoint_file: str, device=None, config=None,
              batch_size: int = 16) -> List[str]:
    device = device or torch.device("cuda" if torch.cuda.is_available() else "cpu")
    g, h = load_generator(checkpoint_file, device, config)
    names = _listdir(input_wavs_dir, ".wav")
    mels = []
    for n in names:
        wav, _ = read_wav(os.path.join(input_wavs_dir, n), h.sampling_rate)
        mels.append(mel_for(h, torch.from_numpy(wav).float().clamp(-1, 1))[0])
    return _write(names, vocode(g, h, mels, device, batch_size), output_dir, "_generated", h)


def from_mels(input_mels_dir: str, output_dir: str, checkpoint_file: str, device=None, config=None,
              batch_size: int = 16) -> List[str]:
    device = device or torch.device("cuda" if torch.cuda.is_available() else "cpu")
    g, h = load_generator(checkpoint_file, device, config)
    names = _listdir(input_mels_dir, ".npy")
    mels = []
    for n in names:
        m = torch.from_numpy(np.load(os.path.join(input_mels_dir, n), allow_pickle=False)).float()
        mels.append(m.reshape(-1, m.shape[-1]) if m.dim() == 3 else m)
    return _write(names, vocode(g, h, mels, device, batch_size), output_dir, "_generated_e2e", h)


def _write(names, wavs, output_dir, suffix, h) -> List[str]:
    os.makedirs(output_dir, exist_ok=True)
    paths = []
    for n, w in zip(names, wavs):
        p = os.path.join(output_dir, os.path.splitext(n)[0] + suffix + ".wav")
        write_wav(p, h.sampling_rate, w)
        paths.append(p)
    return paths
