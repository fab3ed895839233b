"""HiFi-GAN training data (reference ``hifigan/meldataset.py:75-168``).

* filelists: ``name|...`` lines -> ``{wavs_dir}/{name}.wav`` (``get_dataset_filelist``);
* ``split``: random ``segment_size`` crops (train) or whole utterances (validation);
* ``fine_tuning``: the input mel is the ground-truth-aligned mel predicted by the acoustic
  model (``{base_mels_path}/{name}.npy``, [n_mels, T] or [1, n_mels, T]) and the audio crop
  follows the mel crop; the waveform is then NOT peak-normalised (reference behaviour);
* returns (mel, audio, filename, loss_mel) where loss_mel uses ``fmax_for_loss``.
* ``synthetic_n``: that many generated tone segments (plumbing runs without a corpus).
"""
from __future__ import annotations

import math
import os
import random
from typing import List, Optional, Tuple

import numpy as np
import torch

from ..audio.io import read_wav
from .mel import mel_for


def read_filelist(list_path: str, wavs_dir: str) -> List[str]:
    with open(list_path, encoding="utf-8") as f:
        return [os.path.join(wavs_dir, ln.split("|")[0] + ".wav") for ln in f.read().split("\n") if ln.strip()]


def get_dataset_filelist(train_list: str, valid_list: str, wavs_dir: str) -> Tuple[List[str], List[str]]:
    return read_filelist(train_list, wavs_dir), read_filelist(valid_list, wavs_dir)


class MelDataset(torch.utils.data.Dataset):
    def __init__(self, files: List[str], h, split: bool = True, shuffle: bool = True, fine_tuning: bool = False,
                 base_mels_path: Optional[str] = None, synthetic_n: int = 0, seed: int = 1234):
        self.files = list(files)
        self.h = h
        self.split = split
        self.fine_tuning = fine_tuning
        self.base_mels_path = base_mels_path
        self.synthetic_n = synthetic_n
        if shuffle:
            random.Random(seed).shuffle(self.files)

    def __len__(self):
        return self.synthetic_n or len(self.files)

    def _synthetic(self, i):
        n = self.h.segment_size * (1 if self.split else 2)
        t = np.arange(n) / self.h.sampling_rate
        rng = np.random.default_rng(i)
        wav = 0.3 * np.sin(2 * np.pi * (110 + 30 * (i % 7)) * t) + 0.01 * rng.standard_normal(n)
        return wav.astype(np.float32), f"synthetic_{i}"

    def __getitem__(self, i):
        h = self.h
        seg, hop = h.segment_size, h.hop_size
        if self.synthetic_n:
            wav, name = self._synthetic(i)
        else:
            name = self.files[i]
            wav, sr = read_wav(name)
            if sr != h.sampling_rate:
                raise ValueError(f"{name}: sampling rate {sr} != {h.sampling_rate}")
            if not self.fine_tuning:
                wav = 0.95 * wav / max(1e-8, float(np.abs(wav).max()))
        audio = torch.from_numpy(np.ascontiguousarray(wav)).float().unsqueeze(0)
        if not self.fine_tuning:
            if self.split:
                if audio.shape[1] >= seg:
                    s = random.randint(0, audio.shape[1] - seg)
                    audio = audio[:, s:s + seg]
                else:
                    audio = torch.nn.functional.pad(audio, (0, seg - audio.shape[1]))
            mel = mel_for(h, audio)
        else:
            base = os.path.splitext(os.path.basename(name))[0]
            mel = torch.from_numpy(np.load(os.path.join(self.base_mels_path, base + ".npy"), allow_pickle=False))
            mel = mel.float()
            if mel.dim() < 3:
                mel = mel.unsqueeze(0)
            if self.split:
                fps = math.ceil(seg / hop)
                if audio.shape[1] >= seg:
                    ms = random.randint(0, max(0, mel.shape[2] - fps - 1))
                    mel = mel[:, :, ms:ms + fps]
                    audio = audio[:, ms * hop:(ms + fps) * hop]
                else:
                    mel = torch.nn.functional.pad(mel, (0, fps - mel.shape[2]))
                    audio = torch.nn.functional.pad(audio, (0, seg - audio.shape[1]))
        loss_mel = mel_for(h, audio, loss=True)
        return mel.squeeze(0), audio.squeeze(0), name, loss_mel.squeeze(0)
