"""Synthetic LJSpeech-shaped batches, generated directly on the device.

Spec: text ids uniform in [1, 360]; phoneme counts follow the
LJSpeech distribution (drawn from ``preprocessed_data/LJSpeech/train.txt`` when
present: mean 70, p95 107, max 135); integer durations >= 1 with ~8.1 frames per
phoneme so that sum(d) ~= 568 +- 150 frames, capped at ``max_seq_len``; pitch /
energy ~ N(0,1) clipped to the stats range; mels in the log-mel range
[-11.5, 2].  Like the reference loader (``train.py:27-41``, ``dataset.py:127-146``)
utterances are drawn in groups of ``group_size * batch_size``, sorted by text
length and split into batches, which bounds the padding per batch.

Batches are the reference's 12-tuple with tensors already
on ``device`` (no host->device copies in the timed loop).

Frame budget (``frames_per_batch``, the ``mi355x.frames_per_gpu`` knob): instead
of a fixed utterance count, a pool of utterances is sorted by mel length and cut
into batches whose PADDED frame count ``n * max(len)`` stays within the budget
(the PostNet runs on the padded layout, so that is the memory-relevant size);
the utterance count per batch then varies with the lengths.  ``n_speakers > 1``
draws speaker ids uniformly (multi-speaker configs, e.g. LibriTTS's 904).
"""
from __future__ import annotations

import os
import re
from typing import List, Optional

import numpy as np
import torch

_LJ_META = os.path.join(os.path.dirname(__file__), "..", "..", "preprocessed_data", "LJSpeech", "train.txt")


def ljspeech_phone_counts(path: str = _LJ_META) -> Optional[np.ndarray]:
    try:
        counts = []
        with open(path, encoding="utf-8") as f:
            for line in f:
                parts = line.split("|")
                if len(parts) >= 3:
                    m = re.search(r"\{(.*)\}", parts[2])
                    if m:
                        counts.append(len(m.group(1).split()))
        return np.asarray(counts, dtype=np.int64) if counts else None
    except OSError:
        return None


class SyntheticBatches:
    def __init__(self, batch_size: int, device="cpu", n_mel: int = 80, n_speakers: int = 1, max_seq_len: int = 1000,
                 pitch_range=(-2.9, 11.4), energy_range=(-1.4, 8.2), frame_level: bool = False, group_size: int = 4,
                 seed: int = 1234, frames_per_phone: float = 8.1, vocab: int = 360, phone_counts=None,
                 frames_per_batch: Optional[int] = None):
        self.B = batch_size
        self.frame_budget = int(frames_per_batch) if frames_per_batch else None
        if self.frame_budget is not None and self.frame_budget < max_seq_len:
            raise ValueError(f"frames_per_batch={self.frame_budget} cannot hold one utterance of up to "
                             f"max_seq_len={max_seq_len} frames")
        self.device = torch.device(device)
        self.n_mel = n_mel
        self.n_speakers = n_speakers
        self.max_seq_len = max_seq_len
        self.pitch_range = pitch_range
        self.energy_range = energy_range
        self.frame_level = frame_level
        self.group = group_size
        self.fpp = frames_per_phone
        self.vocab = vocab
        self.seed = int(seed)
        self.rng = np.random.default_rng(seed)
        self.gen = torch.Generator(device="cpu").manual_seed(seed)
        pc = phone_counts if phone_counts is not None else ljspeech_phone_counts()
        self.phone_counts = pc if pc is not None else np.clip(self.rng.normal(70, 20, 10000).astype(np.int64), 8, 135)
        self._queue: List[dict] = []

    # ----------------------------------------------------------------- host side
    def _durations(self, T: int) -> np.ndarray:
        d = self.rng.gamma(shape=2.5, scale=self.fpp / 2.5, size=T)
        d = np.maximum(1, np.round(d)).astype(np.int64)
        excess = int(d.sum()) - self.max_seq_len
        while excess > 0:  # trim the longest phonemes until the utterance fits
            i = int(np.argmax(d))
            cut = min(excess, int(d[i]) - 1)
            if cut <= 0:
                break
            d[i] -= cut
            excess -= cut
        return d

    def _refill(self):
        if self.frame_budget is not None:
            return self._refill_budget()
        n = self.B * self.group
        Ts = self.rng.choice(self.phone_counts, size=n)
        order = np.argsort(-Ts, kind="stable")
        for c in range(self.group):
            idx = order[c * self.B:(c + 1) * self.B]
            self._queue.append({"T": Ts[idx], "d": [self._durations(int(t)) for t in Ts[idx]]})
        perm = self.rng.permutation(len(self._queue))
        self._queue = [self._queue[i] for i in perm]

    def _refill_budget(self):
        """~``group`` budget-sized batches: a pool sorted by mel length (descending), cut greedily so
        that ``count * longest <= frame_budget``."""
        est = max(1, int(self.frame_budget / (self.fpp * float(np.mean(self.phone_counts)))))
        Ts = self.rng.choice(self.phone_counts, size=est * self.group)
        ds = [self._durations(int(t)) for t in Ts]
        lens = np.array([min(int(d.sum()), self.max_seq_len) for d in ds])
        order = np.argsort(-lens, kind="stable")
        cur = []
        for i in order:
            longest = lens[cur[0]] if cur else lens[i]
            if cur and (len(cur) + 1) * longest > self.frame_budget:
                self._queue.append({"T": Ts[cur], "d": [ds[j] for j in cur]})
                cur = []
            cur.append(int(i))
        if cur:
            self._queue.append({"T": Ts[cur], "d": [ds[j] for j in cur]})
        perm = self.rng.permutation(len(self._queue))
        self._queue = [self._queue[i] for i in perm]

    def seek(self, index: int):
        """Re-seed both generators from (seed, ``index``) and drop queued plans: batch ``index`` of a
        seeked stream depends on nothing drawn before it, so a resumed run (``train/loop.py``, the
        checkpoint's data position) regenerates exactly the batches an uninterrupted run would."""
        ss = np.random.SeedSequence([self.seed, int(index)])
        self.rng = np.random.default_rng(ss)
        self.gen = torch.Generator(device="cpu").manual_seed(int(ss.generate_state(1, np.uint64)[0] >> 1))
        self._queue = []

    def next_plan(self):
        if not self._queue:
            self._refill()
        return self._queue.pop()

    # ----------------------------------------------------------------- device side
    def make_batch(self, plan=None):
        plan = plan or self.next_plan()
        Ts = plan["T"].astype(np.int64)
        B = len(Ts)
        ds = plan["d"]
        T = int(Ts.max())
        mel_lens = np.array([int(d.sum()) for d in ds], dtype=np.int64)
        M = int(mel_lens.max())
        dur = np.zeros((B, T), dtype=np.int64)
        for i, d in enumerate(ds):
            dur[i, : len(d)] = d
        g = self.gen
        texts = torch.randint(1, self.vocab + 1, (B, T), generator=g)
        src_valid = torch.arange(T).unsqueeze(0) < torch.from_numpy(Ts).unsqueeze(1)
        texts = texts * src_valid
        L_p = M if self.frame_level else T
        pv = torch.arange(L_p).unsqueeze(0) < torch.from_numpy(mel_lens if self.frame_level else Ts).unsqueeze(1)
        pitch = (torch.randn(B, L_p, generator=g).clamp(*self.pitch_range)) * pv
        energy = (torch.randn(B, L_p, generator=g).clamp(*self.energy_range)) * pv
        mel_valid = torch.arange(M).unsqueeze(0) < torch.from_numpy(mel_lens).unsqueeze(1)
        mels = (torch.rand(B, M, self.n_mel, generator=g) * 13.5 - 11.5) * mel_valid.unsqueeze(-1)
        speakers = torch.randint(0, self.n_speakers, (B,), generator=g)
        self.last_valid_frames = int(np.minimum(mel_lens, self.max_seq_len).sum())
        dev = self.device
        nb = dev.type == "cuda"
        tt = lambda x: x.to(dev, non_blocking=nb)  # noqa: E731
        ids = [f"synth_{i}" for i in range(B)]
        ml = tt(torch.from_numpy(mel_lens))
        ml.host_lengths = mel_lens  # host copy: sizes the packed decoder without a device sync
        return (ids, ["" for _ in range(B)], tt(speakers), tt(texts), tt(torch.from_numpy(Ts)), T, tt(mels),
                ml, M, tt(pitch), tt(energy), tt(torch.from_numpy(dur)))

    def __iter__(self):
        while True:
            yield self.make_batch()


