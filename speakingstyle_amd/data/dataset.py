"""Datasets over the reference's preprocessed-data layout.

``{preprocessed_path}/{train,val}.txt`` lines ``basename|speaker|{PH ...}|raw``,
per-utterance ``mel/{spk}-mel-{base}.npy`` ([T,80] f32), ``pitch/``, ``energy/``,
``duration/`` arrays, ``speakers.json``.  Behaviour follows the reference's
``dataset.py:12-218``: the train collate sorts a group by text length
(descending), splits it into ``batch_size`` chunks and drops the tail when
``drop_last``.  Differences: padding is done by one vectorised C++ routine when
the native host library is built (``csrc/host_collate.cpp``, falls back to
numpy), energies are float32, the TextDataset does not print every
batch (D15), and an optional ``(rank, world)`` shard makes each DP rank read a
disjoint slice of every global group.
"""
from __future__ import annotations

import json
import os
from typing import List, Optional, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset as _TorchDataset

from ..text import text_to_sequence
from ..utils.tools import pad_1d, pad_2d


def read_meta(path: str):
    names, speakers, texts, raws = [], [], [], []
    with open(path, "r", encoding="utf-8") as f:
        for line in f:
            line = line.rstrip("\n")
            if not line:
                continue
            n, s, t, r = line.split("|", 3)
            names.append(n)
            speakers.append(s)
            texts.append(t)
            raws.append(r)
    return names, speakers, texts, raws


class Dataset(_TorchDataset):
    def __init__(self, filename, preprocess_config, train_config, sort=False, drop_last=False,
                 shard: Optional[Tuple[int, int]] = None):
        self.dataset_name = preprocess_config["dataset"]
        self.preprocessed_path = preprocess_config["path"]["preprocessed_path"]
        self.cleaners = preprocess_config["preprocessing"]["text"]["text_cleaners"]
        self.batch_size = train_config["optimizer"]["batch_size"]
        self.basename, self.speaker, self.text, self.raw_text = read_meta(os.path.join(self.preprocessed_path, filename))
        with open(os.path.join(self.preprocessed_path, "speakers.json")) as f:
            self.speaker_map = json.load(f)
        self.sort = sort
        self.drop_last = drop_last
        self.shard = shard

    def __len__(self):
        return len(self.text)

    def _npy(self, kind, speaker, basename):
        return np.load(os.path.join(self.preprocessed_path, kind, f"{speaker}-{kind}-{basename}.npy"))

    def __getitem__(self, idx):
        spk = self.speaker[idx]
        base = self.basename[idx]
        return {
            "id": base,
            "speaker": self.speaker_map[spk],
            "text": np.asarray(text_to_sequence(self.text[idx], self.cleaners), dtype=np.int64),
            "raw_text": self.raw_text[idx],
            "mel": self._npy("mel", spk, base).astype(np.float32),
            "pitch": self._npy("pitch", spk, base).astype(np.float32),
            "energy": self._npy("energy", spk, base).astype(np.float32),
            "duration": self._npy("duration", spk, base).astype(np.int64),
        }

    def reprocess(self, data, idxs):
        items = [data[i] for i in idxs]
        texts = [d["text"] for d in items]
        mels = [d["mel"] for d in items]
        text_lens = np.array([t.shape[0] for t in texts], dtype=np.int64)
        mel_lens = np.array([m.shape[0] for m in mels], dtype=np.int64)
        return (
            [d["id"] for d in items],
            [d["raw_text"] for d in items],
            np.array([d["speaker"] for d in items], dtype=np.int64),
            pad_1d(texts),
            text_lens,
            int(text_lens.max()),
            pad_2d(mels),
            mel_lens,
            int(mel_lens.max()),
            pad_1d([d["pitch"] for d in items]),
            pad_1d([d["energy"] for d in items]),
            pad_1d([d["duration"] for d in items]),
        )

    def collate_fn(self, data):
        n = len(data)
        if self.sort:
            order = np.argsort(-np.array([d["text"].shape[0] for d in data]), kind="stable")
        else:
            order = np.arange(n)
        bs = self.batch_size
        full = n - n % bs
        groups: List[List[int]] = order[:full].reshape(-1, bs).tolist() if full else []
        if not self.drop_last and full < n:
            groups.append(order[full:].tolist())
        if self.shard is not None:
            rank, world = self.shard
            groups = [g[rank::world] for g in groups if len(g[rank::world])]
        return [self.reprocess(data, g) for g in groups]

    def text_lengths(self) -> np.ndarray:
        """Phoneme count per utterance from the metadata alone (no .npy reads)."""
        if getattr(self, "_tlens", None) is None:
            self._tlens = np.array([len(text_to_sequence(t, self.cleaners)) for t in self.text], dtype=np.int64)
        return self._tlens

    def mel_lengths(self) -> np.ndarray:
        """Mel frames per utterance, read from the ``.npy`` headers only (memory-mapped, no data
        pages touched); cached.  Sizes the frame-budget batches (``FrameBudgetSampler``)."""
        if getattr(self, "_mlens", None) is None:
            out = np.empty(len(self.text), dtype=np.int64)
            for i, (spk, base) in enumerate(zip(self.speaker, self.basename)):
                path = os.path.join(self.preprocessed_path, "mel", f"{spk}-mel-{base}.npy")
                out[i] = np.load(path, mmap_mode="r").shape[0]
            self._mlens = out
        return self._mlens

    def collate_local(self, data):
        """Collate for ``ShardedGroupSampler``: ``data`` is this rank's rows of one global
        group, already in the global (length-sorted) batch order; split it back into
        the per-batch shards.  ``FrameBudgetSampler`` items are one batch each."""
        sizes = self._local_sizes
        if sizes is None:
            return [self.reprocess(data, list(range(len(data))))]
        out, o = [], 0
        for n in sizes:
            if n:
                out.append(self.reprocess(data, list(range(o, o + n))))
            o += n
        return out


class ShardedGroupSampler:
    """Batch sampler with the reference loader's grouping (``train.py:27-41``,
    ``dataset.py:127-146``: shuffle, groups of ``batch_size * group`` utterances,
    each group sorted by text length and split into ``group`` batches) that shards
    *before* loading: every rank draws the same shuffled group and yields only
    its own rows (``batch[rank::world]`` of each sorted batch), so ``__getitem__``
    -- the .npy reads -- runs on the local shard only.

    ``epoch`` / ``start`` (groups already consumed) make the order resumable:
    the permutation is a pure function of ``seed + epoch``."""

    def __init__(self, dataset: "Dataset", batch_size: int, group: int = 4, rank: int = 0, world: int = 1,
                 seed: int = 1234, epoch: int = 0, start: int = 0, drop_last: bool = True):
        self.ds = dataset
        self.bs = int(batch_size)
        self.group = int(group)
        self.rank, self.world = int(rank), int(world)
        self.seed, self.epoch, self.start = int(seed), int(epoch), int(start)
        self.drop_last = drop_last
        if self.bs < self.world:
            # some rank would get an empty shard of every batch, skip its train steps and leave the
            # others waiting in the next collective until the timeout
            raise ValueError(f"batch_size={self.bs} < world size {self.world}: every rank needs at least one "
                             "utterance per batch (raise batch_size or set mi355x.frames_per_gpu)")
        self.tlens = dataset.text_lengths()
        dataset._local_sizes = [len(range(self.rank, self.bs, self.world))] * self.group

    def __len__(self):
        n = len(self.tlens) // (self.bs * self.group)
        return max(0, n - self.start)

    def __iter__(self):
        g = torch.Generator().manual_seed(self.seed + self.epoch)
        perm = torch.randperm(len(self.tlens), generator=g).numpy()
        gs = self.bs * self.group
        n = len(perm) // gs
        for gi in range(self.start, n):
            idx = perm[gi * gs:(gi + 1) * gs]
            idx = idx[np.argsort(-self.tlens[idx], kind="stable")]
            local = []
            for k in range(self.group):
                local.extend(idx[k * self.bs:(k + 1) * self.bs][self.rank::self.world].tolist())
            yield local


class FrameBudgetSampler:
    """Per-GPU frame budget (``mi355x.frames_per_gpu``): every rank gets a batch whose PADDED mel
    frame count ``n * max(len)`` stays within ``budget`` -- the batch shape is sized for the GPU's
    memory instead of a global utterance count split ``world`` ways.

    Every rank computes the same plan from ``seed + epoch`` and the utterance lengths (no
    communication): the shuffled corpus is cut into pools of ``pool`` utterances, each pool is
    sorted by mel length (descending) and cut greedily into budget-sized batches, and consecutive
    runs of ``world`` batches form one global step -- rank ``r`` takes the ``r``-th.  All ranks
    therefore run the same number of steps, with similar lengths (neighbours in the sorted pool).
    The loss divides by the all-reduced valid counts, so the DP=N gradient equals the single-process
    gradient of the union of the N batches.  ``max_batch`` optionally caps the utterance count.

    Items are one batch each; ``start`` = global steps already consumed (resumable)."""

    def __init__(self, dataset: "Dataset", budget: int, rank: int = 0, world: int = 1, seed: int = 1234,
                 epoch: int = 0, start: int = 0, pool: int = 4096, max_seq_len: int = 1000,
                 max_batch: Optional[int] = None, mel_lens: Optional[np.ndarray] = None):
        self.ds = dataset
        self.budget = int(budget)
        self.rank, self.world = int(rank), int(world)
        self.seed, self.epoch, self.start = int(seed), int(epoch), int(start)
        self.pool = int(pool)
        self.max_batch = max_batch
        lens = dataset.mel_lengths() if mel_lens is None else np.asarray(mel_lens)
        self.lens = np.minimum(lens, max_seq_len)
        if self.budget < int(self.lens.max(initial=1)):
            raise ValueError(f"frames_per_gpu={self.budget} is smaller than the longest utterance "
                             f"({int(self.lens.max())} frames after the max_seq_len cap)")
        if dataset is not None:
            dataset._local_sizes = None
        self._plan_epoch = None

    def plan(self):
        """[global step][rank] -> utterance indices of this epoch."""
        if self._plan_epoch == self.epoch:
            return self._plan
        g = torch.Generator().manual_seed(self.seed + self.epoch)
        perm = torch.randperm(len(self.lens), generator=g).numpy()
        batches = []
        for p0 in range(0, len(perm), self.pool):
            idx = perm[p0:p0 + self.pool]
            idx = idx[np.argsort(-self.lens[idx], kind="stable")]
            cur = []
            for i in idx.tolist():
                longest = self.lens[cur[0]] if cur else self.lens[i]
                full = (len(cur) + 1) * longest > self.budget or (self.max_batch and len(cur) >= self.max_batch)
                if cur and full:
                    batches.append(cur)
                    cur = []
                cur.append(i)
            if cur:
                batches.append(cur)
        n = len(batches) // self.world  # the tail that cannot give every rank a batch is dropped
        steps = [batches[k * self.world:(k + 1) * self.world] for k in range(n)]
        # shuffle the global steps (pool-internal order would run long batches first every pool)
        order = torch.randperm(len(steps), generator=g).numpy() if steps else []
        self._plan = [steps[k] for k in order]
        self._plan_epoch = self.epoch
        return self._plan

    def __len__(self):
        return max(0, len(self.plan()) - self.start)

    def __iter__(self):
        for step in self.plan()[self.start:]:
            yield step[self.rank]


class TextDataset(_TorchDataset):
    """Synthesis-time dataset: (id, speaker, phones, raw, mel) per metadata line."""

    def __init__(self, filepath, preprocess_config, train_config=None):
        self.cleaners = preprocess_config["preprocessing"]["text"]["text_cleaners"]
        self.preprocessed_path = preprocess_config["path"]["preprocessed_path"]
        self.basename, self.speaker, self.text, self.raw_text = read_meta(filepath)
        with open(os.path.join(self.preprocessed_path, "speakers.json")) as f:
            self.speaker_map = json.load(f)

    def __len__(self):
        return len(self.text)

    def __getitem__(self, idx):
        spk, base = self.speaker[idx], self.basename[idx]
        phone = np.asarray(text_to_sequence(self.text[idx], self.cleaners), dtype=np.int64)
        mel_path = os.path.join(self.preprocessed_path, "mel", f"{spk}-mel-{base}.npy")
        mel = np.load(mel_path).astype(np.float32) if os.path.exists(mel_path) else np.zeros((1, 80), np.float32)
        return base, self.speaker_map[spk], phone, self.raw_text[idx], mel

    def collate_fn(self, data):
        texts = [d[2] for d in data]
        mels = [d[4] for d in data]
        text_lens = np.array([t.shape[0] for t in texts], dtype=np.int64)
        mel_lens = np.array([m.shape[0] for m in mels], dtype=np.int64)
        return ([d[0] for d in data], [d[3] for d in data], np.array([d[1] for d in data], dtype=np.int64),
                pad_1d(texts), text_lens, int(text_lens.max()), pad_2d(mels), mel_lens, int(mel_lens.max()))


def to_device(batch, device):
    """numpy tuple -> tensors on ``device`` (reference ``utils/tools.py:18-79``;
    energies cast to f32)."""
    nb = torch.device(device).type == "cuda"

    def t(x, dtype):
        if isinstance(x, torch.Tensor):
            return x.to(device=device, dtype=dtype, non_blocking=nb)
        tt = torch.from_numpy(np.ascontiguousarray(x)).to(dtype)
        if nb:
            tt = tt.pin_memory()
        return tt.to(device, non_blocking=nb)

    if len(batch) == 12:
        ids, raw, spk, texts, src_lens, max_src, mels, mel_lens, max_mel, p, e, d = batch
        ml = t(mel_lens, torch.long)
        # host copy of the lengths: sizes the packed decoder (models/fastspeech2.py) without a sync
        if not (isinstance(mel_lens, torch.Tensor) and mel_lens.is_cuda):
            ml.host_lengths = np.asarray(mel_lens.numpy() if isinstance(mel_lens, torch.Tensor) else mel_lens)
        return (ids, raw, t(spk, torch.long), t(texts, torch.long), t(src_lens, torch.long), max_src,
                t(mels, torch.float32), ml, max_mel, t(p, torch.float32), t(e, torch.float32),
                t(d, torch.long))
    if len(batch) == 9:
        ids, raw, spk, texts, src_lens, max_src, mels, mel_lens, max_mel = batch
        return (ids, raw, t(spk, torch.long), t(texts, torch.long), t(src_lens, torch.long), max_src,
                t(mels, torch.float32), t(mel_lens, torch.long), max_mel)
    raise ValueError(f"unexpected batch arity {len(batch)}")
