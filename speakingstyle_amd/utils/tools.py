"""Small host-side helpers (reference ``utils/tools.py:110-125,285-337``)."""
from __future__ import annotations

import numpy as np
import torch


def pad_1d(inputs, pad_value=0):
    if pad_value == 0:
        from .native import pad_rows

        out = pad_rows(inputs)  # native host library (csrc/host_collate.cpp)
        if out is not None:
            return out
    max_len = max(len(x) for x in inputs)
    out = np.full((len(inputs), max_len), pad_value, dtype=np.asarray(inputs[0]).dtype)
    for i, x in enumerate(inputs):
        out[i, : len(x)] = x
    return out


def pad_2d(inputs, max_len=None):
    from .native import pad_rows

    out = pad_rows(inputs, max_len)  # native host library (csrc/host_collate.cpp)
    if out is not None:
        return out
    max_len = max_len or max(x.shape[0] for x in inputs)
    C = inputs[0].shape[1]
    out = np.zeros((len(inputs), max_len, C), dtype=inputs[0].dtype)
    for i, x in enumerate(inputs):
        if x.shape[0] > max_len:
            raise ValueError("sequence longer than max_len")
        out[i, : x.shape[0]] = x
    return out


def get_mask_from_lengths(lengths: torch.Tensor, max_len=None) -> torch.Tensor:
    """True = padding.  Device follows ``lengths`` (the reference uses a global device, D19)."""
    if max_len is None:
        max_len = int(lengths.max().item())
    return torch.arange(max_len, device=lengths.device).unsqueeze(0) >= lengths.unsqueeze(1)


def expand(values, durations):
    """Repeat values[i] durations[i] times (for phoneme->frame plots)."""
    return np.repeat(np.asarray(values), np.maximum(0, np.asarray(durations).astype(np.int64)))


def get_param_num(model):
    return sum(p.numel() for p in model.parameters())
