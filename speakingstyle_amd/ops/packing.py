"""Packed variable-length sequences for the decoder (no padded frames in the hot path).

The reference runs the decoder on a padded ``[B, M_max, C]`` tensor and masks
(``transformer/Models.py:147-170``): with LJSpeech-like batches ~24 % of the
decoder rows are padding, computed and thrown away by every GEMM, attention and
LayerNorm.  Here the decoder runs on the valid frames only, ``[1, R, C]`` with
``R = sum(min(len_b, M))`` rows, sequence ``b`` at rows ``cu[b] .. cu[b]+len_b-1``:

* row-wise ops (Linear / QKV / k=1 convs / FiLM-free LN) are unchanged GEMMs
  with ``M = R``;
* the k=9 FFN conv zero-pads at sequence ends through a per-row
  ``(position, length)`` table (``rinfo``) read by the GEMM A-loaders;
* attention and LayerNorm find each sequence from ``cu`` / ``lens``;
* the length regulator writes packed rows directly, and ``unpack`` restores
  the padded layout (padded rows = the reference's value there) before the
  PostNet, whose BatchNorm statistics include padded rows.

``R`` must be known on the host (no sync in the step): the data pipeline
provides it with the batch (``data/dataset.py``, ``data/synthetic.py``).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch


@dataclass
class PackInfo:
    B: int            # sequences
    M: int            # longest sequence / padded length
    R: int            # packed rows = sum(min(lens, M))
    lens: torch.Tensor   # int64 [B] (already clamped to M)
    cu: torch.Tensor     # int64 [B+1] row offsets
    rinfo: torch.Tensor  # int32 [R, 2] (position, length)
    dst: torch.Tensor    # int64 [R] row index in the padded [B*M] layout

    @staticmethod
    def build(lens: torch.Tensor, M: int, R: int) -> "PackInfo":
        lens = lens.to(torch.int64).clamp(max=M).contiguous()
        B = lens.shape[0]
        dev = lens.device
        cu = torch.empty(B + 1, dtype=torch.int64, device=dev)
        rinfo = torch.empty(R, 2, dtype=torch.int32, device=dev)
        dst = torch.empty(R, dtype=torch.int64, device=dev)
        if lens.is_cuda:
            from . import hip

            hip.pack_info(lens, M, cu, rinfo, dst)
        else:
            cu[0] = 0
            cu[1:] = torch.cumsum(lens, 0)
            b = torch.repeat_interleave(torch.arange(B, device=dev), lens, output_size=R)
            t = torch.arange(R, device=dev) - cu[:-1][b]
            rinfo[:, 0] = t.to(torch.int32)
            rinfo[:, 1] = lens[b].to(torch.int32)
            dst.copy_(b * M + t)
        return PackInfo(B, M, R, lens, cu, rinfo, dst)


def pack(x: torch.Tensor, p: PackInfo) -> torch.Tensor:
    """[B, M, C] -> [1, R, C] (valid rows)."""
    return x.reshape(p.B * p.M, -1).index_select(0, p.dst).unsqueeze(0)


def unpack(x: torch.Tensor, p: PackInfo, fill=None) -> torch.Tensor:
    """[1, R, C] -> [B, M, C]; padded rows = ``fill`` ([C] row, default 0)."""
    C = x.shape[-1]
    if fill is None:
        base = x.new_zeros(p.B * p.M, C)
    else:
        base = fill.to(x.dtype).reshape(1, C).expand(p.B * p.M, C).clone()
    return base.index_copy(0, p.dst, x.reshape(p.R, C)).view(p.B, p.M, C)
