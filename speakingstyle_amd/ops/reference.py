"""Plain-PyTorch implementations of every fused op (channel-last ``[B, L, C]``).

These are (a) the CPU execution path (BASELINE config #1: "tiny on CPU,
plumbing") and (b) the fp32 numerics oracle the HIP kernels are tested against
(``tests/test_kernels_gpu.py``).  They intentionally mirror the *math* of the
reference modules, cited per function, not their code structure: the reference
works in ``[B, C, L]`` for convolutions with transposes around every conv
(``model/modules.py:300-305``), we stay channel-last.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F


def lengths_to_mask(lengths: torch.Tensor, max_len: int) -> torch.Tensor:
    """True = padding (reference ``utils/tools.py:110-118`` semantics)."""
    ids = torch.arange(max_len, device=lengths.device)
    return ids.unsqueeze(0) >= lengths.unsqueeze(1)


def sinusoid_table(n_position: int, d_hid: int, device=None, dtype=torch.float32) -> torch.Tensor:
    """Sinusoid PE, dim 2i -> sin, 2i+1 -> cos, angle = pos / 10000^(2*(i//2)/d)
    (reference ``transformer/Models.py:10-30``), computed in float64 like numpy."""
    pos = torch.arange(n_position, dtype=torch.float64, device=device).unsqueeze(1)
    idx = torch.arange(d_hid, dtype=torch.float64, device=device)
    angle = pos / torch.pow(10000.0, 2.0 * torch.div(idx, 2, rounding_mode="floor") / d_hid)
    out = torch.empty_like(angle)
    out[:, 0::2] = torch.sin(angle[:, 0::2])
    out[:, 1::2] = torch.cos(angle[:, 1::2])
    return out.to(dtype)


def linear(x, w, b=None, act: Optional[str] = None):
    y = F.linear(x, w.to(x.dtype), None if b is None else b.to(x.dtype))
    return _act(y, act)


def _act(y, act):
    if act is None:
        return y
    if act == "relu":
        return F.relu(y)
    if act == "lrelu":
        return F.leaky_relu(y, 0.1)
    if act == "tanh":
        return torch.tanh(y)
    raise ValueError(act)


def conv1d(x, w, b=None, pad: int = 0, dil: int = 1, act: Optional[str] = None):
    """Channel-last Conv1d: x [B, L, Cin], w [Cout, Cin, K] (PyTorch layout) -> [B, L', Cout]."""
    y = F.conv1d(x.transpose(1, 2), w.to(x.dtype), None if b is None else b.to(x.dtype), padding=pad, dilation=dil)
    return _act(y.transpose(1, 2), act)


def conv_transpose1d(x, w, b, stride: int, pad: int):
    """Channel-last ConvTranspose1d: w [Cin, Cout, K]."""
    y = F.conv_transpose1d(x.transpose(1, 2), w.to(x.dtype), None if b is None else b.to(x.dtype), stride=stride, padding=pad)
    return y.transpose(1, 2)


def attention(qkv: torch.Tensor, lengths: torch.Tensor, n_head: int) -> torch.Tensor:
    """Scaled dot-product MHA core with key-padding mask.

    qkv: [B, L, 3*H*dk] = [q | k | v] with head-major channels (h*dk + d), exactly
    the reference's ``view(sz_b, len, n_head, d_k)`` split (``transformer/SubLayers.py:39-44``).
    Softmax over keys with keys >= length masked to -inf (``transformer/Modules.py:14-21``).
    Returns [B, L, H*dk].  Query rows >= length are zero: the reference computes them and
    masks them after the block (``transformer/Layers.py:27``); every consumer here masks
    them too, so defining them as 0 lets the kernels skip padded query tiles entirely.
    """
    B, L, C3 = qkv.shape
    D = C3 // (3 * n_head)
    q, k, v = qkv.view(B, L, 3, n_head, D).permute(2, 0, 3, 1, 4).unbind(0)  # [B,H,L,D]
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) / math.sqrt(D)
    key_pad = lengths_to_mask(lengths, L)[:, None, None, :]
    s = s.masked_fill(key_pad, float("-inf"))
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, v.float()).masked_fill(lengths_to_mask(lengths, L)[:, None, :, None], 0.0).to(qkv.dtype)
    return o.permute(0, 2, 1, 3).reshape(B, L, n_head * D)


def film(x, gamma, beta, s_gamma, s_beta):
    """(s_g*g + 1) * x + s_b*b, gamma/beta [B, C] broadcast over L (``model/blocks.py:54-62``)."""
    g = (s_gamma * gamma).unsqueeze(1)
    bb = (s_beta * beta).unsqueeze(1)
    return ((g + 1.0) * x.float() + bb).to(x.dtype)


def add_layernorm(
    a: torch.Tensor,
    residual: Optional[torch.Tensor],
    ln_w: torch.Tensor,
    ln_b: torch.Tensor,
    *,
    pre_drop: float = 0.0,
    post_drop: float = 0.0,
    training: bool = False,
    film_params: Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]] = None,
    lengths: Optional[torch.Tensor] = None,
    eps: float = 1e-5,
) -> torch.Tensor:
    """out = rowmask( FiLM( post_drop( LN( pre_drop(a) + residual ) ) ) ).

    Covers: MHA tail (``SubLayers.py:54-55`` + ``Layers.py:27-28``), FFN tail +
    FiLM + mask (``SubLayers.py:89-91``, ``Layers.py:31-35``), variance-predictor
    ReLU->LN->Dropout (``model/modules.py:216-245``) and the ref-encoder conv stack.
    """
    h = F.dropout(a, pre_drop, training) if pre_drop > 0 else a
    if residual is not None:
        h = h + residual
    y = F.layer_norm(h.float(), (h.shape[-1],), ln_w.float(), ln_b.float(), eps)
    if post_drop > 0:
        y = F.dropout(y, post_drop, training)
    if film_params is not None:
        g, b, sg, sb = film_params
        y = (sg * g.float()).unsqueeze(1).add(1.0) * y + (sb * b.float()).unsqueeze(1)
    y = y.to(a.dtype)
    if lengths is not None:
        y = y.masked_fill(lengths_to_mask(lengths, y.shape[1]).unsqueeze(-1), 0.0)
    return y


def length_regulate(x: torch.Tensor, durations: torch.Tensor, max_len: Optional[int]):
    """Expand phoneme i of item b ``durations[b, i]`` times and pad to ``max_len``.

    Equivalent to the reference's per-phoneme ``.item()`` loop
    (``model/modules.py:168-201``) but sync-free when ``max_len`` is given.
    Returns (out [B, M, C], mel_len [B] int64).
    """
    d = durations.long().clamp(min=0)
    mel_len = d.sum(1)
    B, T, C = x.shape
    if max_len is None:
        max_len = int(mel_len.max().item()) if B > 0 else 0
    cum = torch.cumsum(d, dim=1)  # [B, T]
    frames = torch.arange(max_len, device=x.device).unsqueeze(0).expand(B, -1)
    idx = torch.searchsorted(cum, frames.contiguous(), right=True)  # phoneme index per frame
    valid = frames < mel_len.unsqueeze(1)
    idx = idx.clamp(max=max(T - 1, 0))
    out = torch.gather(x, 1, idx.unsqueeze(-1).expand(-1, -1, C))
    out = out.masked_fill(~valid.unsqueeze(-1), 0.0)
    return out, mel_len


def bucketize_embed(values, bins, table):
    """torch.bucketize(values, bins) -> embedding rows (``model/modules.py:83-101``)."""
    return F.embedding(torch.bucketize(values.float(), bins.float()), table)


def masked_mean_mse(pred, target, mask_valid):
    diff = (pred.float() - target.float()) * mask_valid
    n = mask_valid.sum().clamp(min=1)
    return (diff * diff).sum() / n


def fastspeech2_loss_terms(
    mel_pred, postnet_pred, mel_target, mel_valid, p_pred, p_target, p_valid,
    e_pred, e_target, e_valid, logd_pred, d_target, src_valid,
):
    """The five masked terms of ``model/loss.py:43-82`` without ``masked_select``
    compaction: L1(mel), L1(postnet), MSE(pitch), MSE(energy), MSE(log(d+1))."""
    mv = mel_valid.unsqueeze(-1).float()
    nmel = (mv.sum() * mel_target.shape[-1]).clamp(min=1)
    mel_l = ((mel_pred.float() - mel_target.float()).abs() * mv).sum() / nmel
    post_l = ((postnet_pred.float() - mel_target.float()).abs() * mv).sum() / nmel
    pitch_l = masked_mean_mse(p_pred, p_target, p_valid.float())
    energy_l = masked_mean_mse(e_pred, e_target, e_valid.float())
    logd_t = torch.log(d_target.float() + 1.0)
    dur_l = masked_mean_mse(logd_pred, logd_t, src_valid.float())
    return mel_l, post_l, pitch_l, energy_l, dur_l
