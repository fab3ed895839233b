"""Op dispatch: HIP/CDNA4 kernels on the GPU, plain PyTorch on the CPU.

There is exactly one code path per device.  On a CUDA(=HIP) device every op in
this module runs the hand-written kernels of ``csrc/`` (through
``speakingstyle_amd.ops.hip``); if the kernel library is missing on a GPU box
the first op raises instead of silently falling back.  On the CPU the torch
reference implementations (``ops.reference``) run -- they are also the test
oracle.  ``set_backend("reference")`` forces the torch path everywhere (debug /
A-B only).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from . import reference as ref
from .packing import PackInfo, pack as pack_rows, unpack as unpack_rows  # noqa: F401

_FORCED = os.environ.get("SSAMD_BACKEND")  # "reference" | "hip" | None
_NO_MAILBOX = os.environ.get("SSAMD_NO_MAILBOX") == "1"  # A/B switch for the residual-gradient fusion


def set_backend(name: Optional[str]):
    global _FORCED
    assert name in (None, "reference", "hip")
    _FORCED = name


def use_hip(t: torch.Tensor) -> bool:
    if _FORCED == "reference":
        return False
    if t.device.type != "cuda":
        if _FORCED == "hip":
            raise RuntimeError("hip backend forced but tensor is on CPU")
        return False
    return True


def _hip():
    from . import hip  # noqa: WPS433  (lazy: loads libssamd_kernels.so)

    return hip


lengths_to_mask = ref.lengths_to_mask
sinusoid_table = ref.sinusoid_table


def linear(x, w, b=None, act=None):
    if use_hip(x):
        return _hip().linear(x, w, b, act)
    return ref.linear(x, w, b, act)


def residual_mailbox(x, weights=None):
    """A GradMailbox for a sub-layer whose input x is also its LayerNorm residual (HIP path
    only; None otherwise): the residual gradient is added inside the first GEMM's backward."""
    if not use_hip(x) or x.dtype != torch.bfloat16 or not x.requires_grad or _NO_MAILBOX:
        return None
    hip = _hip()
    if weights is not None and hip.gradslots.fused_data(list(weights)) is None:
        return None
    return hip.GradMailbox()


def linear_group(x, weights, biases, mailbox=None):
    """y = x @ cat(weights)^T + cat(biases): one GEMM for several projections (Q/K/V).

    On the HIP path, when the group is contiguous in the flat arena, the fused
    weight is a view (no concatenation) and its gradient is written in place.
    """
    if use_hip(x):
        return _hip().linear_group(x, weights, biases, mailbox)
    return ref.linear(x, torch.cat(list(weights), 0), torch.cat(list(biases), 0))


def conv1d(x, w, b=None, pad=0, dil=1, act=None):
    if use_hip(x):
        return _hip().conv1d(x, w, b, pad, dil, act)
    return ref.conv1d(x, w, b, pad, dil, act)


def ffn(x, w1, b1, w2, b2, pack: Optional[PackInfo] = None, mailbox=None):
    """Position-wise FFN core: conv(k0) -> ReLU -> conv(k1) (``SubLayers.py:84-87``).

    ``pack``: x is packed ``[1, R, C]``; the convs zero-pad at every sequence end."""
    if use_hip(x):
        return _hip().ffn(x, w1, b1, w2, b2, pack, mailbox)
    if pack is not None:
        return pack_rows(ffn(unpack_rows(x, pack), w1, b1, w2, b2), pack)
    h = ref.conv1d(x, w1, b1, (w1.shape[2] - 1) // 2, 1, "relu")
    return ref.conv1d(h, w2, b2, (w2.shape[2] - 1) // 2, 1, None)


def attention(qkv, lengths, n_head, pack: Optional[PackInfo] = None):
    if use_hip(qkv):
        return _hip().attention(qkv, lengths, n_head, pack)
    if pack is not None:
        return pack_rows(ref.attention(unpack_rows(qkv, pack), pack.lens, n_head), pack)
    return ref.attention(qkv, lengths, n_head)


def add_layernorm(a, residual, ln_w, ln_b, pack: Optional[PackInfo] = None, mailbox=None, **kw):
    if use_hip(a):
        return _hip().add_layernorm(a, residual, ln_w, ln_b, pack=pack, mailbox=mailbox, **kw)
    if pack is not None:
        kw["lengths"] = pack.lens
        res = None if residual is None else unpack_rows(residual, pack)
        return pack_rows(ref.add_layernorm(unpack_rows(a, pack), res, ln_w, ln_b, **kw), pack)
    return ref.add_layernorm(a, residual, ln_w, ln_b, **kw)


def length_regulate(x, durations, max_len):
    if use_hip(x):
        return _hip().length_regulate(x, durations, max_len)
    return ref.length_regulate(x, durations, max_len)


def length_regulate_packed(x, durations, pack: PackInfo, pe):
    """LengthRegulator writing packed decoder rows (+ positional encoding)."""
    if use_hip(x):
        return _hip().length_regulate_packed(x, durations, pack, pe)
    out, _ = ref.length_regulate(x, durations, pack.M)
    return pack_rows(out + pe[: pack.M].to(out.dtype).unsqueeze(0), pack)


def embed_add_pe(ids, table, pe, extra=None):
    """table[ids] + pe[:L] (+ extra[B,C] broadcast) -> compute dtype."""
    if use_hip(ids):
        return _hip().embed_add_pe(ids, table, pe, extra)
    out = torch.nn.functional.embedding(ids, table) + pe[: ids.shape[1]].unsqueeze(0).to(table.dtype)
    if extra is not None:
        out = out + extra.unsqueeze(1)
    return out


def bucketize_embed_add(x, values, bins, table):
    """x + table[bucketize(values, bins)]."""
    if use_hip(x):
        return _hip().bucketize_embed_add(x, values, bins, table)
    return x + ref.bucketize_embed(values, bins, table).to(x.dtype)


def predictor_head(h, w, b, lengths=None):
    """Variance-predictor head: Linear(C -> 1) -> squeeze -> pad mask-fill (``modules.py:253-257``)."""
    if use_hip(h):
        return _hip().predictor_head(h, w, b, lengths)
    out = ref.linear(h, w, b).float().squeeze(-1)
    return out if lengths is None else out.masked_fill(ref.lengths_to_mask(lengths, out.shape[1]), 0.0)


def bn_act(h, bn, training, act_tanh, p, out_f32=False):
    """PostNet stage: BatchNorm1d (batch stats over all B*L rows) -> [tanh] -> dropout."""
    if use_hip(h):
        return _hip().bn_act(h, bn, training, act_tanh, p, out_f32)
    import torch.nn.functional as F

    B, L, C = h.shape
    y = F.batch_norm(h.reshape(B * L, C), bn.running_mean, bn.running_var, bn.weight, bn.bias, training,
                     bn.momentum, bn.eps).reshape(B, L, C)
    if training and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    if act_tanh:
        y = torch.tanh(y)
    y = F.dropout(y, p, training) if p > 0 else y
    return y.float() if out_f32 else y
