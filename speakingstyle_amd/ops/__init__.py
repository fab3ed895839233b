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
import torch.nn.functional as F

from . import reference as ref
from .packing import PackInfo, pack as _pack, unpack as _unpack  # noqa: F401

_FORCED = os.environ.get("SSAMD_BACKEND")  # "reference" | "hip" | None


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
    if not use_hip(x) or x.dtype != torch.bfloat16 or not x.requires_grad:
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


class IdCache:
    """Values cached per tensor object (by identity, held weakly): ``WeakKeyDictionary`` compares tensor keys with
    ``==`` (elementwise) and cannot be used for tensors."""

    def __init__(self):
        self._d = {}

    def get(self, t):
        e = self._d.get(id(t))
        return e[1] if e is not None and e[0]() is t else None

    def put(self, t, v):
        import weakref

        if len(self._d) > 256:  # drop entries whose tensor is gone
            self._d = {k: e for k, e in self._d.items() if e[0]() is not None}
        self._d[id(t)] = (weakref.ref(t), v)


def conv1d(x, w, b=None, pad=0, dil=1, act=None, pack: Optional[PackInfo] = None, out_f32: bool = False):
    """``pack``: x is packed ``[1, R, C]``; the conv zero-pads at every sequence end.  ``out_f32``: fp32 output
    (the GPU GEMM writes its fp32 accumulators)."""
    if use_hip(x):
        return _hip().conv1d(x, w, b, pad, dil, act, out_f32=out_f32, pack=pack)
    if pack is not None:
        y = pack_rows(ref.conv1d(unpack_rows(x, pack), w, b, pad, dil, act), pack)
    else:
        y = ref.conv1d(x, w, b, pad, dil, act)
    return y.float() if out_f32 else y


def conv_relu_layernorm(x, w, b, pad, dil, ln_w, ln_b, **kw):
    """LayerNorm(ReLU(conv1d(x))) (+ post-dropout / FiLM via ``kw``): the variance-predictor block
    (``model/modules.py:221-240``).  On the GPU the conv's backward leaves the ReLU mask to the LayerNorm
    backward, which reads the ReLU output anyway -- one elementwise pass over the gradient fewer."""
    if use_hip(x) and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0 and w.shape[0] in (256, 512, 1024):
        h = _hip().conv1d(x, w, b, pad, dil, "relu_ln")
        return _hip().add_layernorm(h, None, ln_w, ln_b, relu_input=True, **kw)
    return add_layernorm(conv1d(x, w, b, pad, dil, "relu"), None, ln_w, ln_b, **kw)


def dual_conv_relu_layernorm(x, ws, bs, pad, dil, lns, post_drop=0.0, training=False):
    """The first blocks of two variance predictors on the same input x (duration and pitch, reference
    ``model/modules.py:121-125``): (LN_d(ReLU(conv_d(x))), LN_p(ReLU(conv_p(x)))) with post-dropout.  On the
    GPU ONE N = 2C GEMM each way (``hip._DualConvReluLNFn``) when the two weights are adjacent in the flat
    arena; otherwise (and on the CPU) the two blocks separately -- same values."""
    p = float(post_drop) if training else 0.0
    if use_hip(x):
        out = _hip().dual_conv_relu_layernorm(x, ws, bs, pad, dil, lns, p)
        if out is not None:
            return out
    return tuple(conv_relu_layernorm(x, w, b, pad, dil, lw, lb, post_drop=post_drop, training=training)
                 for w, b, (lw, lb) in zip(ws, bs, lns))


def repack_rows(x, src_pack: PackInfo, out_pack: PackInfo, pe=None):
    """Rows of one packed layout -> another over the same sequences (+ ``pe[t]``); rows past the
    source length are 0 (e.g. the halo-packed FiLM conv stack -> the FFT blocks' packed rows)."""
    if use_hip(x):
        return _hip().repack_rows(x, src_pack, out_pack, pe)
    y = unpack_rows(x, src_pack)  # [B, M_src, C], 0 past each source length
    if y.shape[1] < out_pack.M:
        y = F.pad(y, (0, 0, 0, out_pack.M - y.shape[1]))
    return pack_rows(y[:, : out_pack.M], out_pack, pe)


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


def needs_grad(*tensors) -> bool:
    """Whether autograd will record an op on these tensors (grad mode on and any of them requires grad): the
    inference-only kernel paths (folded BatchNorm, fused GEMM + LayerNorm) are taken when it does not."""
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in tensors)


def linear_add_layernorm(x, w, b, residual, ln_w, ln_b, pack: Optional[PackInfo] = None, **kw):
    """add_layernorm(linear(x, w, b), residual, ...) -- ``w`` a Linear [C, K] or a k = 1 Conv1d [C, K, 1] weight.
    Inference (no grad, not training) on the GPU runs it as ONE kernel for small row counts (``hip.gemm_addln``:
    batch-1 serving); everything else is the two ops."""
    fp = kw.get("film_params")
    if (use_hip(x) and not kw.get("training", False)
            and not needs_grad(x, w, b, residual, ln_w, ln_b, *(fp if fp is not None else ()))):
        y = _hip().gemm_addln(x, w, b, residual, ln_w, ln_b, film_params=kw.get("film_params"),
                              lengths=kw.get("lengths"), pack=pack, eps=kw.get("eps", 1e-5))
        if y is not None:
            return y
    a = linear(x, w, b) if w.dim() == 2 else conv1d(x, w, b, pack=pack)
    return add_layernorm(a, residual, ln_w, ln_b, pack=pack, **kw)


def length_regulate(x, durations, max_len, mel_len=None):
    if use_hip(x):
        return _hip().length_regulate(x, durations, max_len, mel_len=mel_len)
    return ref.length_regulate(x, durations, max_len)


def duration_round(log_d, lengths, control=1.0):
    """Inference durations: max(round(exp(log_d)-1), 0) * control, rounded, 0 at pads -> (d, mel_len)."""
    if use_hip(log_d):
        return _hip().duration_round(log_d, lengths, control)
    d = torch.clamp(torch.round(torch.exp(log_d) - 1.0), min=0.0)
    if isinstance(control, torch.Tensor):
        control = control.to(d.device, d.dtype)
        if control.dim() == 2 and control.shape[1] != d.shape[1]:
            control = F.pad(control, (0, d.shape[1] - control.shape[1]), value=1.0)[:, : d.shape[1]]
        d = d * control
    elif control != 1.0:
        d = d * control
    d = torch.clamp(torch.round(d), min=0.0)
    d = d.masked_fill(ref.lengths_to_mask(lengths, d.shape[1]), 0.0).long()
    return d, d.sum(1)


def seq_mean(x, divisor=None, pack: Optional[PackInfo] = None):
    """[B, L, C] -> [B, C] fp32 mean over the (padded) length L (``divisor`` overrides L); with
    ``pack``: x is packed ``[1, R, C]``, each sequence's rows summed and divided by ``divisor``."""
    if use_hip(x):
        return _hip().seq_mean(x, divisor, pack)
    if pack is not None:
        x = _unpack(x, pack)
    return x.float().sum(1) / float(divisor or x.shape[1])


def add_rowvec(x, v):
    """x [B, L, C] + v[:, None, :] (per-utterance vector, e.g. the speaker embedding)."""
    if use_hip(x):
        return _hip().add_rowvec(x, v)
    return x + v.to(x.dtype).unsqueeze(1)


def add_table_rows(x, table, ids):
    """x [B, L, C] + table[ids[b]] broadcast over L (the speaker embedding: lookup fused into the add)."""
    if use_hip(x):
        return _hip().add_table_rows(x, table, ids)
    return x + F.embedding(ids, table).to(x.dtype).unsqueeze(1)


def pack_rows(x, pack: PackInfo, pe=None):
    """[B, M, C] -> packed [1, R, C] (+ positional encoding ``pe[t]`` when given)."""
    if use_hip(x):
        return _hip().pack_rows(x, pack, pe)
    return _pack(x if pe is None else x + pe[: pack.M].to(x.dtype).unsqueeze(0), pack)


def unpack_rows(x, pack: PackInfo, fill=None):
    """packed [1, R, C] -> [B, M, C]; padded rows = ``fill`` ([C], default 0)."""
    if use_hip(x):
        return _hip().unpack_rows(x, pack, fill)
    return _unpack(x, pack, fill)


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


def bn_act_conv(h, bn, training, act_tanh, p, w, b, pad):
    """conv(drop(act(BN(h)))): one PostNet link.  On the GPU the conv's data-gradient GEMM starts the
    BatchNorm backward in its epilogue (``hip._BNActConvFn``); elsewhere bn_act followed by conv1d."""
    from .. import experimental

    if use_hip(h) and experimental.get("bn_fuse") and act_tanh != "relu" and _hip().bn_act_conv_ok(h.shape[-1], w):
        return _hip().bn_act_conv(h, bn, training, act_tanh, p, w, b, pad)
    return conv1d(bn_act(h, bn, training, act_tanh, p), w, b, pad)


def bn_act(h, bn, training, act_tanh, p, out_f32=False):
    """PostNet stage: BatchNorm1d (batch stats over all B*L rows) -> [tanh] -> dropout.
    ``act_tanh="relu"`` applies ReLU instead (GST BatchNorm2d over NHWC rows)."""
    if use_hip(h):
        return _hip().bn_act(h, bn, training, act_tanh, p, out_f32)
    B, L, C = h.shape
    y = F.batch_norm(h.reshape(B * L, C), bn.running_mean, bn.running_var, bn.weight, bn.bias, training,
                     bn.momentum, bn.eps).reshape(B, L, C)
    if training and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    if act_tanh == "relu":
        y = F.relu(y)
    elif act_tanh:
        y = torch.tanh(y)
    y = F.dropout(y, p, training) if p > 0 else y
    return y.float() if out_f32 else y


# ------------------------------------------------------------------ GST reference encoder
def conv2d_s2(x, w, b=None):
    """Conv2d(3x3, stride 2, pad 1) on channel-last x [B, H, W, Cin] -> [B, Ho, Wo, Cout]."""
    if use_hip(x):
        return _hip().conv2d_s2(x, w, b)
    y = F.conv2d(x.permute(0, 3, 1, 2), w.to(x.dtype), None if b is None else b.to(x.dtype), stride=2, padding=1)
    return y.permute(0, 2, 3, 1)


def conv2d_s2_prepare(w, b):
    """Inference operand of ``conv2d_s2_infer`` for weight w [Cout, Cin, 3, 3] / bias b (fp32): on the GPU the
    bf16 im2col-order image, built once by the caller's cache instead of per call."""
    b = b.detach().float().contiguous()
    if use_hip(w):
        return ("img", _hip().conv2d_s2_image(w), b)
    return ("ref", w.detach(), b)


def conv2d_s2_infer(x, prep, act=None):
    """Forward-only Conv2d(3x3, s2, p1) (+ activation) with an operand from ``conv2d_s2_prepare``."""
    kind, w, b = prep
    if kind == "img" and use_hip(x):
        return _hip().conv2d_s2_infer(x, w, b, act)
    if kind == "img":
        raise ValueError("conv2d_s2_infer: GPU weight image with a host input")
    y = F.conv2d(x.permute(0, 3, 1, 2), w.to(x.dtype), b.to(x.dtype), stride=2, padding=1).permute(0, 2, 3, 1)
    return ref._act(y, act)


def gru_last(x, gru, last):
    """Batch-first single-layer GRU over x [B, T, I]; returns the hidden state at step last[b] (fp32)."""
    if use_hip(x):
        return _hip().gru_last(x, gru, last)
    # explicit cell loop (torch gate order r, z, n): device-agnostic and differentiable in eval mode
    # (the MIOpen RNN refuses a backward outside training mode)
    gi = F.linear(x.float(), gru.weight_ih_l0, gru.bias_ih_l0)
    h = x.new_zeros(x.shape[0], gru.hidden_size, dtype=torch.float32)
    outs = []
    for t in range(x.shape[1]):
        gr, gz, gn = gi[:, t].chunk(3, -1)
        hr, hz, hn = F.linear(h, gru.weight_hh_l0, gru.bias_hh_l0).chunk(3, -1)
        r, z = torch.sigmoid(gr + hr), torch.sigmoid(gz + hz)
        h = (1 - z) * torch.tanh(gn + r * hn) + z * h
        outs.append(h)
    out = torch.stack(outs, 1)
    idx = last.to(torch.int64).view(-1, 1, 1).expand(-1, 1, out.shape[-1])
    return out.gather(1, idx).squeeze(1)


def token_bank(E, Wk, Wv, n_head):
    """GST token bank: keys = tanh(E) [N, dt]; K / V = keys @ Wk^T / Wv^T as [n_head, N, D] (fp32)."""
    if use_hip(E):
        return _hip().token_bank(E, Wk, Wv, n_head)
    keys = torch.tanh(E.float())
    N = keys.shape[0]
    D = Wk.shape[0] // n_head
    k = (keys @ Wk.float().t()).view(N, n_head, D).transpose(0, 1).contiguous()
    v = (keys @ Wv.float().t()).view(N, n_head, D).transpose(0, 1).contiguous()
    return k, v


def token_attention(q, K, V):
    """Multi-head attention of q [B, NH*D] over a token bank K/V [NH, N, D]:
    returns (style [B, NH*D] fp32, weights [B, NH, N])."""
    if use_hip(q):
        return _hip().token_attention(q, K, V)
    NH, N, D = K.shape
    qh = q.float().view(q.shape[0], NH, 1, D)
    w = torch.softmax(torch.matmul(qh, K.float().transpose(-1, -2).unsqueeze(0)) / (D ** 0.5), -1)
    return torch.matmul(w, V.float().unsqueeze(0)).reshape(q.shape[0], NH * D), w.squeeze(2)
