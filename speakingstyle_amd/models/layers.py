"""Building blocks of the FastSpeech2 family, channel-last and op-dispatched.

Parameter *names and shapes* follow the reference exactly so that reference
checkpoints load, e.g.
``slf_attn.w_qs.weight (256,256)``, ``pos_ffn.w_1.weight (1024,256,9)``,
``film.s_gamma (1,)``.  ``nn.Linear``/``nn.Conv1d``/``nn.LayerNorm`` are used
only as parameter containers (names + PyTorch default init); every forward goes
through ``speakingstyle_amd.ops`` which runs the HIP kernels on the GPU.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops

FiLMParams = Optional[Tuple[torch.Tensor, torch.Tensor]]  # (gamma [B,C], beta [B,C])


class FiLM(nn.Module):
    """Learnable-scale FiLM: (s_g*g + 1)*x + s_b*b (reference ``model/blocks.py:43-62``)."""

    def __init__(self):
        super().__init__()
        self.s_gamma = nn.Parameter(torch.ones(1))
        self.s_beta = nn.Parameter(torch.ones(1))

    def pack(self, style: FiLMParams):
        if style is None:
            return None
        g, b = style
        return (g, b, self.s_gamma, self.s_beta)


class LinearNorm(nn.Module):
    """Xavier-initialised Linear, no bias by default (reference ``model/blocks.py:65-78``)."""

    def __init__(self, in_features, out_features, bias=False):
        super().__init__()
        self.linear = nn.Linear(in_features, out_features, bias)
        nn.init.xavier_uniform_(self.linear.weight)
        if bias:
            nn.init.zeros_(self.linear.bias)

    def forward(self, x):
        return ops.linear(x, self.linear.weight, self.linear.bias)


class ConvHolder(nn.Module):
    """Parameter container named ``conv`` (reference ``ConvNorm`` / ``Conv``)."""

    def __init__(self, cin, cout, k, dilation=1, bias=True):
        super().__init__()
        self.conv = nn.Conv1d(cin, cout, k, padding=dilation * (k - 1) // 2, dilation=dilation, bias=bias)
        self.pad = dilation * (k - 1) // 2
        self.dil = dilation

    def forward(self, x, act=None):
        return ops.conv1d(x, self.conv.weight, self.conv.bias, self.pad, self.dil, act)


def fused_param_groups(module: nn.Module):
    """All contiguous-parameter groups in ``module`` (``train/optim.py::FlatArena``): the Q/K/V projections of
    every attention layer and the sub-modules' own ``arena_groups()`` (the variance adaptor's duration +
    pitch first convs, one N = 512 GEMM)."""
    groups = []
    for m in module.modules():
        if isinstance(m, MultiHeadAttention):
            groups.extend(m.fused_param_groups())
        elif hasattr(m, "arena_groups"):
            groups.extend(m.arena_groups())
    return groups


class MultiHeadAttention(nn.Module):
    """Self-attention + output projection + residual + post-LN.

    Reference: ``transformer/SubLayers.py:8-57``.  The three projections run as
    one fused [3*H*dk x d] GEMM; the core is the fused flash-style attention op.
    """

    def __init__(self, n_head, d_model, d_k, d_v, dropout=0.1):
        super().__init__()
        assert d_k == d_v
        self.n_head, self.d_k = n_head, d_k
        self.w_qs = nn.Linear(d_model, n_head * d_k)
        self.w_ks = nn.Linear(d_model, n_head * d_k)
        self.w_vs = nn.Linear(d_model, n_head * d_v)
        self.layer_norm = nn.LayerNorm(d_model)
        self.fc = nn.Linear(n_head * d_v, d_model)
        self.dropout = dropout

    def fused_param_groups(self):
        """Q/K/V weights (and biases) adjacent in the flat arena -> the fused projection is a view."""
        return [[self.w_qs.weight, self.w_ks.weight, self.w_vs.weight], [self.w_qs.bias, self.w_ks.bias, self.w_vs.bias]]

    def forward(self, x, lengths, pack=None):
        ws = (self.w_qs.weight, self.w_ks.weight, self.w_vs.weight)
        mb = ops.residual_mailbox(x, ws)  # d(residual x) joins the QKV data gradient in its epilogue
        qkv = ops.linear_group(x, ws, (self.w_qs.bias, self.w_ks.bias, self.w_vs.bias), mailbox=mb)
        o = ops.attention(qkv, lengths, self.n_head, pack)
        # LN(dropout(fc(o)) + x), then the FFT block's pad mask-fill (Layers.py:27-28): one addln kernel
        kw = dict(pre_drop=self.dropout, training=self.training, lengths=lengths, pack=pack)
        if mb is None and not self.training and not ops.needs_grad(x, *self.fc.parameters(),
                                                                    *self.layer_norm.parameters()):
            # inference: output projection + residual + LayerNorm as one fused kernel for small batches
            return ops.linear_add_layernorm(o, self.fc.weight, self.fc.bias, x, self.layer_norm.weight,
                                            self.layer_norm.bias, **kw)
        a = ops.linear(o, self.fc.weight, self.fc.bias)
        return ops.add_layernorm(a, x, self.layer_norm.weight, self.layer_norm.bias, mailbox=mb, **kw)


class PositionwiseFeedForward(nn.Module):
    """Conv1d(k0) -> ReLU -> Conv1d(k1) -> dropout -> +res -> LN (``SubLayers.py:60-93``)."""

    def __init__(self, d_in, d_hid, kernel_size: Sequence[int], dropout=0.1):
        super().__init__()
        self.w_1 = nn.Conv1d(d_in, d_hid, kernel_size[0], padding=(kernel_size[0] - 1) // 2)
        self.w_2 = nn.Conv1d(d_hid, d_in, kernel_size[1], padding=(kernel_size[1] - 1) // 2)
        self.layer_norm = nn.LayerNorm(d_in)
        self.dropout = dropout
        self.k = tuple(kernel_size)

    def forward(self, x, lengths, film_params=None, pack=None):
        mb = ops.residual_mailbox(x)  # d(residual x) joins the first conv's data gradient
        kw = dict(pre_drop=self.dropout, training=self.training, film_params=film_params, lengths=lengths, pack=pack)
        if (mb is None and not self.training and self.k[1] == 1
                and not ops.needs_grad(x, *self.parameters(), *(film_params or ()))):
            # inference: conv -> ReLU, then the second conv + residual + LN (+ FiLM) as one kernel for small batches
            h = ops.conv1d(x, self.w_1.weight, self.w_1.bias, (self.k[0] - 1) // 2, 1, "relu", pack=pack)
            return ops.linear_add_layernorm(h, self.w_2.weight, self.w_2.bias, x, self.layer_norm.weight,
                                            self.layer_norm.bias, **kw)
        z = ops.ffn(x, self.w_1.weight, self.w_1.bias, self.w_2.weight, self.w_2.bias, pack, mailbox=mb)
        return ops.add_layernorm(z, x, self.layer_norm.weight, self.layer_norm.bias, mailbox=mb, **kw)


class FFTBlock(nn.Module):
    """MHA -> mask -> FFN -> [FiLM] -> mask (``transformer/Layers.py:11-37``)."""

    def __init__(self, d_model, n_head, d_k, d_v, d_inner, kernel_size, dropout=0.1, film=True):
        super().__init__()
        self.slf_attn = MultiHeadAttention(n_head, d_model, d_k, d_v, dropout=dropout)
        self.pos_ffn = PositionwiseFeedForward(d_model, d_inner, kernel_size, dropout=dropout)
        if film:
            self.film = FiLM()

    def forward(self, x, lengths, style: FiLMParams = None, pack=None):
        """``pack``: x is the packed ``[1, R, C]`` decoder input (``ops/packing.py``)."""
        x = self.slf_attn(x, lengths, pack)
        fp = self.film.pack(style) if (style is not None and hasattr(self, "film")) else None
        return self.pos_ffn(x, lengths, fp, pack)


class PostNet(nn.Module):
    """5 x (Conv1d k5 + BatchNorm1d), tanh on the first 4, dropout 0.5 always in
    training (``transformer/Layers.py:78-148``).  BatchNorm statistics are taken
    over all B*M rows including padding (reference semantics)."""

    def __init__(self, n_mel_channels=80, emb=512, k=5, n=5):
        super().__init__()
        chans = [n_mel_channels] + [emb] * (n - 1) + [n_mel_channels]
        self.convolutions = nn.ModuleList(
            nn.Sequential(ConvHolder(chans[i], chans[i + 1], k), nn.BatchNorm1d(chans[i + 1])) for i in range(n)
        )
        self.dropout = 0.5  # hard-coded in the reference (Layers.py:140-148)

    def forward(self, x):
        # conv_0, then [BN_i + tanh + dropout -> conv_{i+1}] links (the data gradient of conv_{i+1} starts
        # BN_i's backward in its GEMM epilogue on the GPU), then the last BN (fp32 out)
        last = len(self.convolutions) - 1
        h = self.convolutions[0][0](x)
        for i in range(last):
            bn, nxt = self.convolutions[i][1], self.convolutions[i + 1][0]
            h = ops.bn_act_conv(h, bn, self.training, True, self.dropout, nxt.conv.weight, nxt.conv.bias, nxt.pad)
        return ops.bn_act(h, self.convolutions[last][1], self.training, act_tanh=False, p=self.dropout, out_f32=True)

    def forward_packed(self, x, pack):
        """Inference on packed rows [1, R, C] (``ops/packing.py``): eval-mode BatchNorm is a per-channel affine of
        the running statistics (row-independent) and every conv zero-pads at its own sequence's ends -- each
        utterance's PostNet output exactly as when it is synthesized alone.

        The affine is folded into the conv it follows (``folded``): 5 GEMM launches (tanh in the epilogue, the
        last one writing fp32) instead of 5 GEMMs + 5 BatchNorm finalize / apply pairs -- the batch-1 serving
        path is launch-bound."""
        assert not self.training, "PostNet.forward_packed: inference only (training BatchNorm needs the padded rows)"
        layers = self.folded()
        h = x
        for i, (w, b) in enumerate(layers):
            c = self.convolutions[i][0]
            last = i == len(layers) - 1
            h = ops.conv1d(h, w, b, c.pad, c.dil, act=None if last else "tanh", pack=pack, out_f32=last)
        return h

    def folded(self):
        """Per layer (W * s, b * s + t) with s = gamma / sqrt(running_var + eps), t = beta - running_mean * s:
        conv followed by eval BatchNorm as one conv.  Cached per parameter / buffer version (not registered,
        so never in the state dict)."""
        ts = []
        for conv, bn in self.convolutions:
            ts += [conv.conv.weight, conv.conv.bias, bn.weight, bn.bias, bn.running_mean, bn.running_var]
        key = tuple((t.data_ptr(), t._version) for t in ts if t is not None)
        hit = self.__dict__.get("_fold")
        if hit is not None and hit[0] == key:
            return hit[1]
        out = []
        with torch.no_grad():
            for conv, bn in self.convolutions:
                w = conv.conv.weight.detach().float()
                s = bn.weight.detach().float() * torch.rsqrt(bn.running_var.float() + bn.eps)
                t = bn.bias.detach().float() - bn.running_mean.float() * s
                b = conv.conv.bias.detach().float() if conv.conv.bias is not None else torch.zeros_like(s)
                wf = nn.Parameter((w * s.view(-1, *([1] * (w.dim() - 1)))).to(conv.conv.weight.dtype),
                                  requires_grad=False)
                out.append((wf, (b * s + t).contiguous()))
        self.__dict__["_fold"] = (key, out)
        return out
