"""HiFi-GAN V1 vocoder (generator + multi-period / multi-scale discriminators + losses).

Reference: ``hifigan/models.py`` (generator ``:112-174``, ResBlock1 ``:20-110``,
MSD ``:176-232``, losses ``:234-264``) and ``hifigan/config.json``.  The
reference's discriminator side cannot run (``MultiPeriodDiscriminator`` is
imported by ``hifigan/train.py:17`` but never defined, ``spectral_norm`` /
``AvgPool1d`` are not imported -- SURVEY D16); here both discriminators are
implemented (MPD follows the HiFi-GAN paper: periods 2, 3, 5, 7, 11).

State-dict keys of the generator match the reference (``conv_pre``, ``ups.i``,
``resblocks.j.convs{1,2}.k``, ``conv_post`` with weight-norm ``weight_g`` /
``weight_v``), so ``generator_*.pth.tar`` files load.  ``fold_weight_norm()``
replaces every weight-normed conv by its folded weight (reference
``remove_weight_norm``) for inference.

Inference runs channel-last on the HIP kernels (``Generator._infer_hip``): each
transposed convolution is ONE 3-tap implicit GEMM with N = stride * Cout whose
output rows are the interleaved phases (``convT_as_conv3``), activations / bias /
residual / MRF mean sit in GEMM epilogues, the C <= 128 ResBlocks are single fused
layer kernels.  The CPU path (tests) uses the polyphase decomposition.  Training runs in PyTorch NCL
layout with autograd (vocoder training is not a headline config).
"""
from __future__ import annotations

import os
from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.utils import spectral_norm, weight_norm

from .. import ops

LRELU_SLOPE = 0.1
# whole-ResBlock kernel for the narrow stages (False: one fused kernel per layer pair; A/B + tests)
_WHOLE_BLOCK = [True]
# whole-block geometries routed to the per-layer kernel instead (A/B of halo recompute vs three launches)
_WHOLE_SKIP = set()


class AttrDict(dict):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.__dict__ = self


def default_config() -> AttrDict:
    """HiFi-GAN V1 (the reference's ``hifigan/config.json``)."""
    return AttrDict({
        "resblock": "1", "num_gpus": 0, "batch_size": 16, "learning_rate": 0.0002, "adam_b1": 0.8,
        "adam_b2": 0.99, "lr_decay": 0.999, "seed": 1234, "upsample_rates": [8, 8, 2, 2],
        "upsample_kernel_sizes": [16, 16, 4, 4], "upsample_initial_channel": 512,
        "resblock_kernel_sizes": [3, 7, 11], "resblock_dilation_sizes": [[1, 3, 5], [1, 3, 5], [1, 3, 5]],
        "segment_size": 8192, "num_mels": 80, "num_freq": 1025, "n_fft": 1024, "hop_size": 256, "win_size": 1024,
        "sampling_rate": 22050, "fmin": 0, "fmax": 8000, "fmax_for_loss": None, "num_workers": 4,
        "dist_config": {"dist_backend": "nccl", "dist_url": "tcp://127.0.0.1:54321", "world_size": 1},
    })


def get_padding(k, d=1):
    return (k * d - d) // 2


def _init(m, std=0.01):
    if isinstance(m, (nn.Conv1d, nn.ConvTranspose1d)):
        m.weight.data.normal_(0.0, std)


def _w(conv):
    """Effective weight of a (possibly weight-normed) conv."""
    return conv.weight


def _wn(conv):
    """Differentiable effective weight ``g * v / ||v||`` of a weight-normed conv (torch recomputes
    ``conv.weight`` in a forward pre-hook, which the channel-last training path does not run)."""
    if hasattr(conv, "weight_g") and hasattr(conv, "weight_v"):
        return torch._weight_norm(conv.weight_v, conv.weight_g, 0)
    return conv.weight


# generator training on the HIP implicit-GEMM convs (channel-last); 0: torch / MIOpen NCL convs
def _hip_train() -> bool:
    from .. import experimental

    return experimental.get("hifigan_hip_train")


class _TorchGlue:
    """Elementwise glue of the channel-last training path on torch ops (CPU / reference backend)."""

    @staticmethod
    def lrelu(x, slope):
        return F.leaky_relu(x, slope)

    @staticmethod
    def add(a, b):
        return a + b

    @staticmethod
    def mean3(a, b, c):
        return (a + b + c) / 3


def _glue(x):
    """HIP kernels (``vocoder/hip_train.py``: lrelu / residual add / MRF mean / conv_post + tanh as autograd
    Functions) for bf16 GPU activations, torch ops otherwise."""
    if x.is_cuda and ops.use_hip(x) and x.dtype == torch.bfloat16:
        from ..vocoder import hip_train

        return hip_train
    return _TorchGlue


class ResBlock1(nn.Module):
    def __init__(self, channels, kernel_size=3, dilation=(1, 3, 5)):
        super().__init__()
        self.convs1 = nn.ModuleList(
            weight_norm(nn.Conv1d(channels, channels, kernel_size, 1, dilation=d, padding=get_padding(kernel_size, d)))
            for d in dilation)
        self.convs2 = nn.ModuleList(
            weight_norm(nn.Conv1d(channels, channels, kernel_size, 1, dilation=1, padding=get_padding(kernel_size, 1)))
            for _ in dilation)
        self.convs1.apply(_init)
        self.convs2.apply(_init)
        self.kernel_size = kernel_size
        self.dilation = tuple(dilation)

    def forward(self, x):  # NCL, autograd (training path)
        for c1, c2 in zip(self.convs1, self.convs2):
            xt = c2(F.leaky_relu(c1(F.leaky_relu(x, LRELU_SLOPE)), LRELU_SLOPE))
            x = xt + x
        return x

    def forward_cl_train(self, x):
        """Channel-last training path [B, T, C] bf16 on the HIP convs (autograd): lrelu -> dilated
        conv -> lrelu -> conv -> + x per layer; the conv weights are the weight-normed tensors."""
        k = self.kernel_size
        glue = _glue(x)
        for c1, c2, d in zip(self.convs1, self.convs2, self.dilation):
            t = ops.conv1d(glue.lrelu(x, LRELU_SLOPE), _wn(c1), c1.bias, get_padding(k, d), d, None)
            t = ops.conv1d(glue.lrelu(t, LRELU_SLOPE), _wn(c2), c2.bias, get_padding(k, 1), 1, None)
            x = glue.add(t, x)
        return x

    def fusable(self, channels: int, rows=None) -> bool:
        """Geometry covered by the fused ResBlock1 layer kernel (csrc/k_vocoder.hip); C = 256 (K <= 7) on its
        tall tile only, behind ``_RB256``, and (``rows`` given) only for >= ``_RB256_MIN_ROWS`` rows (an A/B knob:
        0, every size, measured best -- even one utterance's few tiles beat the split-K GEMMs)."""
        if max(self.dilation) > 5 or self.kernel_size not in (3, 7, 11):
            return False
        if channels == 256:
            return bool(_RB256[0] and self.kernel_size <= 7 and (rows is None or rows >= _RB256_MIN_ROWS[0]))
        return channels in (32, 64, 128)

    def fused_ok(self, x) -> bool:
        return x.is_cuda and ops.use_hip(x) and x.dtype == torch.bfloat16 and self.fusable(x.shape[-1])

    def forward_cl(self, x, acc=None, out_scale=1.0, x_act=None, post_lrelu=False):
        """Channel-last inference path [B, T, C].  Returns ``(acc +) block(x) * out_scale`` (then
        ``lrelu`` when ``post_lrelu``: the next upsampling conv's input activation).

        GPU: the high-rate stages (C = 32 / 64 / 128) run each layer as ONE fused kernel (lrelu -> dilated
        conv -> lrelu -> conv -> + x [-> + acc, * scale, lrelu], ``csrc/k_vocoder.hip``); the wide stages
        use the implicit-GEMM conv with everything in its epilogues: lrelu after the first conv, the
        residual + a second lrelu'd output (the next layer's input) after the second, and the MRF
        accumulate / mean / post-activation after the block's last conv -- no elementwise pass.
        ``x_act``: lrelu(x) when the caller already has it (shared by the MRF branches)."""
        k = self.kernel_size
        n = len(self.convs1)
        if self.fused_ok(x):
            hip = ops._hip()
            if _WHOLE_BLOCK[0] and n == 3 and hip.resblock_fusable(x.shape[-1], k):
                # all three layers in one kernel: the residual stream stays in registers, no HBM round trips
                return hip.resblock_fused(x, self.convs1, self.convs2, self.dilation, LRELU_SLOPE, acc=acc,
                                          out_scale=out_scale, post_lrelu=post_lrelu)
            for i, (c1, c2, d) in enumerate(zip(self.convs1, self.convs2, self.dilation)):
                last = i == n - 1
                x = hip.resblock_layer(x, c1, c2, d, LRELU_SLOPE, acc=acc if last else None,
                                       out_scale=out_scale if last else 1.0, post_lrelu=post_lrelu and last)
            return x
        if x.is_cuda and ops.use_hip(x) and x.dtype == torch.bfloat16:
            hip = ops._hip()
            a = x_act if x_act is not None else _lrelu(x)
            for i, (c1, c2, d) in enumerate(zip(self.convs1, self.convs2, self.dilation)):
                t = hip.conv1d_infer(a, _w(c1), c1.bias, get_padding(k, d), d, "lrelu")
                if i < n - 1:
                    x, a = hip.conv1d_infer(t, _w(c2), c2.bias, get_padding(k, 1), 1, None, resid=x, dual_lrelu=True)
                else:
                    x = hip.conv1d_infer(t, _w(c2), c2.bias, get_padding(k, 1), 1, None, resid=x, acc=acc,
                                         scale=out_scale, post_act="lrelu" if post_lrelu else None)
            return x
        for i, (c1, c2, d) in enumerate(zip(self.convs1, self.convs2, self.dilation)):
            a = x_act if (i == 0 and x_act is not None) else _lrelu(x)
            xt = ops.conv1d(a, _w(c1), c1.bias, get_padding(k, d), d, "lrelu")
            x = ops.conv1d(xt, _w(c2), c2.bias, get_padding(k, 1), 1, None) + x
        if acc is not None:
            x = acc.add_(x)
        x = x * out_scale if out_scale != 1.0 else x
        return _lrelu(x) if post_lrelu else x


    def forward_packed(self, x, vp, rate, acc=None, out_scale=1.0, x_act=None, post_lrelu=False):
        """``forward_cl`` on packed rows x [R*rate, C] (``hip.VocPack``: every conv zero-pads at its own
        utterance's ends, so each utterance is vocoded exactly as alone, with no padded rows)."""
        hip = ops._hip()
        k = self.kernel_size
        n = len(self.convs1)
        C = x.shape[-1]
        if self.fusable(C, x.shape[0]):
            if _WHOLE_BLOCK[0] and n == 3 and hip.resblock_fusable(C, k) and (C, k) not in _WHOLE_SKIP:
                return hip.resblock_fused_packed(x, vp, rate, self.convs1, self.convs2, self.dilation, LRELU_SLOPE,
                                                 acc=acc, out_scale=out_scale, post_lrelu=post_lrelu)
            for i, (c1, c2, d) in enumerate(zip(self.convs1, self.convs2, self.dilation)):
                last = i == n - 1
                x = hip.resblock_layer_packed(x, vp, rate, c1, c2, d, LRELU_SLOPE, acc=acc if last else None,
                                              out_scale=out_scale if last else 1.0, post_lrelu=post_lrelu and last)
            return x
        a = x_act if x_act is not None else _lrelu(x)
        for i, (c1, c2, d) in enumerate(zip(self.convs1, self.convs2, self.dilation)):
            t = hip.conv1d_infer_packed(a, vp, rate, _w(c1), c1.bias, get_padding(k, d), d, "lrelu")
            if i < n - 1:
                x, a = hip.conv1d_infer_packed(t, vp, rate, _w(c2), c2.bias, get_padding(k, 1), 1, None, resid=x,
                                               dual_lrelu=True)
            else:
                x = hip.conv1d_infer_packed(t, vp, rate, _w(c2), c2.bias, get_padding(k, 1), 1, None, resid=x, acc=acc,
                                            scale=out_scale, post_act="lrelu" if post_lrelu else None)
        return x

    def packed_tiles(self, C: int, rate: int, lens=()):
        """(rate, tile rows) pairs of this block's tiled kernels at channel width C for a packed batch of
        these frame lengths."""
        hip = ops._hip()
        if not self.fusable(C, sum(int(L) for L in lens) * rate):
            return []
        if (_WHOLE_BLOCK[0] and len(self.convs1) == 3 and hip.resblock_fusable(C, self.kernel_size)
                and (C, self.kernel_size) not in _WHOLE_SKIP):
            return [(rate, hip.rf_tile(C, self.kernel_size, self.dilation, lens, rate)[1])]
        return [(rate, hip.rb_layer_tile(C, self.kernel_size, lens, rate)[1])]


def _lrelu(x, slope=LRELU_SLOPE):
    return F.leaky_relu(x, slope)


class Generator(nn.Module):
    def __init__(self, h):
        super().__init__()
        self.h = h
        self.num_kernels = len(h.resblock_kernel_sizes)
        self.num_upsamples = len(h.upsample_rates)
        c0 = h.upsample_initial_channel
        self.conv_pre = weight_norm(nn.Conv1d(h.get("num_mels", 80), c0, 7, 1, padding=3))
        self.ups = nn.ModuleList()
        for i, (u, k) in enumerate(zip(h.upsample_rates, h.upsample_kernel_sizes)):
            self.ups.append(weight_norm(nn.ConvTranspose1d(c0 // 2 ** i, c0 // 2 ** (i + 1), k, u, padding=(k - u) // 2)))
        self.resblocks = nn.ModuleList()
        ch = c0
        for i in range(len(self.ups)):
            ch = c0 // 2 ** (i + 1)
            for k, d in zip(h.resblock_kernel_sizes, h.resblock_dilation_sizes):
                self.resblocks.append(ResBlock1(ch, k, d))
        self.conv_post = weight_norm(nn.Conv1d(ch, 1, 7, 1, padding=3))
        self.ups.apply(_init)
        self.conv_post.apply(_init)

    # ------------------------------------------------------------------ training (NCL)
    def forward(self, x):
        if x.is_cuda and _hip_train() and ops.use_hip(x) and self._hip_train_ok():
            return self._forward_hip_train(x)
        x = self.conv_pre(x)
        for i in range(self.num_upsamples):
            x = self.ups[i](F.leaky_relu(x, LRELU_SLOPE))
            xs = None
            for j in range(self.num_kernels):
                y = self.resblocks[i * self.num_kernels + j](x)
                xs = y if xs is None else xs + y
            x = xs / self.num_kernels
        x = self.conv_post(F.leaky_relu(x))  # default slope 0.01 (reference quirk, D16 preserved)
        return torch.tanh(x)

    def _hip_train_ok(self) -> bool:
        ok = self.conv_pre.in_channels % 8 == 0 and self.conv_pre.out_channels % 8 == 0
        for up in self.ups:
            K, s, pad = up.kernel_size[0], up.stride[0], up.padding[0]
            ok = ok and up.out_channels % 8 == 0 and K == s + 2 * pad and 0 <= pad <= s
        return ok

    def _forward_hip_train(self, x):
        """Generator forward for training on the HIP implicit-GEMM convs (channel-last bf16
        activations, fp32 weight-normed weights, autograd through ``ops.conv1d``): each upsampler
        is the 3-tap conv of ``convT_as_conv3`` (differentiable weight rearrangement) whose
        [B, T, s*Cout] output reshapes to the interleaved [B, T*s, Cout]; LeakyReLU / residual /
        MRF mean are torch elementwise ops; conv_post (one output channel, not MFMA-shaped) is a
        torch conv on the fp32 activation.  Same function as ``forward`` (reference
        ``hifigan/models.py:124-165``), returns [B, 1, T*hop] fp32."""
        B = x.shape[0]
        h = x.transpose(1, 2).to(torch.bfloat16).contiguous()
        glue = _glue(h)
        h = ops.conv1d(h, _wn(self.conv_pre), self.conv_pre.bias, 3, 1, None)
        nk = self.num_kernels
        for i in range(self.num_upsamples):
            up = self.ups[i]
            s = up.stride[0]
            wu = convT_as_conv3(_wn(up).float(), s, up.padding[0])
            bt = None if up.bias is None else up.bias.float().repeat(s)
            T = h.shape[1]
            h = ops.conv1d(glue.lrelu(h, LRELU_SLOPE), wu, bt, 1, 1, None).reshape(B, T * s, -1)
            rs = [self.resblocks[i * nk + j].forward_cl_train(h) for j in range(nk)]
            if nk == 3:
                h = glue.mean3(*rs)
            else:
                xs = rs[0]
                for r in rs[1:]:
                    xs = xs + r
                h = xs / nk
        cp = self.conv_post
        if glue is not _TorchGlue and cp.out_channels == 1:
            # lrelu(0.01) -> conv (Cout = 1) -> tanh on the HIP sconv kernel, fp32 [B, T, 1] -> [B, 1, T]
            return glue.conv_post_tanh(h, _wn(cp), cp.bias, cp.padding[0]).reshape(B, 1, -1)
        z = F.conv1d(F.leaky_relu(h.float(), 0.01).transpose(1, 2), _wn(cp), cp.bias, padding=3)
        return torch.tanh(z)

    # ------------------------------------------------------------------ inference (channel-last, HIP)
    def receptive_radius(self) -> int:
        """Mel frames on each side that one output sample depends on (through every layer, with
        the per-layer zero padding): walk the stack from conv_post back to conv_pre, adding each
        MRF's widest branch (sum over its layers of the dilated + plain conv half-widths) at that
        stage's rate and converting across each transposed conv (input index (o + pad - k) / s)."""
        nk = self.num_kernels
        r = (self.conv_post.kernel_size[0] - 1) // 2
        for i in reversed(range(self.num_upsamples)):
            blocks = [self.resblocks[i * nk + j] for j in range(nk)]
            r += max(sum(d * (b.kernel_size - 1) // 2 + (b.kernel_size - 1) // 2 for d in b.dilation) for b in blocks)
            up = self.ups[i]
            s, K, pad = up.stride[0], up.kernel_size[0], up.padding[0]
            r = -(-(r + max(pad, K - 1 - pad)) // s)
        return r + (self.conv_pre.kernel_size[0] - 1) // 2

    @staticmethod
    def length_buckets(lengths, T: int, halo: int, max_buckets: int = 8, bucket_cost: int = 512):
        """Split utterances (mel-frame ``lengths``, padded length ``T``) into at most ``max_buckets``
        groups of consecutive sorted lengths, each vocoded at ``min(T, max_len + halo)`` frames.
        Exact DP over the sorted lengths minimising sum(rows * frames) + ``bucket_cost`` per group
        (a group's launches / tails cost about that many frame-rows).  Returns [(indices, T_b)]."""
        import numpy as np

        L = np.asarray(lengths, dtype=np.int64)
        order = np.argsort(L, kind="stable")
        Ls = L[order]
        n = len(Ls)
        width = np.minimum(T, Ls + halo).astype(np.float64)  # a group ending at sorted row i-1 runs at width[i-1]
        ii = np.arange(n + 1)
        best = np.full(n + 1, np.inf)
        best[0] = 0.0
        cut = np.zeros((max_buckets + 1, n + 1), dtype=np.int64)
        table = [best]
        for j in range(1, max_buckets + 1):
            prev = table[-1]
            # cand[i, p] = prev[p] + (i - p) * width[i - 1] + bucket_cost, for p < i
            cand = prev[None, :] + (ii[:, None] - ii[None, :]) * np.concatenate([[0.0], width])[:, None] + bucket_cost
            cand[np.triu_indices(n + 1)] = np.inf
            cur = cand.min(axis=1)
            cur[0] = 0.0
            cut[j] = cand.argmin(axis=1)
            table.append(cur)
        j = int(np.argmin([t[n] for t in table[1:]])) + 1
        groups, i = [], n
        while i > 0:
            p = int(cut[j, i])
            groups.append((order[p:i], int(width[i - 1])))
            i, j = p, j - 1
        return groups[::-1]

    @torch.no_grad()
    def infer(self, mel_cl: torch.Tensor, int16_scale=None, lengths=None, max_buckets: int = 8,
              bucket_cost: int = 512) -> torch.Tensor:
        """mel [B, T, n_mel] (channel-last) -> wav [B, T*hop] in [-1, 1] (or int16 samples
        scaled by ``int16_scale``, fused into the conv_post kernel).

        ``lengths`` (host mel-frame counts): vocode length-sorted groups, each truncated to
        ``max_len + receptive_radius()`` frames, instead of the whole padded batch.  Exact for the
        valid samples ``[0, lengths[b] * hop)``: their dependency cone never reaches the truncation
        point (``tests/test_vocoder_buckets_cpu.py``); samples past a group's width are zero.  The
        reference vocodes the padded batch and trims (``utils/model.py:97-115``).

        On the GPU with ``lengths`` the batch is vocoded PACKED instead (``infer_packed``, ``_PACKED``): every
        utterance exactly as if alone, no padded rows; its samples past ``lengths[b] * hop`` are zero."""
        if (lengths is not None and _PACKED[0] and mel_cl.is_cuda and ops.use_hip(mel_cl)
                and mel_cl.dtype in (torch.float32, torch.bfloat16) and self.packable()):
            hop = 1
            for u in self.h.upsample_rates:
                hop *= u
            return self.infer_packed(mel_cl, lengths, int16_scale, width=mel_cl.shape[1] * hop)
        if lengths is not None and mel_cl.shape[0] > 1:
            B, T, _ = mel_cl.shape
            groups = self.length_buckets([int(v) for v in lengths], T, self.receptive_radius(), max_buckets,
                                         bucket_cost)
            if len(groups) > 1 or groups[0][1] < T:
                hop = 1
                for u in self.h.upsample_rates:
                    hop *= u
                out = None
                for idx, Tb in groups:
                    sel = torch.as_tensor(idx, device=mel_cl.device)
                    y = self.infer(mel_cl.index_select(0, sel)[:, :Tb].contiguous(), int16_scale)
                    if out is None:
                        out = y.new_zeros(B, T * hop)
                    out[sel, : y.shape[1]] = y
                return out
        if mel_cl.is_cuda and ops.use_hip(mel_cl):
            return self._infer_hip(mel_cl.to(torch.bfloat16).contiguous(), int16_scale)
        x = ops.conv1d(mel_cl, _w(self.conv_pre), self.conv_pre.bias, 3, 1, None)
        for i in range(self.num_upsamples):
            up = self.ups[i]
            x = conv_transpose_polyphase(_lrelu(x), _w(up), up.bias, up.stride[0], up.padding[0])
            blocks = [self.resblocks[i * self.num_kernels + j] for j in range(self.num_kernels)]
            x_act = _lrelu(x)
            xs = None
            for j, blk in enumerate(blocks):
                last = j == self.num_kernels - 1
                xs = blk.forward_cl(x, acc=xs, out_scale=(1.0 / self.num_kernels) if last else 1.0, x_act=x_act)
            x = xs
        w = _w(self.conv_post)
        y = torch.tanh(ref_conv_post(_lrelu(x, 0.01), w, self.conv_post.bias)).squeeze(-1)
        if int16_scale is not None:
            y = (y * int16_scale).clamp(-32768, 32767).to(torch.int16)
        return y

    def _ups_image(self, i):
        """(fp32 [s*Cout, Cin, 3] weight, bf16 [s*Cout][3][Cin] operand image, tiled bias) of
        upsampling layer i as one 3-tap convolution (``convT_as_conv3``), cached per weight version."""
        up = self.ups[i]
        w = _w(up)
        key = (w.data_ptr(), w._version, None if up.bias is None else up.bias._version)
        cache = self.__dict__.setdefault("_ups_cache", {})
        hit = cache.get(i)
        if hit is not None and hit[0] == key:
            return hit[1]
        wu = convT_as_conv3(w.detach().float(), up.stride[0], up.padding[0])
        if wu is None:
            val = None
        else:
            s = up.stride[0]
            bt = None if up.bias is None else up.bias.detach().float().repeat(s).contiguous()
            val = (wu, wu.permute(0, 2, 1).to(torch.bfloat16).contiguous(), bt)
        cache[i] = (key, val)
        return val

    def _infer_hip(self, mel, int16_scale):
        """GPU inference: every op is a HIP kernel, every activation / bias / accumulate sits in a
        GEMM epilogue.  conv_pre writes lrelu(x) (its only consumer is ups[0]); each upsampling conv
        is ONE implicit GEMM over a 3-tap window with N = stride * Cout whose output rows ARE the
        interleaved phases (no pad / stack / bias pass); each MRF's last branch writes
        lrelu(mean) for the next upsampling conv, or the raw mean for conv_post (slope 0.01, fused)."""
        hip = ops._hip()
        x = hip.conv1d_infer(mel, _w(self.conv_pre), self.conv_pre.bias, 3, 1, "lrelu")
        nk = self.num_kernels
        for i in range(self.num_upsamples):
            up = self.ups[i]
            s = up.stride[0]
            blocks = [self.resblocks[i * nk + j] for j in range(nk)]
            B, T, _ = x.shape
            img = self._ups_image(i)
            fused = all(b.fusable(up.weight.shape[1]) for b in blocks)
            x_act = None
            if img is None:  # generic ConvTranspose geometry: polyphase fallback on the same GEMM kernel
                y = conv_transpose_polyphase(x, _w(up), up.bias, s, up.padding[0])
            else:
                wu, wimg, bt = img
                if fused and _CONV3_SQ[0] and bt is not None and wu.shape[0] == wu.shape[1] in (64, 128):
                    y = hip.conv3_sq(x, wimg, bt)  # N = stride * Cout = Cin: the staged-tile kernel
                else:
                    # the 3-tap form's zero tap per phase half (K = 2s, pad = s/2): skipped per 256-column tile
                    cout = wu.shape[0] // s
                    ks_ = (s // 2) * cout if (_CONVT_KSPLIT[0] and up.kernel_size[0] == 2 * s
                                              and up.padding[0] * 2 == s) else 0
                    if fused:
                        y = hip.conv1d_infer(x, wu, bt, 1, 1, None, wimg=wimg, ksplit=ks_)
                    else:
                        y, x_act = hip.conv1d_infer(x, wu, bt, 1, 1, None, wimg=wimg, dual_lrelu=True, ksplit=ks_)
                y = y.view(B, T * s, -1)
                if x_act is not None:
                    x_act = x_act.view(B, T * s, -1)
            post = i < self.num_upsamples - 1
            xs = None
            for j, blk in enumerate(blocks):
                last = j == nk - 1
                xs = blk.forward_cl(y, acc=xs, out_scale=(1.0 / nk) if last else 1.0, x_act=x_act,
                                    post_lrelu=post and last)
            x = xs
        w = _w(self.conv_post)  # [1, C, 7]: N = 1 output -> VALU kernel (lrelu + conv + tanh [+ int16] fused)
        if x.shape[-1] in (8, 32):
            return hip.conv_post(x, w, self.conv_post.bias, 0.01, int16_scale)
        y = torch.tanh(ref_conv_post(_lrelu(x, 0.01), w, self.conv_post.bias)).squeeze(-1)
        if int16_scale is not None:
            y = (y * int16_scale).clamp(-32768, 32767).to(torch.int16)
        return y

    # ------------------------------------------------------------------ packed (length-exact) inference
    def packable(self) -> bool:
        """Every upsampler has the 3-tap form and conv_post the VALU kernel: ``infer_packed`` applies."""
        c_last = self.h.upsample_initial_channel // 2 ** self.num_upsamples
        return c_last in (8, 32) and all(self._ups_image(i) is not None for i in range(self.num_upsamples))

    @torch.no_grad()
    def infer_packed(self, mel: torch.Tensor, lengths, int16_scale=None, width=None) -> torch.Tensor:
        """mel [B, M, n_mel] (padded, channel-last, fp32 / bf16) + host frame ``lengths`` -> wav [B, W] (W = ``width``
        or max(lengths) * hop; int16 when ``int16_scale``), samples past ``lengths[b] * hop`` zero.

        The utterances' valid frames are packed back to back ([R, C] rows per stage, ``hip.VocPack``) and every
        kernel zero-pads each conv at the utterance's own ends (the GEMM stages through a per-row position table,
        the tiled ResBlock / upsampler / conv_post kernels through per-tile tables whose tiles never straddle two
        utterances), so each utterance is vocoded exactly as if alone -- the reference vocodes the padded batch
        and trims (``utils/model.py:97-115``) -- with no padded rows at any stage and one launch per layer for the
        whole batch (the length-bucketed ``infer`` pads each bucket to its longest utterance + the receptive radius:
        ~10 % extra rows at 8 buckets, and 8x the launches)."""
        hip = ops._hip()
        dev = mel.device
        rows_in = mel.dim() == 2  # already packed [R, n_mel] rows in ``lengths`` order (FastSpeech2.infer_packed)
        B = len(lengths) if rows_in else mel.shape[0]
        lens = [max(0, int(v)) for v in lengths] if rows_in else [max(0, min(int(v), mel.shape[1])) for v in lengths]
        if rows_in:
            assert mel.shape[0] == sum(lens), "infer_packed: packed rows vs lengths"
        hop = 1
        for u in self.h.upsample_rates:
            hop *= u
        W = int(width) if width is not None else max(lens) * hop
        nk = self.num_kernels
        # every (rate, tile height) the tiled kernels will ask for: one host-built table buffer, one H2D copy
        geoms, rate = [], 1
        for i in range(self.num_upsamples):
            up = self.ups[i]
            s = up.stride[0]
            blocks = [self.resblocks[i * nk + j] for j in range(nk)]
            wu, _, bt = self._ups_image(i)
            cout = wu.shape[0] // s
            if all(b.fusable(cout, sum(lens) * rate * s) for b in blocks) and _CONV3_SQ[0] and bt is not None and \
                    wu.shape[0] == wu.shape[1] in (64, 128):
                geoms.append((rate, hip.voc_tile_rows(2, wu.shape[1])))
            rate *= s
            for blk in blocks:
                geoms.extend(blk.packed_tiles(cout, rate, lens))
        c_last = self.h.upsample_initial_channel // 2 ** self.num_upsamples
        geoms.append((rate, hip.voc_tile_rows("post", c_last)))
        vp = hip.voc_pack_for(lens, dev, geoms)
        out = torch.zeros(B, W, device=dev, dtype=torch.int16 if int16_scale is not None else torch.float32)
        if vp.R == 0:
            return out
        x = mel.to(torch.bfloat16).contiguous() if rows_in else hip.voc_pack(mel, vp)
        x = hip.conv1d_infer_packed(x, vp, 1, _w(self.conv_pre), self.conv_pre.bias, 3, 1, "lrelu")
        rate = 1
        for i in range(self.num_upsamples):
            up = self.ups[i]
            s = up.stride[0]
            blocks = [self.resblocks[i * nk + j] for j in range(nk)]
            wu, wimg, bt = self._ups_image(i)
            cout = wu.shape[0] // s
            # lrelu(y) as a second GEMM output only when some branch runs on the GEMM path (it needs it as input)
            fused = all(b.fusable(cout, vp.R * rate * s) for b in blocks)
            x_act = None
            if fused and _CONV3_SQ[0] and bt is not None and wu.shape[0] == wu.shape[1] in (64, 128):
                y = hip.conv3_sq_packed(x, vp, rate, wimg, bt)
            else:
                ks_ = (s // 2) * cout if (_CONVT_KSPLIT[0] and up.kernel_size[0] == 2 * s
                                          and up.padding[0] * 2 == s) else 0
                if fused:
                    y = hip.conv1d_infer_packed(x, vp, rate, wu, bt, 1, 1, None, wimg=wimg, ksplit=ks_)
                else:
                    y, x_act = hip.conv1d_infer_packed(x, vp, rate, wu, bt, 1, 1, None, wimg=wimg, dual_lrelu=True,
                                                       ksplit=ks_)
            # [R*rate, s*Cout] rows ARE the interleaved [R*rate*s, Cout] rows (each utterance's block stays whole)
            rate *= s
            y = y.view(vp.R * rate, cout)
            if x_act is not None:
                x_act = x_act.view(vp.R * rate, cout)
            post = i < self.num_upsamples - 1
            xs = None
            for j, blk in enumerate(blocks):
                last = j == nk - 1
                xs = blk.forward_packed(y, vp, rate, acc=xs, out_scale=(1.0 / nk) if last else 1.0, x_act=x_act,
                                        post_lrelu=post and last)
            x = xs
        return hip.conv_post_packed(x, vp, rate, _w(self.conv_post), self.conv_post.bias, out, 0.01, int16_scale)

    def fold_weight_norm(self):
        for m in self.modules():
            if isinstance(m, (nn.Conv1d, nn.ConvTranspose1d)) and hasattr(m, "weight_g"):
                torch.nn.utils.remove_weight_norm(m)
        return self

    remove_weight_norm = fold_weight_norm


# the C = 256 MRF (K = 3 / 7 branches) on the tall per-layer ResBlock kernel instead of two GEMMs per layer pair
_RB256 = [True]
# row count from which the C = 256 MRF takes the kernel path: above the skinny GEMM kernel's range (<= 1024 rows,
# csrc/k_gemm.hip), whose GEMMs beat it at batch 1 (904 rows: b1 1.661 / 1.673 ms vs 1.728 / 1.750 ms); the kernel
# beat the tile GEMMs at every size (profiles/r6_b1_latency.txt)
_RB256_MIN_ROWS = [1025]
# GPU inference with host lengths: the packed, length-exact path (infer_packed) instead of length buckets
_PACKED = [True]
# square upsamplers (N = stride * Cout = Cin in {64, 128}) on ``hip.conv3_sq`` instead of the generic GEMM
_CONV3_SQ = [True]
# the other upsamplers' 3-tap GEMM skips each 256-column tile's all-zero tap (ConvGeom::ksplit in csrc/k_gemm.hip)
_CONVT_KSPLIT = [True]


def ref_conv_post(x, w, b):
    return ops.ref.conv1d(x.float(), w.float(), None if b is None else b.float(), 3, 1, None)


def convT_as_conv3(w, stride: int, pad: int):
    """ConvTranspose1d weight [Cin, Cout, K] -> an ordinary 3-tap conv weight [stride*Cout, Cin, 3].

    y[s*q + r] = sum_k x[q + (r + pad - k)/s] w[:, :, k] over the taps k with (r + pad - k) divisible
    by s.  When K == s + 2*pad and pad <= s (every HiFi-GAN upsampler: K = 2s, pad = s/2) the input
    offset (r + pad - k)/s is always -1, 0 or +1, so output phase r of frame q is a 3-tap conv of
    x[q-1 .. q+1] with W3[r*Cout + co, cin, t] = w[cin, co, r + pad - s*(t-1)] (zero where that tap does
    not exist).  The GEMM output [B, T, s*Cout] then IS the interleaved [B, T*s, Cout] result.  1.5x the
    MACs of the exact polyphase form, but one wide GEMM (N = s*Cout) with no interleave / pad / bias
    pass.  Returns None for other geometries."""
    Cin, Cout, K = w.shape
    s = int(stride)
    if K != s + 2 * pad or pad > s or pad < 0:
        return None
    wu = w.new_zeros(s, Cout, Cin, 3)
    for r in range(s):
        for t in range(3):
            k = r + pad - s * (t - 1)
            if 0 <= k < K:
                wu[r, :, :, t] = w[:, :, k].t()
    return wu.reshape(s * Cout, Cin, 3).contiguous()


def conv_transpose_polyphase(x, w, b, stride: int, pad: int):
    """ConvTranspose1d as ``stride`` phase convolutions (channel-last).

    y[s*q + r] = sum_j x[q - j + c_r] * w[:, :, r + pad ... ] -- for output phase r, the taps
    k = (r + pad) mod s + s*j hit input index (s*q + r + pad - k)/s.  Each phase is a normal
    (correlation) conv over x with the tap-reversed sub-kernel, evaluated on the MFMA
    implicit-GEMM kernel; phases are interleaved into the output.
    x [B, T, Cin], w [Cin, Cout, K] (PyTorch ConvTranspose layout).
    """
    B, T, Cin = x.shape
    Cout, K = w.shape[1], w.shape[2]
    T_out = (T - 1) * stride - 2 * pad + K
    outs = []
    for r in range(stride):
        k0 = (r + pad) % stride
        ks = list(range(k0, K, stride))
        if not ks:
            outs.append(torch.zeros(B, (T_out - r + stride - 1) // stride, Cout, device=x.device, dtype=x.dtype))
            continue
        off = (r + pad - k0) // stride  # input index of tap j=0 for q=0
        sub = w[:, :, ks].permute(1, 0, 2).flip(2).contiguous()  # [Cout, Cin, J] correlation taps
        J = len(ks)
        n_q = (T_out - r + stride - 1) // stride
        # y_r[q] = sum_j x[q + off - j] * w[..., k0 + s*j]  ==  corr(x_padded, sub)[q + off - (J-1)]
        left = (J - 1) - off
        right = max(0, n_q + off - T)
        xp = x
        if left > 0 or right > 0:
            xp = F.pad(x, (0, 0, max(left, 0), right))
        start = 0 if left >= 0 else -left
        y = ops.conv1d(xp.contiguous(), sub, None, 0, 1, None)
        y = y[:, start:start + n_q]
        outs.append(y)
    y = torch.stack([o[:, : (T_out + stride - 1) // stride] if o.shape[1] >= (T_out + stride - 1) // stride
                     else F.pad(o, (0, 0, 0, (T_out + stride - 1) // stride - o.shape[1])) for o in outs], dim=2)
    y = y.reshape(B, -1, Cout)[:, :T_out]
    if b is not None:
        y = y + b.to(y.dtype)
    return y


# ------------------------------------------------------------------ discriminators (training)
class DiscriminatorP(nn.Module):
    def __init__(self, period, kernel_size=5, stride=3, use_spectral_norm=False):
        super().__init__()
        self.period = period
        norm_f = spectral_norm if use_spectral_norm else weight_norm
        chans = [1, 32, 128, 512, 1024]
        self.convs = nn.ModuleList(
            [norm_f(nn.Conv2d(chans[i], chans[i + 1], (kernel_size, 1), (stride, 1), padding=(get_padding(5, 1), 0)))
             for i in range(4)]
            + [norm_f(nn.Conv2d(1024, 1024, (kernel_size, 1), 1, padding=(2, 0)))])
        self.conv_post = norm_f(nn.Conv2d(1024, 1, (3, 1), 1, padding=(1, 0)))

    def forward(self, x):
        fmap = []
        b, c, t = x.shape
        if t % self.period:
            n_pad = self.period - (t % self.period)
            x = F.pad(x, (0, n_pad), "reflect")
            t = t + n_pad
        x = x.view(b, c, t // self.period, self.period)
        for layer in self.convs:
            x = F.leaky_relu(layer(x), LRELU_SLOPE)
            fmap.append(x)
        x = self.conv_post(x)
        fmap.append(x)
        return torch.flatten(x, 1, -1), fmap


class MultiPeriodDiscriminator(nn.Module):
    def __init__(self, periods=(2, 3, 5, 7, 11)):
        super().__init__()
        self.discriminators = nn.ModuleList(DiscriminatorP(p) for p in periods)

    def forward(self, y, y_hat):
        rs, gs, frs, fgs = [], [], [], []
        for d in self.discriminators:
            a, fa = d(y)
            b, fb = d(y_hat)
            rs.append(a); frs.append(fa); gs.append(b); fgs.append(fb)
        return rs, gs, frs, fgs


class DiscriminatorS(nn.Module):
    def __init__(self, use_spectral_norm=False):
        super().__init__()
        norm_f = spectral_norm if use_spectral_norm else weight_norm
        self.convs = nn.ModuleList([
            norm_f(nn.Conv1d(1, 128, 15, 1, padding=7)),
            norm_f(nn.Conv1d(128, 128, 41, 2, groups=4, padding=20)),
            norm_f(nn.Conv1d(128, 256, 41, 2, groups=16, padding=20)),
            norm_f(nn.Conv1d(256, 512, 41, 4, groups=16, padding=20)),
            norm_f(nn.Conv1d(512, 1024, 41, 4, groups=16, padding=20)),
            norm_f(nn.Conv1d(1024, 1024, 41, 1, groups=16, padding=20)),
            norm_f(nn.Conv1d(1024, 1024, 5, 1, padding=2)),
        ])
        self.conv_post = norm_f(nn.Conv1d(1024, 1, 3, 1, padding=1))

    def forward(self, x):
        fmap = []
        for layer in self.convs:
            x = F.leaky_relu(layer(x), LRELU_SLOPE)
            fmap.append(x)
        x = self.conv_post(x)
        fmap.append(x)
        return torch.flatten(x, 1, -1), fmap


class MultiScaleDiscriminator(nn.Module):
    def __init__(self):
        super().__init__()
        self.discriminators = nn.ModuleList([DiscriminatorS(use_spectral_norm=True), DiscriminatorS(), DiscriminatorS()])
        self.meanpools = nn.ModuleList([nn.AvgPool1d(4, 2, padding=2), nn.AvgPool1d(4, 2, padding=2)])

    def forward(self, y, y_hat):
        rs, gs, frs, fgs = [], [], [], []
        for i, d in enumerate(self.discriminators):
            if i:
                y = self.meanpools[i - 1](y)
                y_hat = self.meanpools[i - 1](y_hat)
            a, fa = d(y)
            b, fb = d(y_hat)
            rs.append(a); frs.append(fa); gs.append(b); fgs.append(fb)
        return rs, gs, frs, fgs


def feature_loss(fmap_r, fmap_g):
    loss = 0.0
    for dr, dg in zip(fmap_r, fmap_g):
        for rl, gl in zip(dr, dg):
            loss = loss + torch.mean(torch.abs(rl - gl))
    return loss * 2


def discriminator_loss(real_outs, gen_outs):
    loss = 0.0
    r_losses, g_losses = [], []
    for dr, dg in zip(real_outs, gen_outs):
        r = torch.mean((1 - dr) ** 2)
        g = torch.mean(dg ** 2)
        loss = loss + r + g
        r_losses.append(r.detach())
        g_losses.append(g.detach())
    return loss, r_losses, g_losses


def generator_loss(gen_outs):
    loss = 0.0
    losses: List[torch.Tensor] = []
    for dg in gen_outs:
        l_ = torch.mean((1 - dg) ** 2)
        losses.append(l_)
        loss = loss + l_
    return loss, losses
