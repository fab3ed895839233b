"""Speaking-style encoders producing FiLM (gamma, beta).

* ``ReferenceEncoder`` -- the reference's FiLM variant (``model/modules.py:307-406``):
  3 x (Conv1d k3 -> ReLU -> LN -> Dropout) on the mel, + PE(1024), LinearNorm
  1024->256, 4 FFT blocks (8 heads, d_k 32, FFN k=[3,3], no FiLM), mean over time
  (dividing by the padded length), LinearNorm 256->512 -> (gamma, beta).
* ``GlobalStyleTokens`` -- the GST path that the reference only declares in a
  commented-out config block (``config/BC2013/model.yaml:33-39``) and in its
  README research goal: Wang et al. 2018 reference encoder (6 x Conv2d 3x3/s2 +
  BN + ReLU -> GRU) + multi-head attention over a bank of style tokens.  The
  resulting style embedding is projected to the same FiLM (gamma, beta), so it
  drives exactly the FiLM sites the reference uses.  ``from_token_weights`` gives
  direct token-weight style control at synthesis (no reference audio).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .layers import ConvHolder, FFTBlock, LinearNorm


class ReferenceEncoder(nn.Module):
    def __init__(self, preprocess_config, model_config, mean_over_valid: bool = False):
        super().__init__()
        rc = model_config["reference_encoder"]
        n_mel = preprocess_config["preprocessing"]["mel"]["n_mel_channels"]
        self.max_seq_len = model_config["max_seq_len"] + 1  # reference quirk: 1001
        k = rc["conv_kernel_size"]
        self.filter_size = fs = rc["conv_filter_size"]
        self.d_model = d = rc["encoder_hidden"]
        nh = rc["encoder_head"]
        self.dropout = rc["dropout"]
        self.mean_over_valid = mean_over_valid
        self.layer_stack = nn.ModuleList(
            nn.Sequential(ConvHolder(n_mel if i == 0 else fs, fs, k), nn.ReLU(), nn.LayerNorm(fs), nn.Dropout(self.dropout))
            for i in range(rc["conv_layer"])
        )
        self.position_enc = nn.Parameter(ops.sinusoid_table(self.max_seq_len, fs).unsqueeze(0), requires_grad=False)
        self.fftb_linear = LinearNorm(fs, d)
        self.fftb_stack = nn.ModuleList(
            FFTBlock(d, nh, d // nh, d // nh, fs, [k, k], dropout=self.dropout, film=False) for _ in range(rc["encoder_layer"])
        )
        self.feature_wise_affine = LinearNorm(d, 2 * d)

    def forward(self, mel, mel_lens, max_len=None):
        host = getattr(mel_lens, "host_lengths", None)
        M = mel.shape[1]
        if (host is not None and not self.mean_over_valid and ops.use_hip(mel)
                and (self.training or M <= self.max_seq_len)):
            return self._forward_packed(mel, mel_lens, host)
        h = mel
        for seq in self.layer_stack:
            conv, ln = seq[0], seq[2]
            h = conv(h, act="relu")
            h = ops.add_layernorm(h, None, ln.weight, ln.bias, post_drop=self.dropout, training=self.training)
        # pad frames are zeroed once after the whole conv stack (modules.py:370-371)
        h = h.masked_fill(ops.lengths_to_mask(mel_lens, M).unsqueeze(-1), 0.0)
        if (not self.training) and M > self.max_seq_len:
            pe = ops.sinusoid_table(M, self.filter_size, device=h.device)
        else:
            M = min(M, self.max_seq_len)
            h = h[:, :M]
            pe = self.position_enc[0, :M]
        lens = mel_lens.clamp(max=M)
        h = h + pe.to(h.dtype).unsqueeze(0)
        h = self.fftb_linear(h)
        for blk in self.fftb_stack:
            h = blk(h, lens, None)
        if self.mean_over_valid:
            pooled = h.float().sum(1) / lens.clamp(min=1).unsqueeze(1).float()
        else:
            pooled = ops.seq_mean(h)  # over the padded length, like the reference (D8)
        gb = self.feature_wise_affine(pooled.to(h.dtype))
        return gb[:, : self.d_model], gb[:, self.d_model:]

    def halo(self) -> int:
        """Frames past a sequence's end that the conv stack must still compute for its valid
        outputs to equal the padded computation: the reference zeroes pads only AFTER the stack
        (``model/modules.py:366-371``), so layer l sees the previous layers' non-zero values in the
        first (k-1)/2 * (layers-1) pad frames."""
        k = self.layer_stack[0][0].conv.kernel_size[0]
        return (k - 1) // 2 * (len(self.layer_stack) - 1)

    def _forward_packed(self, mel, mel_lens, host):
        """Valid frames only (``ops/packing.py``), same result as the padded path.

        * conv stack on rows packed with a halo of ``halo()`` pad frames per sequence (mel pad rows
          are zero, as in the padded batch); the packed convs zero-pad past each packed length, which
          is exactly where the padded path's inputs are zero or irrelevant to the valid outputs;
        * the FFT blocks on the valid rows (repacked from the halo layout with the PE added): pad rows
          there are zeroed after every sublayer, so they contribute nothing to the attention (masked
          keys), to the k=3 FFN convs or to the mean, which still divides by the padded length (D8).
        The host lengths size both packings without a device sync."""
        Mf = mel.shape[1]
        hl = self.halo()
        R_h = int(sum(min(int(v) + hl, Mf) for v in host))
        pk_h = ops.PackInfo.build((mel_lens.clamp(max=Mf) + hl).clamp(max=Mf), Mf, R_h)
        h = ops.pack_rows(mel, pk_h)
        for seq in self.layer_stack:
            conv, ln = seq[0], seq[2]
            h = ops.conv1d(h, conv.conv.weight, conv.conv.bias, conv.pad, conv.dil, "relu", pack=pk_h)
            h = ops.add_layernorm(h, None, ln.weight, ln.bias, post_drop=self.dropout, training=self.training)
        M = min(Mf, self.max_seq_len)
        R = int(sum(min(int(v), M) for v in host))
        pk = ops.PackInfo.build(mel_lens, M, R)
        x = ops.repack_rows(h, pk_h, pk, self.position_enc[0, :M])
        x = self.fftb_linear(x)
        for blk in self.fftb_stack:
            x = blk(x, pk.lens, None, pack=pk)
        pooled = ops.seq_mean(x, divisor=M, pack=pk)
        gb = self.feature_wise_affine(pooled.to(x.dtype))
        return gb[:, : self.d_model], gb[:, self.d_model:]


class GlobalStyleTokens(nn.Module):
    def __init__(self, preprocess_config, model_config):
        super().__init__()
        g = model_config["gst"]
        n_mel = preprocess_config["preprocessing"]["mel"]["n_mel_channels"]
        filters = [1] + list(g["conv_filters"])
        self.convs = nn.ModuleList(nn.Conv2d(filters[i], filters[i + 1], 3, 2, 1) for i in range(len(filters) - 1))
        self.bns = nn.ModuleList(nn.BatchNorm2d(c) for c in filters[1:])
        freq = n_mel
        for _ in range(len(filters) - 1):
            freq = (freq - 3 + 2) // 2 + 1
        self.gru = nn.GRU(filters[-1] * freq, g["gru_hidden"], batch_first=True)
        self.n_head = g["attn_head"]
        self.token_size = g["token_size"]
        assert self.token_size % self.n_head == 0
        self.embed = nn.Parameter(torch.randn(g["n_style_token"], self.token_size // self.n_head) * 0.5)
        self.w_query = nn.Linear(g["gru_hidden"], self.token_size, bias=False)
        self.w_key = nn.Linear(self.token_size // self.n_head, self.token_size, bias=False)
        self.w_value = nn.Linear(self.token_size // self.n_head, self.token_size, bias=False)
        d = model_config["transformer"]["encoder_hidden"]
        self.d_model = d
        self.feature_wise_affine = LinearNorm(self.token_size, 2 * d)

    def reference_embedding(self, mel, mel_lens):
        """mel [B, T, n_mel] -> last valid GRU state [B, H] (fp32).

        Channel-last throughout: the mel is an NHWC image [B, T, n_mel, 1]; each layer is
        ``ops.conv2d_s2`` (im2col + MFMA GEMM on the GPU) and ``ops.bn_act`` (BatchNorm2d batch
        statistics over all B*H*W positions, fused ReLU).  The GRU input features are ordered
        (channel, frequency) like the NCHW formulation, so the GRU weights mean the same thing."""
        x = mel.unsqueeze(-1)
        if not ops.use_hip(x):
            x = x.float()
        if not self.training and not ops.needs_grad(mel, *self.convs.parameters(), *self.bns.parameters()):
            # eval BatchNorm is a per-channel affine: folded into the conv, ReLU in its GEMM epilogue
            for prep in self.folded_convs():
                x = ops.conv2d_s2_infer(x, prep, "relu")
        else:
            for conv, bn in zip(self.convs, self.bns):
                y = ops.conv2d_s2(x, conv.weight, conv.bias)
                B, Ho, Wo, C = y.shape
                x = ops.bn_act(y.reshape(B, Ho * Wo, C), bn, self.training, "relu", 0.0).view(B, Ho, Wo, C)
        # each stride-2 conv maps a length l to (l - 1) // 2 + 1 = ceil(l / 2), so n of them give ceil(l / 2^n) and
        # the last valid GRU step is ceil(l / 2^n) - 1 = (l - 1) >> n (-1 -> 0 for an empty mel): three tiny device
        # ops instead of three per layer
        n = len(self.convs)
        B, T, Fq, C = x.shape
        x = x.permute(0, 1, 3, 2).reshape(B, T, C * Fq)
        return ops.gru_last(x, self.gru, ((mel_lens - 1) >> n).clamp(0, T - 1))

    def folded_convs(self):
        """Per layer the ``ops.conv2d_s2_prepare`` operand of (W * s, b * s + t), s = gamma / sqrt(running_var +
        eps), t = beta - running_mean * s: Conv2d + eval BatchNorm2d as one conv.  Cached per parameter / buffer
        version (not registered: never in the state dict); on the GPU the weight images are built here once
        instead of per call (batch-1 serving is launch-bound)."""
        ts = []
        for conv, bn in zip(self.convs, self.bns):
            ts += [conv.weight, conv.bias, bn.weight, bn.bias, bn.running_mean, bn.running_var]
        key = tuple((t.data_ptr(), t._version, t.device) for t in ts if t is not None)
        hit = self.__dict__.get("_fold")
        if hit is not None and hit[0] == key:
            return hit[1]
        out = []
        with torch.no_grad():
            for conv, bn in zip(self.convs, self.bns):
                s = bn.weight.float() * torch.rsqrt(bn.running_var.float() + bn.eps)
                t = bn.bias.float() - bn.running_mean.float() * s
                b = conv.bias.float() if conv.bias is not None else torch.zeros_like(s)
                out.append(ops.conv2d_s2_prepare(conv.weight.float() * s.view(-1, 1, 1, 1), b * s + t))
        self.__dict__["_fold"] = (key, out)
        return out

    def token_bank(self):
        """Keys / values of the style-token bank, [heads, n_tok, token_size/heads] each."""
        return ops.token_bank(self.embed, self.w_key.weight, self.w_value.weight, self.n_head)

    def token_attention(self, query):
        """query [B, token_size] -> style embedding [B, token_size] and weights [B, heads, n_tok]."""
        k, v = self.token_bank()
        return ops.token_attention(query, k, v)

    def _film(self, style_emb):
        gb = self.feature_wise_affine(style_emb)
        return gb[:, : self.d_model], gb[:, self.d_model:]

    def forward(self, mel, mel_lens, max_len=None):
        ref = self.reference_embedding(mel, mel_lens)
        q = ops.linear(ref.to(mel.dtype), self.w_query.weight, None)
        style, _ = self.token_attention(q)
        return self._film(style.to(mel.dtype))

    def from_token_weights(self, weights):
        """weights [B, n_tok] (or [B, heads, n_tok]) -> FiLM params; style without audio."""
        _, v = self.token_bank()  # [h, N, d]
        if weights.dim() == 2:
            weights = weights.unsqueeze(1).expand(-1, self.n_head, -1)
        o = torch.einsum("bhn,hnd->bhd", weights.float(), v.float()).reshape(weights.shape[0], self.token_size)
        return self._film(o)
