"""FastSpeech2 with optional speaking-style conditioning (FiLM reference encoder or GST).

Forward order and outputs follow the reference's ``model/fastspeech2.py:44-120``:
masks -> style encoder (gamma, beta) -> encoder (FiLM) -> + speaker embedding ->
VarianceAdaptor -> decoder (FiLM) -> mel_linear -> PostNet residual, returning
the same 10-tuple.  Activations are channel-last in the compute dtype (bf16 on
MI355X, fp32 on CPU); mel outputs are fp32.

Fixed reference bugs: no per-forward debug prints (D3),
style encoder optional (D2), consistent rounding of controlled durations (D11),
device derived from tensors (D19), synthesis without a reference mel uses a
neutral style.
"""
from __future__ import annotations

import json
import math
import os
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..config import style_mode
from ..text.symbols import symbols
from .layers import FFTBlock, FiLM, LinearNorm, PostNet, fused_param_groups
from .style import GlobalStyleTokens, ReferenceEncoder


def _pe_param(n_position: int, d: int) -> nn.Parameter:
    return nn.Parameter(ops.sinusoid_table(n_position, d).unsqueeze(0), requires_grad=False)


_PE_CAST = ops.IdCache()  # positional table -> ((dtype, version, address), cast copy)


def positional_rows(pe_param: torch.Tensor, length: int, d: int, device, dtype=None) -> torch.Tensor:
    """First ``length`` sinusoid rows; beyond the stored table (eval on long
    inputs, reference ``transformer/Models.py:82-87``) they are generated.  ``dtype``: the rows in that dtype,
    from a per-dtype copy of the (constant, non-trainable) table made once."""
    if length <= pe_param.shape[1]:
        if dtype is None or dtype == pe_param.dtype:
            return pe_param[0, :length]
        hit = _PE_CAST.get(pe_param)
        if hit is None or hit[0] != (dtype, pe_param._version, pe_param.data_ptr()):
            hit = ((dtype, pe_param._version, pe_param.data_ptr()), pe_param.detach()[0].to(dtype).contiguous())
            _PE_CAST.put(pe_param, hit)
        return hit[1][:length]
    t = ops.sinusoid_table(length, d, device=device)
    return t if dtype is None else t.to(dtype)


class Encoder(nn.Module):
    """Phoneme embedding + PE + N FFT blocks (``transformer/Models.py:33-101``)."""

    def __init__(self, config, film=False):
        super().__init__()
        tr = config["transformer"]
        d = tr["encoder_hidden"]
        self.max_seq_len = config["max_seq_len"]
        self.d_model = d
        self.src_word_emb = nn.Embedding(len(symbols) + 1, d, padding_idx=0)
        self.position_enc = _pe_param(self.max_seq_len + 1, d)
        nh = tr["encoder_head"]
        self.layer_stack = nn.ModuleList(
            FFTBlock(d, nh, d // nh, d // nh, tr["conv_filter_size"], tr["conv_kernel_size"], tr["encoder_dropout"], film=film)
            for _ in range(tr["encoder_layer"])
        )

    def forward(self, texts, src_lens, style=None, compute_dtype=torch.float32):
        T = texts.shape[1]
        pe = positional_rows(self.position_enc, T, self.d_model, texts.device, compute_dtype)
        # the fp32 table itself: the HIP op reads its cached bf16 image and writes the gradient slot
        tab = self.src_word_emb.weight if ops.use_hip(texts) else self.src_word_emb.weight.to(compute_dtype)
        x = ops.embed_add_pe(texts, tab, pe)
        for layer in self.layer_stack:
            x = layer(x, src_lens, style)
        return x


class Decoder(nn.Module):
    """PE + N FFT blocks; training truncates to ``max_seq_len`` frames
    (``transformer/Models.py:104-170``)."""

    def __init__(self, config, film=False):
        super().__init__()
        tr = config["transformer"]
        d = tr["decoder_hidden"]
        self.max_seq_len = config["max_seq_len"]
        self.d_model = d
        self.position_enc = _pe_param(self.max_seq_len + 1, d)
        nh = tr["decoder_head"]
        self.layer_stack = nn.ModuleList(
            FFTBlock(d, nh, d // nh, d // nh, tr["conv_filter_size"], tr["conv_kernel_size"], tr["decoder_dropout"], film=film)
            for _ in range(tr["decoder_layer"])
        )

    def forward(self, x, mel_lens, style=None):
        M = x.shape[1]
        if self.training and M > self.max_seq_len:
            M = self.max_seq_len
            x = x[:, :M]
            mel_lens = mel_lens.clamp(max=M)
        pe = positional_rows(self.position_enc, M, self.d_model, x.device, x.dtype)
        x = x + pe.unsqueeze(0)
        for layer in self.layer_stack:
            x = layer(x, mel_lens, style)
        return x, mel_lens

    def forward_packed(self, x_phone, durations, mel_lens, M, R, style=None):
        """Length regulation + decoder over the valid frames only (``ops/packing.py``).

        Same result as ``forward(LR(x_phone))`` on every valid frame; returns the packed
        ``[1, R, C]`` output, the (truncated) lengths and the PackInfo."""
        if self.training and M > self.max_seq_len:
            M = self.max_seq_len
        dec_lens = mel_lens.clamp(max=M)
        pk = ops.PackInfo.build(dec_lens, M, R)
        pe = positional_rows(self.position_enc, M, self.d_model, x_phone.device, x_phone.dtype)
        x = ops.length_regulate_packed(x_phone, durations, pk, pe)
        for layer in self.layer_stack:
            x = layer(x, dec_lens, style, pack=pk)
        return x, dec_lens, pk


class VariancePredictor(nn.Module):
    """[Conv1d k3 -> ReLU -> LN -> Dropout] x2 -> [FiLM] -> Linear(1) -> mask
    (``model/modules.py:204-259``)."""

    def __init__(self, model_config, film=False):
        super().__init__()
        d_in = model_config["transformer"]["encoder_hidden"]
        vp = model_config["variance_predictor"]
        fs, k, self.dropout = vp["filter_size"], vp["kernel_size"], vp["dropout"]
        from collections import OrderedDict

        from .layers import ConvHolder

        self.conv_layer = nn.Sequential(OrderedDict([
            ("conv1d_1", ConvHolder(d_in, fs, k)),
            ("relu_1", nn.ReLU()),
            ("layer_norm_1", nn.LayerNorm(fs)),
            ("dropout_1", nn.Dropout(self.dropout)),
            ("conv1d_2", ConvHolder(fs, fs, k)),
            ("relu_2", nn.ReLU()),
            ("layer_norm_2", nn.LayerNorm(fs)),
            ("dropout_2", nn.Dropout(self.dropout)),
        ]))
        if film:
            self.film = FiLM()
        self.linear_layer = nn.Linear(fs, 1)

    def forward(self, x, lengths, style=None):
        cl = self.conv_layer
        c1 = cl.conv1d_1
        h = ops.conv_relu_layernorm(x, c1.conv.weight, c1.conv.bias, c1.pad, c1.dil, cl.layer_norm_1.weight,
                                    cl.layer_norm_1.bias, post_drop=self.dropout, training=self.training)
        return self.rest(h, lengths, style)

    def first_block(self):
        """(conv weight, conv bias, (LN weight, LN bias)) of the first conv block (fused with another
        predictor's on a shared input: ``ops.dual_conv_relu_layernorm``)."""
        cl = self.conv_layer
        return cl.conv1d_1.conv.weight, cl.conv1d_1.conv.bias, (cl.layer_norm_1.weight, cl.layer_norm_1.bias)

    def rest(self, h, lengths, style=None):
        """Everything after the first block: conv 2 -> ReLU -> LN -> dropout -> [FiLM] -> Linear -> mask."""
        cl = self.conv_layer
        c2 = cl.conv1d_2
        fp = self.film.pack(style) if (style is not None and hasattr(self, "film")) else None
        h = ops.conv_relu_layernorm(h, c2.conv.weight, c2.conv.bias, c2.pad, c2.dil, cl.layer_norm_2.weight,
                                    cl.layer_norm_2.bias, post_drop=self.dropout, training=self.training,
                                    film_params=fp)
        return ops.predictor_head(h, self.linear_layer.weight, self.linear_layer.bias, lengths)


def _apply_control(pred, control):
    if isinstance(control, torch.Tensor):
        control = control.to(pred.device, pred.dtype)
        if control.dim() == 2 and control.shape[1] != pred.shape[1]:
            control = F.pad(control, (0, pred.shape[1] - control.shape[1]), value=1.0)[:, : pred.shape[1]]
        return pred * control
    return pred * control if control != 1.0 else pred


class VarianceAdaptor(nn.Module):
    """Duration / pitch / energy predictors, bucketized embeddings and the
    length regulator (``model/modules.py:20-165``).  Only the duration predictor
    receives the style FiLM (``modules.py:121``; D7 preserved).  Controls may be
    scalars or per-phoneme ``[B, T]`` tensors (word-level control, the reference
    ``notebooks/control.ipynb`` cells 17-23)."""

    def __init__(self, preprocess_config, model_config, film=False):
        super().__init__()
        self.duration_predictor = VariancePredictor(model_config, film)
        self.pitch_predictor = VariancePredictor(model_config, film)
        self.energy_predictor = VariancePredictor(model_config, film)
        pp = preprocess_config["preprocessing"]
        self.pitch_feature_level = pp["pitch"]["feature"]
        self.energy_feature_level = pp["energy"]["feature"]
        ve = model_config["variance_embedding"]
        n_bins = ve["n_bins"]
        stats = _load_stats(preprocess_config)
        p_min, p_max = stats["pitch"][:2]
        e_min, e_max = stats["energy"][:2]
        self.pitch_bins = nn.Parameter(_bins(p_min, p_max, n_bins, ve["pitch_quantization"]), requires_grad=False)
        self.energy_bins = nn.Parameter(_bins(e_min, e_max, n_bins, ve["energy_quantization"]), requires_grad=False)
        d = model_config["transformer"]["encoder_hidden"]
        self.pitch_embedding = nn.Embedding(n_bins, d)
        self.energy_embedding = nn.Embedding(n_bins, d)

    def arena_groups(self):
        """Duration + pitch first convs adjacent in the flat arena (both read the encoder output x when
        pitch is phoneme-level): the fused [512, 256, k] weight of ONE GEMM is a view."""
        if self.pitch_feature_level != "phoneme_level":
            return []
        d = self.duration_predictor.conv_layer.conv1d_1.conv
        p = self.pitch_predictor.conv_layer.conv1d_1.conv
        return [[d.weight, p.weight], [d.bias, p.bias]]

    def _variance(self, predictor, bins, table, x, target, lengths, control, h1=None):
        pred = predictor(x, lengths) if h1 is None else predictor.rest(h1, lengths)
        if target is not None:
            values = target
        else:
            pred = _apply_control(pred, control)
            values = pred
        x = ops.bucketize_embed_add(x, values, bins, table.weight if ops.use_hip(x) else table.weight.to(x.dtype))
        return pred, x

    def packable(self):
        """Frame-level variance features act on the padded frame domain: no packed decoder then."""
        return self.pitch_feature_level == "phoneme_level" and self.energy_feature_level == "phoneme_level"

    def forward(self, x, src_lens, mel_lens=None, max_len=None, pitch_target=None, energy_target=None,
                duration_target=None, p_control=1.0, e_control=1.0, d_control=1.0, style=None, regulate=True):
        p_pred = e_pred = None
        if self.pitch_feature_level == "phoneme_level":
            # duration and pitch predictors read the same x: their first conv blocks run as one GEMM
            dp, pp_ = self.duration_predictor, self.pitch_predictor
            wd, bd, lnd = dp.first_block()
            wp, bp, lnp = pp_.first_block()
            c1 = dp.conv_layer.conv1d_1
            h_d, h_p = ops.dual_conv_relu_layernorm(x, (wd, wp), (bd, bp), c1.pad, c1.dil, (lnd, lnp),
                                                    post_drop=dp.dropout, training=self.training)
            log_d = dp.rest(h_d, src_lens, style)
            p_pred, x = self._variance(pp_, self.pitch_bins, self.pitch_embedding, x, pitch_target, src_lens, p_control,
                                       h1=h_p)
        else:
            log_d = self.duration_predictor(x, src_lens, style)
        if self.energy_feature_level == "phoneme_level":
            e_pred, x = self._variance(self.energy_predictor, self.energy_bins, self.energy_embedding, x, energy_target, src_lens, e_control)

        if not regulate:  # the packed decoder regulates itself (Decoder.forward_packed)
            return x, p_pred, e_pred, log_d, duration_target, mel_lens
        if duration_target is not None:
            d_rounded = duration_target
            x, mel_len = ops.length_regulate(x, duration_target, max_len)
            if mel_lens is not None:
                mel_len = mel_lens
        else:
            d_rounded, mel_len = ops.duration_round(log_d, src_lens, d_control)  # one kernel on the GPU
            x, mel_len = ops.length_regulate(x, d_rounded, None, mel_len=mel_len)

        if self.pitch_feature_level == "frame_level":
            p_pred, x = self._variance(self.pitch_predictor, self.pitch_bins, self.pitch_embedding, x, pitch_target, mel_len, p_control)
        if self.energy_feature_level == "frame_level":
            e_pred, x = self._variance(self.energy_predictor, self.energy_bins, self.energy_embedding, x, energy_target, mel_len, e_control)
        return x, p_pred, e_pred, log_d, d_rounded, mel_len


def _bins(lo, hi, n_bins, quant):
    if quant == "log":
        if not lo > 0:
            raise ValueError(
                f"log pitch/energy quantization needs positive feature stats (min={lo}); z-score normalised "
                "features (preprocessing.*.normalization: True) only work with linear quantization")
        return torch.exp(torch.linspace(math.log(lo), math.log(hi), n_bins - 1))
    return torch.linspace(lo, hi, n_bins - 1)


def _load_stats(preprocess_config):
    path = os.path.join(preprocess_config["path"]["preprocessed_path"], "stats.json")
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    # no stats.json (synthetic runs / fresh configs): a generous range in the features' own units --
    # z-scores when normalised, Hz and STFT-magnitude energy otherwise (positive: log bins work)
    pp = preprocess_config["preprocessing"]
    norm_p = pp["pitch"].get("normalization", True)
    norm_e = pp["energy"].get("normalization", True)
    return {"pitch": [-4.0, 12.0, 0.0, 1.0] if norm_p else [40.0, 900.0, 0.0, 1.0],
            "energy": [-2.0, 10.0, 0.0, 1.0] if norm_e else [0.01, 400.0, 0.0, 1.0]}


def _spker_table(preprocess_config):
    """[n_speakers, dim] fp32 table of ``spker_embed/{speaker}-spker_embed.npy`` (ordered by the
    speakers.json ids), or None when no speaker embedder is configured.  Missing files are an error."""
    emb = preprocess_config["preprocessing"].get("speaker_embedder", "none")
    if emb in (None, "none"):
        return None
    root = preprocess_config["path"]["preprocessed_path"]
    with open(os.path.join(root, "speakers.json")) as f:
        smap = json.load(f)
    import numpy as np

    rows = [None] * len(smap)
    for name, i in smap.items():
        v = np.load(os.path.join(root, "spker_embed", f"{name}-spker_embed.npy"), allow_pickle=False)
        rows[int(i)] = np.asarray(v, dtype=np.float32).reshape(-1)
    return torch.from_numpy(np.stack(rows))


def _n_speakers(preprocess_config):
    path = os.path.join(preprocess_config["path"]["preprocessed_path"], "speakers.json")
    if os.path.exists(path):
        with open(path) as f:
            return len(json.load(f))
    return int(preprocess_config.get("n_speakers", 1))


class FastSpeech2(nn.Module):
    def __init__(self, preprocess_config, model_config):
        super().__init__()
        self.model_config = model_config
        self.style = style_mode(model_config)
        film = self.style != "none"
        self.encoder = Encoder(model_config, film=film)
        if self.style == "film":
            self.reference_encoder = ReferenceEncoder(preprocess_config, model_config)
        elif self.style == "gst":
            self.gst = GlobalStyleTokens(preprocess_config, model_config)
        self.variance_adaptor = VarianceAdaptor(preprocess_config, model_config, film=film)
        self.decoder = Decoder(model_config, film=film)
        n_mel = preprocess_config["preprocessing"]["mel"]["n_mel_channels"]
        self.mel_linear = nn.Linear(model_config["transformer"]["decoder_hidden"], n_mel)
        self.postnet = PostNet(n_mel)
        self.speaker_emb = None
        d = model_config["transformer"]["encoder_hidden"]
        if model_config["multi_speaker"]:
            self.speaker_emb = nn.Embedding(_n_speakers(preprocess_config), d)
        # external speaker embeddings (reference ``synthesize.py:268-277``: ``{spk}-spker_embed.npy`` under
        # ``preprocessed_path/spker_embed`` when ``preprocessing.speaker_embedder != 'none'``).  The
        # reference loads them and drops them, and so does this model unless ``speaker_embed_proj: true``
        # is set in model.yaml (opt-in: it adds a trainable projection the reference checkpoints lack).
        # With it, a per-speaker table (non-persistent buffer, looked up by speaker id in training and
        # synthesis alike) is projected to the encoder width and added next to the speaker-id embedding.
        use_table = model_config["multi_speaker"] and bool(model_config.get("speaker_embed_proj", False))
        table = _spker_table(preprocess_config) if use_table else None
        self.spker_embed_proj = None
        if table is not None:
            self.register_buffer("spker_table", table, persistent=False)
            self.spker_embed_proj = nn.Linear(table.shape[1], d)
        self.compute_dtype = torch.float32

    # ------------------------------------------------------------------ helpers
    def set_compute_dtype(self, dtype):
        self.compute_dtype = dtype
        return self

    def fused_param_groups(self):
        return fused_param_groups(self)

    def style_encoder(self):
        return getattr(self, "reference_encoder", None) or getattr(self, "gst", None)

    def film_scalars(self):
        """Stacked s_gamma/s_beta parameters (reference ``utils/model.py:53-59``).  The parameter
        list is collected once (named_parameters() walks the whole module tree every call)."""
        ps = self._film_param_list()
        if not ps:
            return None
        if ops.use_hip(ps[0]):
            from ..ops import hip

            return hip.film_scalars_cat(ps)  # L2 gradient folded into the sites' FiLM kernels
        return torch.cat(ps)

    def _film_param_list(self):
        ps = self.__dict__.get("_film_ps")
        if ps is None:
            ps = [p for n, p in self.named_parameters() if ("s_gamma" in n or "s_beta" in n)]
            self.__dict__["_film_ps"] = ps
        return ps

    def compute_style(self, mels, mel_lens, max_mel_len, batch, device, style_weights=None):
        enc = self.style_encoder()
        if enc is None:
            return None
        if style_weights is not None and self.style == "gst":
            g, b = self.gst.from_token_weights(style_weights.to(device))
        elif mels is None:
            d = self.model_config["transformer"]["encoder_hidden"]
            z = torch.zeros(batch, d, device=device, dtype=self.compute_dtype)
            return (z, z)
        else:
            g, b = enc(mels.to(self.compute_dtype), mel_lens, max_mel_len)
        g, b = g.to(self.compute_dtype), b.to(self.compute_dtype)
        if ops.use_hip(g):  # fresh per forward, read only by FiLM LayerNorm sites: one shared gradient buffer (_FilmAcc)
            g._ssamd_film_acc = b._ssamd_film_acc = True
        return (g, b)

    # ------------------------------------------------------------------ forward
    def forward(self, speakers, texts, src_lens, max_src_len, mels=None, mel_lens=None, max_mel_len=None,
                p_targets=None, e_targets=None, d_targets=None, p_control=1.0, e_control=1.0, d_control=1.0,
                style_weights=None, mel_lens_host=None):
        """Reference ``model/fastspeech2.py:45-113``.  ``mel_lens_host`` (host int array of the
        batch's mel lengths, provided by the data pipeline) enables the packed decoder in training."""
        dev = texts.device
        cd = self.compute_dtype
        if torch.is_grad_enabled() and ops.use_hip(texts):
            ps = self._film_param_list()
            if ps:  # the FiLM-L2 holder exists before the sites' forward (same hook pattern every step)
                from ..ops import gradslots

                gradslots.film_holder_for(ps)
        if mel_lens_host is None and mel_lens is not None:
            mel_lens_host = getattr(mel_lens, "host_lengths", None)
        if mels is not None and max_mel_len is None:
            max_mel_len = mels.shape[1]
        style = self.compute_style(mels, mel_lens, max_mel_len, texts.shape[0], dev, style_weights)
        x = self.encoder(texts, src_lens, style, cd)
        if self.speaker_emb is not None:
            if self.spker_embed_proj is None:  # table lookup fused into the add (one HIP kernel each way)
                x = ops.add_table_rows(x, self.speaker_emb.weight, speakers)
            else:
                spk = self.speaker_emb(speakers) + self.spker_embed_proj(self.spker_table[speakers])
                x = ops.add_rowvec(x, spk)
        training_lr = d_targets is not None
        packed = (self.training and training_lr and mel_lens is not None and mel_lens_host is not None
                  and max_mel_len is not None and self.variance_adaptor.packable())
        x, p_pred, e_pred, log_d, d_rounded, mel_lens_out = self.variance_adaptor(
            x, src_lens, mel_lens, max_mel_len if training_lr else None, p_targets, e_targets, d_targets,
            p_control, e_control, d_control, style, regulate=not packed,
        )
        if packed:
            M = min(int(max_mel_len), self.decoder.max_seq_len)
            R = int(sum(min(int(v), M) for v in mel_lens_host))
            x, dec_lens, pk = self.decoder.forward_packed(x, d_targets, mel_lens, int(max_mel_len), R, style)
            mel = ops.linear(x, self.mel_linear.weight, self.mel_linear.bias).float()
            # padded frames: decoder output 0 -> mel_linear gives the bias there (reference semantics)
            mel = ops.unpack_rows(mel, pk, fill=self.mel_linear.bias)
        else:
            x, dec_lens = self.decoder(x, mel_lens_out, style)
            mel = ops.linear(x, self.mel_linear.weight, self.mel_linear.bias).float()
        post = self.postnet(mel.to(cd)).float() + mel
        src_masks = ops.lengths_to_mask(src_lens, texts.shape[1])
        mel_masks = ops.lengths_to_mask(dec_lens, mel.shape[1])
        return (mel, post, p_pred, e_pred, log_d, d_rounded, src_masks, mel_masks, src_lens, mel_lens_out)

    def packed_inference_ok(self, texts) -> bool:
        return (not self.training and ops.use_hip(texts) and self.variance_adaptor.packable()
                and self.compute_dtype == torch.bfloat16)

    @torch.no_grad()
    def infer_packed(self, speakers, texts, src_lens, max_src_len, mels=None, mel_lens=None, max_mel_len=None,
                     p_control=1.0, e_control=1.0, d_control=1.0, style_weights=None):
        """Synthesis with predicted durations, the length-regulated half on PACKED rows: the decoder, mel_linear
        and the PostNet run on the R = sum(mel lengths) valid frames only (``Decoder.forward_packed``,
        ``PostNet.forward_packed``) instead of B x max(mel length) padded rows -- at batch 256 of LJSpeech-like
        lengths ~45 % of the padded rows.  Each utterance's frames are exactly its batch-1 synthesis (every conv
        zero-pads at its own ends; the padded reference path lets the padded frames' mel_linear bias leak into the
        last PostNet frames of shorter utterances).  The one host sync is the same as the padded path's (the mel
        lengths, which size the length regulator): here all B lengths come back at once.
        Returns (post-net mel [R, n_mel] fp32 rows of utterance b at cu[b].., host lengths (list), device mel_len)."""
        front = self.infer_front(speakers, texts, src_lens, max_src_len, mels, mel_lens, max_mel_len, p_control,
                                 e_control, d_control, style_weights)
        lens = [int(v) for v in front[2].cpu().tolist()]  # the one D2H: sizes the packed decoder
        return self.infer_back(front, lens), lens, front[2]

    @torch.no_grad()
    def infer_front(self, speakers, texts, src_lens, max_src_len, mels=None, mel_lens=None, max_mel_len=None,
                    p_control=1.0, e_control=1.0, d_control=1.0, style_weights=None):
        """``infer_packed`` up to the durations (no host sync, fixed shapes: HIP-graph capturable,
        ``infer/graphs.py``) -> (x [B, T, d], rounded durations [B, T], mel_len [B], style)."""
        cd = self.compute_dtype
        dev = texts.device
        if mels is not None and max_mel_len is None:
            max_mel_len = mels.shape[1]
        style = self.compute_style(mels, mel_lens, max_mel_len, texts.shape[0], dev, style_weights)
        x = self.encoder(texts, src_lens, style, cd)
        if self.speaker_emb is not None:
            if self.spker_embed_proj is None:
                x = ops.add_table_rows(x, self.speaker_emb.weight, speakers)
            else:
                spk = self.speaker_emb(speakers) + self.spker_embed_proj(self.spker_table[speakers])
                x = ops.add_rowvec(x, spk)
        x, _, _, log_d, _, _ = self.variance_adaptor(x, src_lens, None, None, None, None, None, p_control,
                                                     e_control, d_control, style, regulate=False)
        d_rounded, mel_len = ops.duration_round(log_d, src_lens, d_control)
        return x, d_rounded, mel_len, style

    @torch.no_grad()
    def infer_back(self, front, lens):
        """``infer_packed`` after the durations, for host mel lengths ``lens`` (fixed shapes given lens:
        capturable) -> post-net mel rows [R, n_mel] fp32."""
        x, d_rounded, mel_len, style = front
        M, R = max(lens) if lens else 0, sum(lens)
        x, dec_lens, pk = self.decoder.forward_packed(x, d_rounded, mel_len, M, R, style)
        mel = ops.linear(x, self.mel_linear.weight, self.mel_linear.bias).float()
        post = self.postnet.forward_packed(mel.to(self.compute_dtype), pk).float() + mel
        return post.reshape(R, -1)
