"""HiFi-GAN training on the HIP kernels (``csrc/k_disc.hip``).

Reference: ``hifigan/models.py:176-264`` (MultiPeriodDiscriminator / MultiScaleDiscriminator, feature /
LSGAN losses), ``hifigan/meldataset.py:49-72`` (mel_spectrogram), ``hifigan/train.py:113-160`` (the D and G
steps).  The torch modules of ``models/hifigan.py`` keep the parameters (weight-norm / spectral-norm
parametrisations, state-dict keys); this module runs them channel-last on the GPU:

* every discriminator layer is ONE ``sconv`` launch (strided / grouped / dilated implicit-GEMM conv with the
  LeakyReLU in its epilogue) on ``[rows, T, C]`` bf16 activations.  DiscriminatorP's (k, 1) Conv2d over
  ``[B, C, T/p, p]`` is a conv1d over T/p for each of the p columns: the waveform is reflect-padded and
  folded once into ``[B*p, T/p, 1]`` sequences (``mpd_fold``) and every later layer is a plain sconv;
* the real and generated waveforms go through each discriminator as ONE batch ``[y; y_hat]`` (the
  reference calls the discriminator twice): one launch per layer, and in the D step the weight gradient of
  the real and fake halves is one reduction;
* ``d_step`` (D step): LSGAN loss + backward to the discriminator weights only -- the data gradient
  of the first layer (the waveform) is skipped, the generator output is detached;
* ``g_adv`` (G step): LSGAN + feature-matching loss of the fake half + backward to the generated
  waveform only: no discriminator weight gradients (the reference's ``loss_gen_all.backward()`` computes
  them and ``optim_d.zero_grad()`` discards them before they are used), the real half runs without
  autograd.  The feature-matching gradient 2 sign(g - r) / n is fused into the LeakyReLU backward of its
  layer (``act_bwd``);
* ``mel_l1``: the STFT is an sconv of the reflect-padded waveform with the windowed DFT basis as
  weights (stride = hop), fp32-accurate through a bf16 hi / lo split of the waveform and the basis; one
  kernel per frame does |X|, the mel projection, log-clamp, L1 and the whole gradient d loss / d(re, im);
  the backward is the polyphase data gradient of the DFT conv (4 taps per sample) + the reflect-pad fold.
* generator glue (``lrelu``, ``add``, ``mean3``, ``conv_post_tanh``): autograd Functions on HIP kernels.

Documented deviations: spectral_norm's power iteration runs twice per discriminator call as in the
reference (it calls ``d(y)`` and ``d(y_hat)``), but both halves of the joint batch use the second
iterate's weight (the reference uses the first for ``y``); scores are fp32, activations bf16.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

from ..ops import hip

LRELU = 0.1
_P = hip._ptr


def _lib():
    return hip.lib()


def _s():
    return hip._stream()


def _chk(rc, name):
    hip._check(rc, name)


# ------------------------------------------------------------------------------------------- weight images
def fwd_image(w: torch.Tensor, G: int = 1) -> torch.Tensor:
    """[Cout, Cg, ks] -> bf16 [Cout, Kp]: row o = W[o, c, j] at column j * Cg + c (Kp = round8(ks * Cg))."""
    Cout, Cg, ks = w.shape[:3]
    Kp = (ks * Cg + 7) // 8 * 8
    if w.is_cuda:
        wf = w.detach().float().contiguous()
        img = torch.empty(Cout, Kp, device=w.device, dtype=torch.bfloat16)
        _chk(_lib().ssamd_sconv_images(_P(wf), _P(img), None, Cout, Cg * G, G, ks, 1, _s()), "ssamd_sconv_images")
        return img
    img = w.detach().float().reshape(Cout, Cg, ks).permute(0, 2, 1).reshape(Cout, ks * Cg)
    return F.pad(img, (0, Kp - ks * Cg)).to(torch.bfloat16).contiguous()


def dgrad_image(w: torch.Tensor, G: int, s: int) -> torch.Tensor:
    """[Cout, Cg, ks] -> bf16 [G*Cg, s, UNp]: row g*Cg + c, residue r, column u*Ng + n = W[g*Ng + n, c, r + s*u]."""
    Cout, Cg, ks = w.shape[:3]
    Ng = Cout // G
    U = -(-ks // s)
    UNp = (U * Ng + 7) // 8 * 8
    if w.is_cuda:
        wf = w.detach().float().contiguous()
        img = torch.empty(G * Cg, s, UNp, device=w.device, dtype=torch.bfloat16)
        _chk(_lib().ssamd_sconv_images(_P(wf), None, _P(img), Cout, Cg * G, G, ks, s, _s()), "ssamd_sconv_images")
        return img
    wp = F.pad(w.detach().float().reshape(Cout, Cg, ks), (0, U * s - ks)).view(G, Ng, Cg, U, s)
    img = wp.permute(0, 2, 4, 3, 1).reshape(G * Cg, s, U * Ng)
    return F.pad(img, (0, UNp - U * Ng)).to(torch.bfloat16).contiguous()


# ------------------------------------------------------------------------------------------- raw launches
def sconv_out_len(Tin, ks, s, d, p) -> int:
    return int(_lib().ssamd_sconv_tout(Tin, ks, s, d, p))


def sconv_fwd(x, wimg, bias, G, ks, s, d, p, act=0, slope=LRELU, out_f32=False):
    """x [B, Tin, Cin] bf16 -> [B, Tout, Cout]; act 0 none, 1 lrelu(slope), 2 tanh."""
    hip._need(x, torch.bfloat16, "sconv.x")
    B, Tin, Cin = x.shape
    Cout = wimg.shape[0]
    assert wimg.shape[1] == (ks * (Cin // G) + 7) // 8 * 8, "sconv: weight image / geometry mismatch"
    Tout = sconv_out_len(Tin, ks, s, d, p)
    assert Tout > 0, "sconv: empty output"
    y = torch.empty(B, Tout, Cout, device=x.device, dtype=torch.float32 if out_f32 else torch.bfloat16)
    bf = None if bias is None else bias.detach().float().contiguous()
    _chk(_lib().ssamd_sconv_fwd(_P(x), _P(wimg), _P(bf), _P(y), B, Tin, Cin, Cout, G, ks, s, d, p, int(act),
                                float(slope), int(out_f32), _s()), "ssamd_sconv_fwd")
    return y


def sconv_dgrad(dz, wdimg, Tin, Cin, G, ks, s, d, p, out_f32=False, out=None):
    """dz [B, Tout, Cout] bf16 -> dx [B, Tin, Cin] (``out``: fp32 buffer accumulated into)."""
    hip._need(dz, torch.bfloat16, "sconv_dgrad.dz")
    B, Tout, Cout = dz.shape
    assert Tout == sconv_out_len(Tin, ks, s, d, p), "sconv_dgrad: dz length"
    assert wdimg.shape[0] == Cin and wdimg.shape[1] == s, "sconv_dgrad: weight image"
    accum = out is not None
    if out is None:
        out = torch.empty(B, Tin, Cin, device=dz.device, dtype=torch.float32 if out_f32 else torch.bfloat16)
    else:
        hip._need(out, torch.float32, "sconv_dgrad.out")
        assert out.numel() == B * Tin * Cin
        out_f32 = True
    _chk(_lib().ssamd_sconv_dgrad(_P(dz), _P(wdimg), _P(out), B, Tin, Cin, Cout, G, ks, s, d, p, int(out_f32),
                                  int(accum), _s()), "ssamd_sconv_dgrad")
    return out


def sconv_wgrad(dz, x, G, ks, s, d, p, with_bias=False):
    """-> dW fp32 [Cout, Cin/G, ks] (torch layout) [, db fp32 [Cout] = column sums of dz]."""
    hip._need(dz, torch.bfloat16, "sconv_wgrad.dz")
    hip._need(x, torch.bfloat16, "sconv_wgrad.x")
    B, Tin, Cin = x.shape
    Cout = dz.shape[-1]
    assert dz.shape[0] == B and dz.shape[1] == sconv_out_len(Tin, ks, s, d, p)
    n_ws = int(_lib().ssamd_sconv_wgrad_ws(B, Tin, Cin, Cout, G, ks, s, d, p))
    ws = hip._workspace(x.device, n_ws)
    dW = torch.empty(Cout, Cin // G, ks, device=x.device, dtype=torch.float32)
    db = torch.empty(Cout, device=x.device, dtype=torch.float32) if with_bias else None
    _chk(_lib().ssamd_sconv_wgrad(_P(dz), _P(x), _P(ws), ws.numel(), _P(dW), _P(db), B, Tin, Cin, Cout, G, ks, s, d, p,
                                  _s()), "ssamd_sconv_wgrad")
    return (dW, db) if with_bias else dW


def act_bwd(dy, y, act=1, slope=LRELU, r=None, fm_scale=0.0, out=None):
    """((dy or 0) + fm_scale * sign(y - r)) * act'(y), bf16."""
    hip._need(y, torch.bfloat16, "act_bwd.y")
    out = torch.empty_like(y) if out is None else out
    _chk(_lib().ssamd_act_bwd(_P(dy), _P(y), _P(r), float(fm_scale), _P(out), y.numel(), int(act), float(slope), _s()),
         "ssamd_act_bwd")
    return out


def _ew(op, a, b=None, c=None, s=0.0, out=None):
    hip._need(a, torch.bfloat16, "ew.a")
    out = torch.empty_like(a) if out is None else out
    _chk(_lib().ssamd_ew(op, _P(a), _P(b), _P(c), _P(out), a.numel(), float(s), _s()), "ssamd_ew")
    return out


def l1_sum_into(loss, a, b, scale, part):
    """loss[0] += scale * sum |a - b|."""
    f32 = a.dtype == torch.float32
    _chk(_lib().ssamd_l1_sum(_P(a), _P(b), a.numel(), int(f32), float(scale), _P(part), _P(loss), 1, _s()),
         "ssamd_l1_sum")


def lsgan_into(loss, s, target, gscale=1.0, ds=None, r=None, fm_scale=0.0):
    """loss[0] += mean((target - s)^2) [+ fm_scale * sum |s - r|]; ds = d/ds * gscale (bf16) when given.
    s (and r) fp32 contiguous."""
    if r is not None:
        assert r.dtype == torch.float32 and r.is_contiguous() and r.numel() == s.numel(), "lsgan_into: r"
    _chk(_lib().ssamd_lsgan(_P(s), s.numel(), float(target), float(gscale), _P(r), float(fm_scale), _P(ds), _P(loss),
                            _s()), "ssamd_lsgan")


def avgpool4(x):
    """AvgPool1d(4, 2, padding=2) over rows of x [R, T] (bf16)."""
    R, T = x.shape
    y = torch.empty(R, T // 2 + 1, device=x.device, dtype=torch.bfloat16)
    _chk(_lib().ssamd_avgpool4(_P(x), _P(y), R, T, _s()), "ssamd_avgpool4")
    return y


def avgpool4_bwd_into(dx, dy, T):
    R = dx.shape[0]
    _chk(_lib().ssamd_avgpool4_bwd(_P(dy), _P(dx), R, T, 1, _s()), "ssamd_avgpool4_bwd")


# ------------------------------------------------------------------------------------------- discriminators
def _refresh(conv, times=1):
    """Run the module's forward pre-hooks (weight_norm / spectral_norm recompute ``conv.weight``)."""
    for _ in range(times):
        for h in conv._forward_pre_hooks.values():
            h(conv, None)


def _layer_geom(conv):
    w = conv.weight
    if w.dim() == 4:  # Conv2d (k, 1) of DiscriminatorP
        return dict(w=w.squeeze(-1), b=conv.bias, ks=conv.kernel_size[0], s=conv.stride[0], d=conv.dilation[0],
                    p=conv.padding[0], G=conv.groups)
    return dict(w=w, b=conv.bias, ks=conv.kernel_size[0], s=conv.stride[0], d=conv.dilation[0], p=conv.padding[0],
                G=conv.groups)


class _Disc:
    """One discriminator's layers with their bf16 images (rebuilt per call: the weights change every step)."""

    def __init__(self, d, hook_times=1):
        self.module = d
        for c in list(d.convs) + [d.conv_post]:
            _refresh(c, hook_times)
        self.layers = [_layer_geom(c) for c in d.convs]
        self.post = _layer_geom(d.conv_post)
        for L in self.layers + [self.post]:
            L["img"] = fwd_image(L["w"], L["G"])
        self.period = getattr(d, "period", None)

    def dimg(self, L):
        if "dimg" not in L:
            L["dimg"] = dgrad_image(L["w"], L["G"], L["s"])
        return L["dimg"]

    def prep(self, u):
        """u [R, T] bf16 waveform rows -> x0 [R', T', 1]."""
        if self.period is None:
            return u.unsqueeze(-1)
        R, T = u.shape
        p = self.period
        H = -(-T // p)
        out = torch.empty(R * p, H, 1, device=u.device, dtype=torch.bfloat16)
        _chk(_lib().ssamd_mpd_fold(_P(u), _P(out), R, T, p, _s()), "ssamd_mpd_fold")
        return out

    def forward(self, x0):
        """-> (inputs of every layer incl. conv_post, fmaps (post-lrelu), fp32 scores [R', T', 1])."""
        xs, x = [], x0
        for L in self.layers:
            xs.append(x)
            x = sconv_fwd(x, L["img"], L["b"], L["G"], L["ks"], L["s"], L["d"], L["p"], act=1)
        xs.append(x)
        P = self.post
        score = sconv_fwd(x, P["img"], P["b"], P["G"], P["ks"], P["s"], P["d"], P["p"], act=0, out_f32=True)
        return xs, xs[1:], score


def _half(t):
    n = t.shape[0] // 2
    return t[:n], t[n:]


def _has_sn(d):
    return any(type(h).__name__ == "SpectralNorm" for h in d.convs[0]._forward_pre_hooks.values())


def _disc_d(d, u, loss, ws, gs):
    """D step of one discriminator on the joint rows u = [y; y_hat] (bf16 [2B, T]): loss[0] += mean((1 - D(y))^2)
    + mean(D(y_hat)^2); appends (effective weight, dW) / (bias, db) pairs -- no data gradient of the input."""
    disc = _Disc(d, hook_times=2 if _has_sn(d) else 1)
    xs, _, score = disc.forward(disc.prep(u))
    ds = torch.empty(score.shape, device=u.device, dtype=torch.bfloat16)
    sr, sg = _half(score)
    dr, dg = _half(ds)
    lsgan_into(loss, sr, 1.0, 1.0, dr)
    lsgan_into(loss, sg, 0.0, 1.0, dg)
    convs = list(d.convs) + [d.conv_post]
    layers = disc.layers + [disc.post]
    dz = ds
    for li in range(len(layers) - 1, -1, -1):
        L = layers[li]
        if li < len(layers) - 1:
            dz = act_bwd(dx, xs[li + 1], 1, LRELU)
        x_in = xs[li]
        has_b = convs[li].bias is not None
        dW, db = sconv_wgrad(dz, x_in, L["G"], L["ks"], L["s"], L["d"], L["p"], with_bias=True)
        w_eff = convs[li].weight
        ws.append(w_eff)
        gs.append(dW.view(w_eff.shape).to(w_eff.dtype))
        if has_b:
            ws.append(convs[li].bias)
            gs.append(db.to(convs[li].bias.dtype))
        if li > 0:
            dx = sconv_dgrad(dz, disc.dimg(L), x_in.shape[1], x_in.shape[2], L["G"], L["ks"], L["s"], L["d"], L["p"])


def d_step(mpd, msd, y, y_hat):
    """Discriminator loss (reference ``discriminator_loss`` over MPD + MSD, ``train.py:113-127``) and its gradient,
    accumulated into the discriminators' parameters (through their weight_norm / spectral_norm parametrisations).
    y, y_hat: [B, T] waveforms (y_hat detached).  Returns the loss as a device tensor [1]."""
    u = torch.cat([y.detach(), y_hat.detach()], 0).to(torch.bfloat16).contiguous()
    loss = torch.zeros(1, device=u.device, dtype=torch.float32)
    ws, gs = [], []
    for d in mpd.discriminators:
        _disc_d(d, u, loss, ws, gs)
    for i, d in enumerate(msd.discriminators):
        if i:
            u = avgpool4(u)
        _disc_d(d, u, loss, ws, gs)
    torch.autograd.backward(ws, gs)
    return loss


def _disc_g(d, u, loss, part, out0=None):
    """G step of one discriminator on u = [y; y_hat]: loss[0] += mean((1 - D(y_hat))^2) + 2 sum_l mean|fmap_l(y_hat)
    - fmap_l(y)| over every feature map -- the post-lrelu conv outputs AND the conv_post score map (the reference
    ``DiscriminatorP/S.forward`` appends the score to ``fmap``, hifigan/models.py:193-198); returns d loss / d (fake
    half of the layer-0 input), fp32 [B*, T*, 1]."""
    disc = _Disc(d, hook_times=2 if _has_sn(d) else 1)
    xs, fmaps, score = disc.forward(disc.prep(u))
    sr, sg = _half(score)
    ds = torch.empty(sg.shape, device=u.device, dtype=torch.bfloat16)
    # adversarial term + the score map's feature-matching term 2 * mean|D(y_hat) - D(y)| in one kernel
    lsgan_into(loss, sg, 1.0, 1.0, ds, r=sr, fm_scale=2.0 / sg.numel())
    fm = []
    for f in fmaps:
        fr, fg = _half(f)
        sc = 2.0 / fg.numel()
        l1_sum_into(loss, fg, fr, sc, part)
        fm.append(sc)
    layers = disc.layers + [disc.post]
    dz = ds
    dx = None
    for li in range(len(layers) - 1, -1, -1):
        L = layers[li]
        if li < len(layers) - 1:
            yr, yg = _half(xs[li + 1])
            dz = act_bwd(dx, yg, 1, LRELU, r=yr, fm_scale=fm[li])
        x_in = _half(xs[li])[1]
        dx = sconv_dgrad(dz, disc.dimg(L), x_in.shape[1], x_in.shape[2], L["G"], L["ks"], L["s"], L["d"], L["p"],
                         out_f32=li == 0, out=out0 if li == 0 else None)
    return disc, dx


def g_adv(mpd, msd, y, y_hat, dy):
    """Generator adversarial + feature-matching loss (reference ``generator_loss`` + ``feature_loss`` over MPD and
    MSD, ``train.py:137-146``); adds its gradient w.r.t. y_hat into dy (fp32 [B, T]).  Returns the loss [1]."""
    B, T = y_hat.shape
    u = torch.cat([y.detach(), y_hat.detach()], 0).to(torch.bfloat16).contiguous()
    loss = torch.zeros(1, device=u.device, dtype=torch.float32)
    part = torch.empty(256, device=u.device, dtype=torch.float32)
    for d in mpd.discriminators:
        disc, dx = _disc_g(d, u, loss, part)
        _chk(_lib().ssamd_mpd_unfold(_P(dx), _P(dy), B, T, disc.period, _s()), "ssamd_mpd_unfold")
    # MSD: discriminator i sees the waveform pooled i times; its input gradient goes back through the pools
    # (deepest first) into dy -- every step accumulates in a kernel
    us = [u]
    for i in range(1, len(msd.discriminators)):
        us.append(avgpool4(us[-1]))
    outs = [dy] + [torch.zeros(B, ui.shape[1], device=u.device, dtype=torch.float32) for ui in us[1:]]
    for i, d in enumerate(msd.discriminators):
        _disc_g(d, us[i], loss, part, out0=outs[i])
    for i in range(len(outs) - 1, 0, -1):
        avgpool4_bwd_into(outs[i - 1], outs[i], us[i - 1].shape[1])
    return loss


# ------------------------------------------------------------------------------------------- mel loss
_DFT: Dict[Tuple, Tuple[torch.Tensor, torch.Tensor]] = {}


def _dft_images(n_fft, win, device):
    """(forward image bf16 [Cpad, n_fft * 8] for the hi / lo split input, data-gradient image) of the windowed
    one-sided DFT: rows k < NB = n_fft/2 + 1: w[j] cos(2 pi k j / n_fft); rows NB + k: -w[j] sin(...)."""
    key = (n_fft, win, str(device))
    hit = _DFT.get(key)
    if hit is not None:
        return hit
    NB = n_fft // 2 + 1
    Cp = (2 * NB + 7) // 8 * 8
    j = torch.arange(n_fft, dtype=torch.float64)
    k = torch.arange(NB, dtype=torch.float64)
    window = torch.hann_window(win, dtype=torch.float64)
    if win < n_fft:
        lp = (n_fft - win) // 2
        window = F.pad(window, (lp, n_fft - win - lp))
    ang = 2 * math.pi * torch.outer(k, j) / n_fft
    W = torch.zeros(Cp, n_fft, dtype=torch.float64)
    W[:NB] = window * torch.cos(ang)
    W[NB:2 * NB] = -window * torch.sin(ang)
    W = W.float()
    hi = W.to(torch.bfloat16)
    lo = (W - hi.float()).to(torch.bfloat16)
    img = torch.zeros(Cp, n_fft, 8, dtype=torch.bfloat16)
    img[:, :, 0] = hi
    img[:, :, 1] = hi
    img[:, :, 2] = lo
    fimg = img.reshape(Cp, n_fft * 8).contiguous().to(device)
    hit = (fimg, W.to(device))
    _DFT[key] = hit
    return hit


_DIMG: Dict[Tuple, torch.Tensor] = {}


def _dft_dgrad_image(n_fft, win, hop, device):
    key = (n_fft, win, hop, str(device))
    hit = _DIMG.get(key)
    if hit is None:
        _, W = _dft_images(n_fft, win, device)
        hit = _DIMG[key] = dgrad_image(W.view(W.shape[0], 1, n_fft), 1, hop)
    return hit


_BASIS: Dict[Tuple, torch.Tensor] = {}


def _basis(sr, n_fft, n_mels, fmin, fmax, device):
    from ..audio.mel import mel_filterbank

    key = (sr, n_fft, n_mels, fmin, fmax, str(device))
    hit = _BASIS.get(key)
    if hit is None:
        hit = _BASIS[key] = torch.from_numpy(mel_filterbank(sr, n_fft, n_mels, fmin, fmax)).float().contiguous().to(device)
    return hit


def mel_l1(h, y_hat, y_mel, weight, dy):
    """weight * mean |log-mel(y_hat) - y_mel| (reference ``train.py:135`` with ``meldataset.mel_spectrogram``) on
    the HIP STFT / mel kernels, frames trimmed to the shorter of the two; adds its gradient w.r.t. y_hat into dy
    (fp32 [B, T]).  y_hat [B, T], y_mel [B, n_mels, F].  Returns the loss [1]."""
    dev = y_hat.device
    y = y_hat.detach().float().contiguous()
    R, N = y.shape
    n_fft, hop, win = int(h.n_fft), int(h.hop_size), int(h.win_size)
    Pd = (n_fft - hop) // 2
    fimg, _ = _dft_images(n_fft, win, dev)
    Cp = fimg.shape[0]
    xp = torch.empty(R, N + 2 * Pd, 8, device=dev, dtype=torch.bfloat16)
    _chk(_lib().ssamd_stft_prep(_P(y), _P(xp), R, N, Pd, _s()), "ssamd_stft_prep")
    spec = sconv_fwd(xp, fimg, None, 1, n_fft, hop, 1, 0, act=0, out_f32=True)  # [R, Fr, Cp]
    Fr = spec.shape[1]
    NB = n_fft // 2 + 1
    basis = _basis(h.sampling_rate, n_fft, h.num_mels, h.fmin, h.get("fmax_for_loss"), dev)
    tgt = y_mel.float().contiguous()
    Ft = tgt.shape[-1]
    Fv = min(Fr, Ft)
    scale = float(weight) / (R * h.num_mels * Fv)
    part = torch.empty(R * Fr, device=dev, dtype=torch.float32)
    dspec = torch.empty(R, Fr, Cp, device=dev, dtype=torch.bfloat16)
    _chk(_lib().ssamd_mel_l1(_P(spec), Cp, _P(basis), NB, h.num_mels, _P(tgt), Ft, R, Fr, Fv, scale, _P(part),
                             _P(dspec), Cp, _s()), "ssamd_mel_l1")
    loss = torch.zeros(1, device=dev, dtype=torch.float32)
    _chk(_lib().ssamd_sum_parts(_P(part), R * Fr, scale, _P(loss), 0, _s()), "ssamd_sum_parts")
    dimg = _dft_dgrad_image(n_fft, win, hop, dev)
    dxp = sconv_dgrad(dspec, dimg, N + 2 * Pd, 1, 1, n_fft, hop, 1, 0, out_f32=True)  # [R, N + 2Pd, 1]
    _chk(_lib().ssamd_stft_unpad(_P(dxp), _P(dy), R, N, Pd, 1, _s()), "ssamd_stft_unpad")
    return loss


def mel_hip(h, y, loss=True):
    """log-mel [B, n_mels, F] of y [B, N] on the HIP STFT (forward only; validation / logging)."""
    dev = y.device
    y = y.float().contiguous()
    R, N = y.shape
    n_fft, hop, win = int(h.n_fft), int(h.hop_size), int(h.win_size)
    Pd = (n_fft - hop) // 2
    fimg, _ = _dft_images(n_fft, win, dev)
    xp = torch.empty(R, N + 2 * Pd, 8, device=dev, dtype=torch.bfloat16)
    _chk(_lib().ssamd_stft_prep(_P(y), _P(xp), R, N, Pd, _s()), "ssamd_stft_prep")
    spec = sconv_fwd(xp, fimg, None, 1, n_fft, hop, 1, 0, act=0, out_f32=True)
    NB = n_fft // 2 + 1
    mag = torch.sqrt(spec[..., :NB] ** 2 + spec[..., NB:2 * NB] ** 2 + 1e-9)
    basis = _basis(h.sampling_rate, n_fft, h.num_mels, h.fmin, h.get("fmax_for_loss") if loss else h.fmax, dev)
    return torch.log(torch.clamp(mag @ basis.t(), min=1e-5)).transpose(1, 2)


# ------------------------------------------------------------------------------------------- generator glue
class _LReLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, slope):
        xc = x.contiguous()
        ctx.slope = slope
        ctx.save_for_backward(xc)
        return _ew(0, xc, s=slope)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return _ew(4, dy.to(torch.bfloat16).contiguous(), x, s=ctx.slope), None


class _AddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        return _ew(1, a.contiguous(), b.contiguous())

    @staticmethod
    def backward(ctx, dy):
        return dy, dy


class _Mean3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, c):
        return _ew(2, a.contiguous(), b.contiguous(), c.contiguous(), s=1.0 / 3.0)

    @staticmethod
    def backward(ctx, dy):
        g = _ew(3, dy.to(torch.bfloat16).contiguous(), s=1.0 / 3.0)
        return g, g, g


class _ConvPostTanhFn(torch.autograd.Function):
    """tanh(conv1d(a, w, b)) with Cout = 1 (the generator's conv_post; a = lrelu(x, 0.01) bf16 [B, T, C])
    -> fp32 [B, T, 1]."""

    @staticmethod
    def forward(ctx, a, w, b, pad):
        ks = w.shape[-1]
        img = fwd_image(w.float())
        y = sconv_fwd(a, img, b, 1, ks, 1, 1, pad, act=2, out_f32=True)
        ctx.save_for_backward(a, w, y)
        ctx.pad = pad
        return y

    @staticmethod
    def backward(ctx, dy):
        a, w, y = ctx.saved_tensors
        ks = w.shape[-1]
        dyc = dy.float().contiguous()
        dz = torch.empty(y.shape, device=y.device, dtype=torch.bfloat16)
        _chk(_lib().ssamd_tanh_bwd_f32(_P(dyc), _P(y), _P(dz), y.numel(), _s()), "ssamd_tanh_bwd_f32")
        da = sconv_dgrad(dz, dgrad_image(w.float(), 1, 1), a.shape[1], a.shape[2], 1, ks, 1, 1, ctx.pad)
        dW, db = sconv_wgrad(dz, a, 1, ks, 1, 1, ctx.pad, with_bias=True)
        return da, dW.view_as(w).to(w.dtype), db.to(w.dtype), None


def lrelu(x, slope=LRELU):
    return _LReLUFn.apply(x, slope)


def add(a, b):
    return _AddFn.apply(a, b)


def mean3(a, b, c):
    return _Mean3Fn.apply(a, b, c)


def conv_post_tanh(x, w, b, pad, slope=0.01):
    return _ConvPostTanhFn.apply(lrelu(x, slope), w, b, pad)


def available(x) -> bool:
    return x.is_cuda and hip.available()
