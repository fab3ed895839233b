"""HiFi-GAN training on the HIP kernels (csrc/k_disc.hip, speakingstyle_amd/vocoder/hip_train.py) against the
fp32 torch modules of models/hifigan.py (reference hifigan/models.py:176-264, meldataset.py:49-72,
train.py:113-160): the strided / grouped / dilated conv kernels (forward, data and weight gradients), the D step
(loss + discriminator weight gradients), the G step's adversarial + feature-matching gradient w.r.t. the
generated waveform, the STFT mel-L1 loss and its gradient, and the generator's HIP glue."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _bf(t):
    return t.to(torch.bfloat16).float()


@pytest.fixture(scope="module", autouse=True)
def _native():
    from speakingstyle_amd.ops import hip

    assert hip.available() and hip.has("ssamd_sconv_fwd"), "HIP kernel library (k_disc) not loaded"


CONV_CASES = [
    # (Cin, Cout, ks, s, d, p, G, act)         act 0 none, 1 lrelu, 2 tanh
    (1, 32, 5, 3, 1, 2, 1, 1),       # MPD layer 0 (Cin = 1: scalar gathers)
    (32, 128, 5, 3, 1, 2, 1, 1),     # MPD layer 1
    (1, 128, 15, 1, 1, 7, 1, 1),     # MSD layer 0
    (128, 128, 41, 2, 1, 20, 4, 1),  # MSD grouped, stride 2
    (128, 256, 41, 2, 1, 20, 16, 1),  # Cg = 8, Ng = 16
    (256, 512, 41, 4, 1, 20, 16, 1),  # stride 4
    (256, 256, 41, 1, 1, 20, 16, 1),  # Ng = 16, stride 1
    (256, 1, 3, 1, 1, 1, 1, 0),      # conv_post (Cout = 1)
    (64, 64, 7, 1, 3, 9, 1, 1),      # dilated
    (32, 1, 7, 1, 1, 3, 1, 2),       # generator conv_post + tanh
    (8, 40, 64, 16, 1, 0, 1, 0),     # STFT-like: long kernel, large stride
]


@pytest.mark.parametrize("case", CONV_CASES, ids=[str(c) for c in CONV_CASES])
def test_sconv_fwd_dgrad_wgrad_vs_torch(case):
    from speakingstyle_amd.vocoder import hip_train as HT

    Cin, Cout, ks, s, d, p, G, act = case
    torch.manual_seed(0)
    B, T = 3, 301
    x = _bf(torch.randn(B, T, Cin, device="cuda"))
    w = _bf(torch.randn(Cout, Cin // G, ks, device="cuda") / (Cin // G * ks) ** 0.5)
    b = torch.randn(Cout, device="cuda") * 0.1
    xr = x.transpose(1, 2).clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    z = F.conv1d(xr, wr, br, stride=s, padding=p, dilation=d, groups=G)
    yr = F.leaky_relu(z, 0.1) if act == 1 else (torch.tanh(z) if act == 2 else z)
    y = HT.sconv_fwd(x.to(torch.bfloat16).contiguous(), HT.fwd_image(w), b, G, ks, s, d, p, act=act, out_f32=True)
    assert y.shape == (B, yr.shape[2], Cout)
    assert _rel(y, yr.transpose(1, 2)) < 5e-3, _rel(y, yr.transpose(1, 2))
    # gradients of <yr, g> w.r.t. x / w / b; the HIP path gets dz = g * act'(y) (bf16)
    g = _bf(torch.randn_like(yr))
    yr.backward(g)
    g_cl = g.transpose(1, 2).contiguous()
    yb = y.to(torch.bfloat16).contiguous()
    if act == 1:
        dz = HT.act_bwd(g_cl.to(torch.bfloat16).contiguous(), yb, 1, 0.1)
    elif act == 2:
        dz = (g_cl * (1 - y * y)).to(torch.bfloat16).contiguous()
    else:
        dz = g_cl.to(torch.bfloat16).contiguous()
    dx = HT.sconv_dgrad(dz, HT.dgrad_image(w, G, s), T, Cin, G, ks, s, d, p, out_f32=True)
    assert _rel(dx, xr.grad.transpose(1, 2)) < 2e-2, _rel(dx, xr.grad.transpose(1, 2))
    dW = HT.sconv_wgrad(dz, x.to(torch.bfloat16).contiguous(), G, ks, s, d, p)
    assert _rel(dW, wr.grad) < 2e-2, _rel(dW, wr.grad)
    from speakingstyle_amd.ops import hip

    db = hip.colsum_raw(dz, Cout)
    assert _rel(db, br.grad) < 2e-2
    dW2, db2 = HT.sconv_wgrad(dz, x.to(torch.bfloat16).contiguous(), G, ks, s, d, p, with_bias=True)
    assert torch.equal(dW2, dW) and _rel(db2, br.grad) < 2e-2
    # the HIP image kernels vs the torch construction
    assert torch.equal(HT.fwd_image(w, G), HT.fwd_image(w.cpu(), G).cuda())
    assert torch.equal(HT.dgrad_image(w, G, s), HT.dgrad_image(w.cpu(), G, s).cuda())


def test_sconv_dgrad_accumulates_fp32():
    from speakingstyle_amd.vocoder import hip_train as HT

    torch.manual_seed(1)
    B, T, Cin, Cout, ks, s, p = 2, 200, 16, 32, 5, 3, 2
    w = _bf(torch.randn(Cout, Cin, ks, device="cuda"))
    Tout = HT.sconv_out_len(T, ks, s, 1, p)
    dz = torch.randn(B, Tout, Cout, device="cuda").to(torch.bfloat16)
    base = torch.randn(B, T, Cin, device="cuda")
    out = base.clone()
    HT.sconv_dgrad(dz, HT.dgrad_image(w, 1, s), T, Cin, 1, ks, s, 1, p, out=out)
    ref = HT.sconv_dgrad(dz, HT.dgrad_image(w, 1, s), T, Cin, 1, ks, s, 1, p, out_f32=True)
    torch.testing.assert_close(out, base + ref, rtol=0, atol=1e-5)


def _discs():
    from speakingstyle_amd.models import hifigan as H

    torch.manual_seed(3)
    mpd = H.MultiPeriodDiscriminator().cuda()
    msd = H.MultiScaleDiscriminator().cuda()
    with torch.no_grad():  # converge spectral_norm's power iteration (a fresh u gives sigma ~ 0 and 1e28 grads)
        w = torch.randn(1, 1, 2048, device="cuda") * 0.1
        for _ in range(30):
            msd.discriminators[0](w)
    # eval: spectral_norm without further power iterations -- the same weight in both paths
    return H, mpd.eval(), msd.eval()


def _wave(B, T, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return _bf(torch.randn(B, T, device="cuda", generator=g) * 0.3)


def test_d_step_loss_and_grads_vs_torch():
    from speakingstyle_amd.vocoder import hip_train as HT

    H, mpd, msd = _discs()
    B, T = 2, 4096
    y, yh = _wave(B, T, 1), _wave(B, T, 2)
    # torch reference (fp32)
    r, g_, _, _ = mpd(y.unsqueeze(1), yh.unsqueeze(1))
    r2, g2, _, _ = msd(y.unsqueeze(1), yh.unsqueeze(1))
    loss_ref = H.discriminator_loss(r, g_)[0] + H.discriminator_loss(r2, g2)[0]
    params = [p for p in list(mpd.parameters()) + list(msd.parameters()) if p.requires_grad]
    gref = torch.autograd.grad(loss_ref, params, allow_unused=True)
    for p in params:
        p.grad = None
    loss = HT.d_step(mpd, msd, y, yh)
    assert abs(loss.item() - loss_ref.item()) / abs(loss_ref.item()) < 2e-2, (loss.item(), loss_ref.item())
    num = den = 0.0
    worst = 0.0
    for p, gr in zip(params, gref):
        if gr is None:
            assert p.grad is None or p.grad.abs().max() == 0
            continue
        assert p.grad is not None
        num += (p.grad.double() - gr.double()).norm().item() ** 2
        den += gr.double().norm().item() ** 2
        worst = max(worst, _rel(p.grad, gr))
    # bf16 activations: ~1 % per tensor; the first layers' weight_v (projected gradients of a Cin = 1 conv) ~7 %
    assert (num / den) ** 0.5 < 3e-2 and worst < 0.12, ((num / den) ** 0.5, worst)


@pytest.mark.parametrize("post_gain", [1.0, 30.0])
def test_g_adv_grad_vs_torch(post_gain):
    """post_gain > 1 scales every weight-normed discriminator's conv_post, so D(y) and D(y_hat) differ widely and the
    score map's feature-matching term (part of the reference's fmap lists) dominates loss and gradient: a G step
    that dropped it fails here."""
    from speakingstyle_amd.vocoder import hip_train as HT

    H, mpd, msd = _discs()
    if post_gain != 1.0:
        with torch.no_grad():
            for d in list(mpd.discriminators) + list(msd.discriminators)[1:]:
                d.conv_post.weight_g.mul_(post_gain)
    B, T = 2, 4096
    y, yh0 = _wave(B, T, 4), _wave(B, T, 5)
    yh = yh0.clone().requires_grad_(True)
    _, g_, fr, fg = mpd(y.unsqueeze(1), yh.unsqueeze(1))
    _, g2, fr2, fg2 = msd(y.unsqueeze(1), yh.unsqueeze(1))
    loss_ref = H.generator_loss(g_)[0] + H.generator_loss(g2)[0] + H.feature_loss(fr, fg) + H.feature_loss(fr2, fg2)
    (dref,) = torch.autograd.grad(loss_ref, [yh], retain_graph=post_gain != 1.0)
    dy = torch.zeros(B, T, device="cuda")
    loss = HT.g_adv(mpd, msd, y, yh0, dy)
    assert abs(loss.item() - loss_ref.item()) / abs(loss_ref.item()) < 2e-2, (loss.item(), loss_ref.item())
    # the boosted score term's gradient runs back through every discriminator layer in bf16: ~8 % vs fp32 torch
    tol = 5e-2 if post_gain == 1.0 else 0.12
    assert _rel(dy, dref) < tol, _rel(dy, dref)
    if post_gain != 1.0:
        # discriminating power: the objective WITHOUT the score-map feature term is far from both
        no_score = (H.generator_loss(g_)[0] + H.generator_loss(g2)[0] + H.feature_loss([f[:-1] for f in fr],
                    [f[:-1] for f in fg]) + H.feature_loss([f[:-1] for f in fr2], [f[:-1] for f in fg2]))
        (dref_ns,) = torch.autograd.grad(no_score, [yh])
        assert _rel(dref_ns, dref) > 3 * tol and _rel(dy, dref_ns) > 3 * tol, (_rel(dref_ns, dref), _rel(dy, dref_ns))
        assert abs(no_score.item() - loss_ref.item()) / abs(loss_ref.item()) > 0.03  # > the 2e-2 loss tolerance


@pytest.mark.parametrize("T", [8192, 8192 + 512])
def test_mel_l1_loss_and_grad_vs_torch(T):
    from speakingstyle_amd.models import hifigan as H
    from speakingstyle_amd.vocoder import hip_train as HT
    from speakingstyle_amd.vocoder.mel import mel_for

    h = H.default_config()
    B = 3
    torch.manual_seed(7)
    y = torch.randn(B, T, device="cuda") * 0.2
    tgt = mel_for(h, torch.randn(B, 8192, device="cuda") * 0.2, loss=True)  # [B, 80, 32]
    yr = y.clone().requires_grad_(True)
    m = mel_for(h, yr, loss=True)
    Fv = min(m.shape[-1], tgt.shape[-1])
    loss_ref = F.l1_loss(tgt[..., :Fv], m[..., :Fv]) * 45
    (dref,) = torch.autograd.grad(loss_ref, [yr])
    dy = torch.zeros(B, T, device="cuda")
    loss = HT.mel_l1(h, y, tgt, 45.0, dy)
    assert abs(loss.item() - loss_ref.item()) / loss_ref.item() < 1e-3, (loss.item(), loss_ref.item())
    assert _rel(dy, dref) < 2e-2, _rel(dy, dref)
    # the HIP STFT log-mel itself (forward only)
    assert _rel(HT.mel_hip(h, y), mel_for(h, y, loss=True)) < 1e-3


def test_generator_hip_glue_matches_torch_path():
    """The channel-last training forward (HIP convs + HIP lrelu / add / mean / conv_post+tanh) against the NCL torch
    forward on the same weights, and the input-weight gradients of <out, r>."""
    from speakingstyle_amd import experimental
    from speakingstyle_amd.models import hifigan as H

    torch.manual_seed(11)
    h = H.default_config()
    g = H.Generator(h).cuda()
    mel = torch.randn(2, 80, 16, device="cuda")
    r = torch.randn(2, 1, 16 * 256, device="cuda")
    with experimental.overrides(hifigan_hip_train=False):
        out_ref = g(mel)
        (out_ref * r).sum().backward()
    gref = {n: p.grad.clone() for n, p in g.named_parameters() if p.grad is not None}
    g.zero_grad(set_to_none=True)
    with experimental.overrides(hifigan_hip_train=True):
        out = g(mel)
        (out * r).sum().backward()
    assert out.shape == out_ref.shape
    assert _rel(out, out_ref) < 3e-2, _rel(out, out_ref)
    for n, p in g.named_parameters():
        if n in gref:
            assert p.grad is not None, n
    # conv_post and the last upsampler's gradients (short chains): bf16 tolerance
    for n in ("conv_post.bias", "conv_post.weight_v", "conv_pre.bias"):
        assert _rel(g.get_parameter(n).grad, gref[n]) < 0.1, (n, _rel(g.get_parameter(n).grad, gref[n]))


def test_hip_step_updates_and_is_finite():
    from speakingstyle_amd.models import hifigan as H
    from speakingstyle_amd.vocoder.mel import mel_for
    from speakingstyle_amd.vocoder.train import hip_step

    torch.manual_seed(5)
    h = H.default_config()
    gen = H.Generator(h).cuda()
    mpd = H.MultiPeriodDiscriminator().cuda()
    msd = H.MultiScaleDiscriminator().cuda()
    opt_g = torch.optim.AdamW(gen.parameters(), 2e-4, betas=(0.8, 0.99))
    opt_d = torch.optim.AdamW(list(mpd.parameters()) + list(msd.parameters()), 2e-4, betas=(0.8, 0.99))
    B, frames = 2, 32
    y = torch.randn(B, frames * 256, device="cuda") * 0.2
    x = mel_for(h, y)
    y_mel = mel_for(h, y, loss=True)
    d0 = next(mpd.parameters()).detach().clone()
    g0 = gen.conv_post.bias.detach().clone()
    for _ in range(2):
        y_g = gen(x)
        loss_g, loss_mel = hip_step(h, mpd, msd, opt_d, opt_g, y, y_g.squeeze(1), y_mel)
        assert torch.isfinite(loss_g).all() and torch.isfinite(loss_mel).all()
    assert not torch.equal(next(mpd.parameters()).detach(), d0)
    assert not torch.equal(gen.conv_post.bias.detach(), g0)


def test_hifigan_train_cli_on_gpu(tmp_path):
    """``hifigan_train.py`` end to end on the GPU (synthetic tones, V1 config at batch 2): the HIP step
    (vocoder/train.py:hip_step) runs, logs the reference's TensorBoard tags, validates, checkpoints."""
    import json
    import os
    import subprocess
    import sys

    from speakingstyle_amd.models.hifigan import default_config
    from speakingstyle_amd.utils.tb import read_scalars

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    h = default_config()
    h.update(batch_size=2, num_workers=0)
    cfg = tmp_path / "config.json"
    cfg.write_text(json.dumps(dict(h)))
    ck = tmp_path / "ck"
    args = [sys.executable, "hifigan_train.py", "--synthetic", "--config", str(cfg), "--checkpoint_path", str(ck),
            "--checkpoint_interval", "2", "--validation_interval", "2", "--summary_interval", "1",
            "--stdout_interval", "1", "--num_workers", "0", "--training_steps", "3"]
    r = subprocess.run(args, cwd=root, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "Steps : 2," in r.stdout
    assert (ck / "g_00000002").exists() and (ck / "do_00000002").exists()
    logs = ck / "logs"
    tags = {t for f in os.listdir(logs) if f.startswith("events") for _, t, _ in read_scalars(str(logs / f))}
    assert {"training/gen_loss_total", "training/mel_spec_error", "validation/mel_spec_error"} <= tags
