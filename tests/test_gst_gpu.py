"""GST reference-encoder kernels (csrc/k_gst.hip + k_bn.hip ReLU mode) vs plain-PyTorch fp32.

Conv2d(3x3, s2) via im2col + MFMA GEMM / col2im, the persistent GRU forward + BPTT, the
style-token attention, BatchNorm+ReLU, and the whole ``GlobalStyleTokens`` module on the GPU
against the same module evaluated on the CPU in fp32.
"""
import copy
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from speakingstyle_amd.ops import hip  # noqa: E402

DEV = "cuda"


def _rel(a, b):
    return ((a.float().cpu() - b.float().cpu()).norm() / (b.float().cpu().norm() + 1e-12)).item()


@pytest.fixture(autouse=True, scope="module")
def _lib_loaded():
    assert hip.available() and hip.has("ssamd_gru_fwd"), "kernel library with k_gst must be built"


@pytest.mark.parametrize("B,H,W,C,Co", [(3, 37, 80, 1, 32), (2, 19, 20, 32, 64), (2, 16, 5, 64, 128)])
def test_conv2d_s2(B, H, W, C, Co):
    torch.manual_seed(0)
    x = torch.randn(B, H, W, C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(Co, C, 3, 3, device=DEV) / math.sqrt(9 * C)).requires_grad_(True)
    b = torch.randn(Co, device=DEV).requires_grad_(True)
    xh = x.clone().requires_grad_(C > 1)
    y = hip.conv2d_s2(xh, w, b)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.detach().to(torch.bfloat16).float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, br, stride=2, padding=1).permute(0, 2, 3, 1)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    if C > 1:
        assert _rel(xh.grad, xr.grad.permute(0, 2, 3, 1)) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2
    assert _rel(b.grad, br.grad) < 1e-2


def test_bn_relu():
    torch.manual_seed(1)
    bn = torch.nn.BatchNorm1d(64).to(DEV)
    bn.weight.data.uniform_(0.5, 1.5)
    bn.bias.data.uniform_(-0.3, 0.3)
    bnr = copy.deepcopy(bn)
    h = torch.randn(3, 50, 64, device=DEV).to(torch.bfloat16).requires_grad_(True)
    hr = h.detach().float().requires_grad_(True)
    y = hip.bn_act(h, bn, True, "relu", 0.0)
    yr = F.relu(F.batch_norm(hr.reshape(-1, 64), bnr.running_mean, bnr.running_var, bnr.weight, bnr.bias, True,
                             0.1, bnr.eps)).reshape(3, 50, 64)
    assert _rel(y, yr) < 1e-2
    assert _rel(bn.running_var, bnr.running_var) < 1e-4
    g = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    assert _rel(h.grad, hr.grad) < 2e-2
    assert _rel(bn.weight.grad, bnr.weight.grad) < 1e-2


@pytest.mark.parametrize("B,T,I,Hd", [(37, 13, 256, 128), (5, 16, 128, 64), (17, 7, 256, 256)])
def test_gru_last(B, T, I, Hd):
    torch.manual_seed(2)
    gru = torch.nn.GRU(I, Hd, batch_first=True).to(DEV)
    grr = copy.deepcopy(gru)
    with torch.no_grad():  # the reference sees the bf16-rounded weights the kernels use
        for p in (grr.weight_ih_l0, grr.weight_hh_l0):
            p.copy_(p.to(torch.bfloat16).float())
    x = (0.5 * torch.randn(B, T, I, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    lens = torch.randint(1, T + 1, (B,), device=DEV)
    lens[0] = T
    last = lens - 1
    h = hip.gru_last(x, gru, last)
    xr = x.detach().float().requires_grad_(True)
    out, _ = grr(xr)
    hr = out.gather(1, last.view(-1, 1, 1).expand(-1, 1, Hd)).squeeze(1)
    assert _rel(h, hr) < 1e-2
    g = torch.randn_like(hr)
    h.backward(g)
    hr.backward(g)
    assert _rel(x.grad, xr.grad) < 3e-2
    for p, pr in zip(gru.parameters(), grr.parameters()):
        assert _rel(p.grad, pr.grad) < 3e-2, p.shape


def test_token_attention():
    torch.manual_seed(3)
    B, NH, N, D = 37, 4, 10, 32
    q = torch.randn(B, NH * D, device=DEV, requires_grad=True)
    K = torch.randn(NH, N, D, device=DEV, requires_grad=True)
    V = torch.randn(NH, N, D, device=DEV, requires_grad=True)
    o, w = hip.token_attention(q, K, V)
    qr, Kr, Vr = (t.detach().clone().requires_grad_(True) for t in (q, K, V))
    wr = torch.softmax(torch.matmul(qr.view(B, NH, 1, D), Kr.transpose(-1, -2).unsqueeze(0)) / math.sqrt(D), -1)
    orr = torch.matmul(wr, Vr.unsqueeze(0)).reshape(B, NH * D)
    assert _rel(o, orr) < 1e-5 and _rel(w, wr.squeeze(2)) < 1e-5
    g = torch.randn_like(orr)
    gw = torch.randn_like(w)  # a loss on the weights too (style-token tuning uses one)
    (o * g).sum().backward(retain_graph=True)
    ((w * gw).sum()).backward()
    ((orr * g).sum() + (wr.squeeze(2) * gw).sum()).backward()
    for t, tr in ((q, qr), (K, Kr), (V, Vr)):
        assert _rel(t.grad, tr.grad) < 1e-4


@pytest.mark.parametrize("filters", [[32, 64], None])
def test_gst_module_matches_cpu(filters):
    """Whole GST encoder on the GPU vs the same module on the CPU in fp32.

    With the full 6-layer stack the gradients of the bottom conv / BN layers differ from fp32 by
    ~17 %: six batch-statistics BatchNorms amplify bf16 rounding.  A CPU run of the fp32 module
    with bf16 rounding inserted at the GPU's storage points shows the same 16 % (measured), so the
    deep case checks the forward and the gradients above the stack, and a 2-layer stack checks
    every gradient at bf16 tolerance (layout, im2col order, GRU feature order, lengths)."""
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.models.style import GlobalStyleTokens

    pp, mc, _ = load_named("BC2013_GST")
    if filters:
        mc["gst"]["conv_filters"] = filters
    torch.manual_seed(4)
    cpu = GlobalStyleTokens(pp, mc).train()
    gpu = copy.deepcopy(cpu).to(DEV)
    B, M = 9, 203
    mel = torch.randn(B, M, 80).to(torch.bfloat16)
    lens = torch.randint(40, M + 1, (B,))
    lens[0] = M
    g_c, b_c = cpu(mel.float(), lens)
    g_g, b_g = gpu(mel.to(DEV), lens.to(DEV))
    assert _rel(g_g, g_c) < 3e-2 and _rel(b_g, b_c) < 3e-2
    (g_c.float().sum() + (b_c.float() ** 2).sum()).backward()
    (g_g.float().sum() + (b_g.float() ** 2).sum()).backward()
    nconv = len(cpu.convs)
    errs = {}
    for (n, p), pg in zip(cpu.named_parameters(), gpu.parameters()):
        assert pg.grad is not None, n
        if n.startswith("convs.") and n.endswith(".bias"):
            # a bias feeding batch-statistics BN has an exactly-zero true gradient: compare absolutely
            assert pg.grad.abs().max().item() < 2e-2 * cpu.convs[int(n.split(".")[1])].weight.grad.abs().max().item() + 1e-4
            continue
        if filters is None and (n.startswith("convs.") or (n.startswith("bns.") and int(n.split(".")[1]) < nconv - 1)):
            continue
        errs[n] = round(_rel(pg.grad, p.grad), 4)
    # the bottom layer sits under one more BatchNorm backward (~7 % of bf16 amplification, the
    # same order as one layer in the emulated run); everything above it at plain bf16 tolerance
    bad = {n: e for n, e in errs.items() if e > (0.1 if n.startswith(("convs.0", "bns.0")) else 6e-2)}
    assert not bad, (bad, errs)


def test_gst_eval_folded_matches_cpu():
    """Inference (eval, no grad): the conv + BatchNorm2d stack runs folded (``folded_convs``: ReLU in the GEMM
    epilogue, cached weight images) -- against the fp32 CPU module in eval, with non-trivial running stats."""
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.models.style import GlobalStyleTokens

    pp, mc, _ = load_named("BC2013_GST")
    torch.manual_seed(5)
    cpu = GlobalStyleTokens(pp, mc)
    for bn in cpu.bns:
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 2.0)
    cpu.eval()
    gpu = copy.deepcopy(cpu).to(DEV)
    mel = torch.randn(3, 150, 80).to(torch.bfloat16)
    lens = torch.tensor([150, 97, 41])
    with torch.no_grad():
        g_c, b_c = cpu(mel.float(), lens)
        g_g, b_g = gpu(mel.to(DEV), lens.to(DEV))
        assert "_fold" in gpu.__dict__ and gpu.__dict__["_fold"][1][0][0] == "img"
        g_g2, _ = gpu(mel.to(DEV), lens.to(DEV))  # cached fold: same result
    assert _rel(g_g, g_c) < 3e-2 and _rel(b_g, b_c) < 3e-2
    assert torch.equal(g_g, g_g2)


def test_style_tuner_gpu():
    """Style-token bank tuning on the GPU path (HIP encoder + token-attention backward)."""
    import numpy as np

    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.train.style_tuning import StyleTokenTuner

    pp, mc, _ = load_named("BC2013_GST")
    mc["transformer"]["encoder_layer"] = mc["transformer"]["decoder_layer"] = 1
    torch.manual_seed(0)
    model = FastSpeech2(pp, mc).to(DEV).set_compute_dtype(torch.bfloat16).eval()
    with torch.no_grad():
        model.gst.w_query.weight.mul_(30.0)  # trained-encoder query magnitude (see the CPU test)
    rng = np.random.default_rng(0)
    f = np.linspace(-1, 1, 80, dtype=np.float32)
    mels, labels = [], []
    for c in range(3):
        for _ in range(6):
            T = int(rng.integers(60, 140))
            mels.append((-6 + 3.0 * c + (c - 1) * 4.0 * f + 0.4 * rng.standard_normal((T, 80))).astype(np.float32))
            labels.append(c)
    res = StyleTokenTuner(model, lr=5e-2, steps=300, tune_projections=True).fit(mels, np.eye(10, dtype=np.float32)[labels])
    assert res["history"][-1]["ce"] < 0.5 * res["history"][0]["ce"]
    assert res["accuracy"] == 1.0


@pytest.mark.parametrize("N,dt,NH,T", [(10, 32, 4, 128), (10, 256, 8, 256), (7, 40, 2, 72)])
def test_token_bank_kernel_vs_torch(N, dt, NH, T):
    """GST token bank (tanh(E) -> key / value projections split into heads) on the HIP kernels vs the
    torch fp32 formulation, forward and the three parameter gradients (multi-workgroup grids, ragged
    last workgroup)."""
    from speakingstyle_amd import ops
    from speakingstyle_amd.ops import hip

    torch.manual_seed(5)
    E = (torch.randn(N, dt, device="cuda") * 0.5).requires_grad_(True)
    Wk = (torch.randn(T, dt, device="cuda") * 0.2).requires_grad_(True)
    Wv = (torch.randn(T, dt, device="cuda") * 0.2).requires_grad_(True)
    Er, Wkr, Wvr = (t.detach().clone().requires_grad_(True) for t in (E, Wk, Wv))
    k, v = hip.token_bank(E, Wk, Wv, NH)
    ops.set_backend("reference")
    try:
        kr, vr = ops.token_bank(Er, Wkr, Wvr, NH)
    finally:
        ops.set_backend(None)
    torch.testing.assert_close(k, kr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(v, vr, rtol=1e-5, atol=1e-5)
    gk, gv = torch.randn_like(kr), torch.randn_like(vr)
    (k * gk + v * gv).sum().backward()
    (kr * gk + vr * gv).sum().backward()
    for a, b in ((E, Er), (Wk, Wkr), (Wv, Wvr)):
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-4, atol=1e-5)
