"""Fused residual+LayerNorm GEMM tail vs separate addln kernels across dropout seeds: forward / input-gradient
agreement and the worst per-parameter gradient difference (diagnostic for test_gemm_fused_layernorm)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/tests")
from speakingstyle_amd import experimental, ops  # noqa: E402
from speakingstyle_amd.models.layers import FFTBlock  # noqa: E402
from speakingstyle_amd.ops import hip  # noqa: E402

DEV = "cuda"


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def probe(seed, packed, film):
    torch.manual_seed(3)
    blk = FFTBlock(256, 2, 128, 128, 1024, (9, 1), dropout=0.1, film=True).to(DEV).train()
    B, L = 4, 50
    lens = torch.tensor([50, 31, 7, 44], device=DEV)
    x0 = torch.randn(B, L, 256, device=DEV).to(torch.bfloat16)
    style = (torch.randn(B, 256, device=DEV).to(torch.bfloat16), torch.randn(B, 256, device=DEV).to(torch.bfloat16))
    with torch.no_grad():
        blk.film.s_gamma.fill_(0.3)
        blk.film.s_beta.fill_(-0.2)
    pk = None
    if packed:
        R = int(lens.sum())
        pk = ops.PackInfo.build(lens, L, R)
        x0 = torch.cat([x0[b, : int(lens[b])] for b in range(B)], 0).unsqueeze(0).contiguous()

    def run(no_fuse):
        with experimental.overrides(ln_fuse=not no_fuse):
            hip.set_seed(seed)
            blk.zero_grad()
            x = x0.clone().requires_grad_(True)
            y = blk(x, lens, style if film else None, pack=pk)
            g = torch.randn(y.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(1)).to(torch.bfloat16)
            y.backward(g)
            return y.detach().float(), x.grad.float(), [(n, p.grad.clone()) for n, p in blk.named_parameters()
                                                         if p.grad is not None]

    y1, gx1, gp1 = run(False)
    y2, gx2, gp2 = run(True)
    worst = max(((_rel(a, b), n) for (n, a), (_, b) in zip(gp1, gp2)))
    print(f"seed {seed} packed {packed} film {film}: y {_rel(y1, y2):.2e} gx {_rel(gx1, gx2):.2e} "
          f"all {_rel(torch.cat([a.flatten() for _, a in gp1]), torch.cat([b.flatten() for _, b in gp2])):.2e} "
          f"worst {worst[0]:.3f} {worst[1]}", flush=True)


for sd in (70, 73, 77, 78):
    for packed, film in ((False, False), (False, True), (True, True)):
        probe(sd, packed, film)
