"""Per-parameter comparison of the HIP D step / G step against torch (debug helper, GPU box)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.models import hifigan as H  # noqa: E402
from speakingstyle_amd.vocoder import hip_train as HT  # noqa: E402

torch.manual_seed(3)
mpd = H.MultiPeriodDiscriminator().cuda().eval()
msd = H.MultiScaleDiscriminator().cuda().eval()
B, T = 2, 4096
g = torch.Generator(device="cuda").manual_seed(1)
y = (torch.randn(B, T, device="cuda", generator=g) * 0.3).bfloat16().float()
yh = (torch.randn(B, T, device="cuda", generator=g) * 0.3).bfloat16().float()
r, g_, fr, fg = mpd(y.unsqueeze(1), yh.unsqueeze(1))
r2, g2, fr2, fg2 = msd(y.unsqueeze(1), yh.unsqueeze(1))
for name, outs in (("mpd_r", r), ("mpd_g", g_), ("msd_r", r2), ("msd_g", g2)):
    print(name, [f"{o.float().abs().max().item():.3g}" for o in outs])
loss_ref = H.discriminator_loss(r, g_)[0] + H.discriminator_loss(r2, g2)[0]
named = [(n, p) for n, p in list(mpd.named_parameters()) + [("msd." + n, p) for n, p in msd.named_parameters()]]
gref = torch.autograd.grad(loss_ref, [p for _, p in named], allow_unused=True)
for _, p in named:
    p.grad = None
loss = HT.d_step(mpd, msd, y, yh)
print("loss", loss.item(), loss_ref.item())
for (n, p), gr in zip(named, gref):
    if gr is None:
        print(n, "ref None", None if p.grad is None else p.grad.abs().max().item())
        continue
    a = p.grad.double()
    b = gr.double()
    print(f"{n:40s} ref|{b.norm().item():.3e}| hip|{a.norm().item():.3e}| rel {((a - b).norm() / b.norm()).item():.3e}"
          f" finite {torch.isfinite(a).all().item()} {torch.isfinite(b).all().item()}")
