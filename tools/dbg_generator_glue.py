import sys, os
sys.path.insert(0, os.getcwd())
import torch
from speakingstyle_amd.models import hifigan as H
def rel(a, b): return ((a.double() - b.double()).norm() / b.double().norm()).item()
def run(glue_torch, loss="mse"):
    h = H.default_config(); h.upsample_initial_channel = 128
    torch.manual_seed(4)
    g = H.Generator(h).cuda()
    for m in g.modules():
        if isinstance(m, (torch.nn.Conv1d, torch.nn.ConvTranspose1d)) and hasattr(m, "weight_v"):
            m.weight_v.data.normal_(0.0, 0.05)
    mel = torch.randn(2, h.num_mels, 12, device="cuda"); target = torch.randn(2, 1, 12 * 256, device="cuda") * 0.1
    saved_glue = H._glue
    if glue_torch: H._glue = lambda x: H._TorchGlue
    y = g(mel); ((y - target) ** 2).mean().backward()
    H._glue = saved_glue
    gh = {n: p.grad.clone() for n, p in g.named_parameters() if p.grad is not None}
    g.zero_grad(set_to_none=True)
    s = H._hip_train; H._hip_train = lambda: False
    yr = g(mel); ((yr - target) ** 2).mean().backward(); H._hip_train = s
    worst = sorted(((rel(gh[n], p.grad), n, p.grad.norm().item()) for n, p in g.named_parameters() if n in gh and p.grad.norm() > 1e-8), reverse=True)[:6]
    print("torch_glue" if glue_torch else "hip_glue", "out rel", rel(y, yr), [(round(a, 3), n, f"{b:.2e}") for a, n, b in worst])
run(True); run(False)
