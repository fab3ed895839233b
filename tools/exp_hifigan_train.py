"""HiFi-GAN V1 generator training step (forward + L1 + backward), HIP channel-last convs vs torch
NCL convs (MIOpen), at the reference training shape (batch 16 x 8192-sample segments) (GPU box)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.models import hifigan as H  # noqa: E402


def run(hip_on, B, frames, iters=10):
    H._hip_train = lambda: hip_on
    torch.manual_seed(0)
    g = H.Generator(H.default_config()).cuda()
    mel = torch.randn(B, 80, frames, device="cuda")
    tgt = torch.randn(B, 1, frames * 256, device="cuda") * 0.1
    for _ in range(3):
        (g(mel) - tgt).abs().mean().backward()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        g.zero_grad(set_to_none=True)
        (g(mel) - tgt).abs().mean().backward()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1000


for B, frames in ((16, 32), (64, 32)):
    res = {"batch": B, "frames": frames}
    for hip_on in (True, False, True, False):
        res.setdefault("hip_ms" if hip_on else "torch_ms", []).append(round(run(hip_on, B, frames), 2))
    print(json.dumps(res), flush=True)
