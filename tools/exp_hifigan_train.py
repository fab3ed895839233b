"""HiFi-GAN V1 training step at the reference shape (batch 16 x 8192-sample segments, hifigan/config.json):
the whole D + G update (generator forward, discriminator loss + backward + AdamW, mel-L1 + adversarial +
feature-matching loss, generator backward + AdamW) on the HIP kernels (vocoder/train.py:hip_step) against the
torch modules on MIOpen (torch_step), and the generator-only forward + L1 + backward of earlier rounds (GPU box).
Prints one JSON line per configuration."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd import experimental  # noqa: E402
from speakingstyle_amd.models import hifigan as H  # noqa: E402
from speakingstyle_amd.vocoder.mel import mel_for  # noqa: E402
from speakingstyle_amd.vocoder.train import hip_step, torch_step  # noqa: E402


def full_step(use_hip, B, frames, iters=5, warm=2):
    torch.manual_seed(0)
    h = H.default_config()
    gen = H.Generator(h).cuda()
    mpd = H.MultiPeriodDiscriminator().cuda()
    msd = H.MultiScaleDiscriminator().cuda()
    opt_g = torch.optim.AdamW(gen.parameters(), h.learning_rate, betas=(h.adam_b1, h.adam_b2))
    opt_d = torch.optim.AdamW(list(mpd.parameters()) + list(msd.parameters()), h.learning_rate,
                              betas=(h.adam_b1, h.adam_b2))
    y = torch.randn(B, frames * 256, device="cuda") * 0.2
    x = mel_for(h, y)
    y_mel = mel_for(h, y, loss=True)

    def step():
        with experimental.overrides(hifigan_hip_train=use_hip):
            y_g = gen(x)
            if use_hip:
                return hip_step(h, mpd, msd, opt_d, opt_g, y, y_g.squeeze(1), y_mel)
            return torch_step(h, mpd, msd, opt_d, opt_g, y.unsqueeze(1), y_g, y_mel)

    for _ in range(warm):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        loss_g, loss_mel = step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / iters * 1000
    return ms, float(loss_g.detach()), float(loss_mel.detach())


def gen_only(hip_on, B, frames, iters=10):
    torch.manual_seed(0)
    g = H.Generator(H.default_config()).cuda()
    mel = torch.randn(B, 80, frames, device="cuda")
    tgt = torch.randn(B, 1, frames * 256, device="cuda") * 0.1
    with experimental.overrides(hifigan_hip_train=hip_on):
        for _ in range(3):
            (g(mel) - tgt).abs().mean().backward()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            g.zero_grad(set_to_none=True)
            (g(mel) - tgt).abs().mean().backward()
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1000


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "full"
    if which in ("full", "all"):
        for B in (16,):
            res = {"what": "hifigan train step (D + G, AdamW)", "batch": B, "segment": 8192}
            for use_hip in (True, False, True, False):
                ms, lg, lm = full_step(use_hip, B, 32)
                key = "hip" if use_hip else "torch"
                res.setdefault(key + "_ms", []).append(round(ms, 2))
                res[key + "_loss_g"] = round(lg, 4)
                res[key + "_loss_mel"] = round(lm, 4)
            print(json.dumps(res), flush=True)
    if which == "hip":  # profiling: the HIP step only
        ms, lg, lm = full_step(True, 16, 32, iters=3, warm=2)
        print(json.dumps({"what": "hifigan train step (HIP)", "batch": 16, "hip_ms": round(ms, 2)}), flush=True)
    if which in ("gen", "all"):
        for B, frames in ((16, 32),):
            res = {"what": "generator fwd + L1 + bwd", "batch": B, "frames": frames}
            for hip_on in (True, False):
                res.setdefault("hip_ms" if hip_on else "torch_ms", []).append(round(gen_only(hip_on, B, frames), 2))
            print(json.dumps(res), flush=True)
