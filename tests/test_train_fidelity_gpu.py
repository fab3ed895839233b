"""Training fidelity beyond one step: the HIP bf16 training path and the torch fp32 path
(``set_backend("reference")``: plain PyTorch ops, fp32 activations) overfit the same fixed batch
from the same initial weights for 200 steps on the same GPU.  The loss curves must track each
other (reference loss ``model/loss.py:43-99``, optimizer ``model/optimizer.py``).

Dropout is off in both (the HIP kernels draw counter-hash masks, torch its own RNG: with dropout
the two runs would follow different noise, not different numerics).  The learning rate is held
at 5e-4 (the reference schedule's warm-up would keep it ~1e-6 for the first 200 steps)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
STEPS = 200


def _configs(name):
    from speakingstyle_amd.config import load_named

    pp, mc, tc = load_named(name)
    mc["transformer"].update(encoder_dropout=0.0, decoder_dropout=0.0)
    mc["variance_predictor"]["dropout"] = 0.0
    if mc.get("reference_encoder"):
        mc["reference_encoder"]["dropout"] = 0.0
    tc["optimizer"].update(init_lr=5e-4, anneal_lr=5e-4)
    tc["loss"]["anneal_steps"] = 1
    return pp, mc, tc


def _run(cfg, model, batch, hip: bool):
    from speakingstyle_amd import ops
    from speakingstyle_amd.train.trainer import Trainer

    ops.set_backend(None if hip else "reference")
    try:
        model.set_compute_dtype(torch.bfloat16 if hip else torch.float32)
        model.postnet.dropout = 0.0
        tr = Trainer(model, cfg, seed=1234)
        curve = []
        for _ in range(STEPS):
            losses, _, _ = tr.train_step(batch)
            curve.append(losses[0].detach().float().reshape(()))
        torch.cuda.synchronize()
        return torch.stack(curve).cpu(), int(tr.opt.skipped_steps)
    finally:
        ops.set_backend(None)


@pytest.mark.parametrize("name", ["LJSpeech", "BC2013"])
def test_overfit_curves_hip_bf16_vs_torch_fp32(name):
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2

    cfg = _configs(name)
    torch.manual_seed(21)
    m_hip = FastSpeech2(cfg[0], cfg[1]).to(DEV)
    m_ref = copy.deepcopy(m_hip)
    fl = cfg[0]["preprocessing"]["pitch"]["feature"] == "frame_level"
    batch = SyntheticBatches(8, device=DEV, seed=4, frame_level=fl).make_batch()
    c_hip, sk_hip = _run(cfg, m_hip, batch, hip=True)
    c_ref, sk_ref = _run(cfg, m_ref, batch, hip=False)
    assert sk_hip == sk_ref == 0
    assert torch.isfinite(c_hip).all() and torch.isfinite(c_ref).all()
    # it trains: the fixed batch is fitted well below the initial loss
    assert c_ref[-1] < 0.5 * c_ref[0] and c_hip[-1] < 0.5 * c_hip[0]
    # final loss (mean of the last 10 steps) within 5 %; the gap between the 10-step-smoothed curves
    # from step 20 on within 4 % on average and 2.5 % at the median.  Not pointwise: the overfit
    # trajectory is chaotic -- a transient loss bump lands a few steps apart in the two runs (measured
    # on MI355X, LJSpeech: one window at 15 % while the final losses agree to 0.07 %, mean gap 1.7 %)
    tail = lambda c: c[-10:].mean()  # noqa: E731
    k = 10
    sm = lambda c: torch.nn.functional.avg_pool1d(c.view(1, 1, -1), k, k).view(-1)  # noqa: E731
    rel = ((sm(c_hip) - sm(c_ref)).abs() / sm(c_ref))[2:]
    print(f"{name}: loss hip {c_hip[0]:.3f} -> {tail(c_hip):.4f}, fp32 {c_ref[0]:.3f} -> {tail(c_ref):.4f}; "
          f"smoothed-curve gap max {rel.max():.4f} mean {rel.mean():.4f}")
    assert abs(tail(c_hip) - tail(c_ref)) <= 0.05 * tail(c_ref), (tail(c_hip), tail(c_ref))
    assert rel.mean().item() <= 0.04 and rel.median().item() <= 0.025, rel
