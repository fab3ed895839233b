"""Training-step guarantees on the GPU:

* determinism -- every cross-block reduction of the step is fixed-order (csrc/k_reduce.hip),
  dropout masks are a pure function of (seed, rank, step): two runs with the same seed give
  bitwise-identical losses, gradients norms and parameters;
* checkpoint/resume -- ``Trainer`` for 5 steps == 3 steps, save (model + optimizer), restore
  into a fresh model/trainer, 2 more steps: bitwise identical (the reference's resume drops the
  weights)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _setup(name="LJSpeech", layers=2, dropout=True):
    from speakingstyle_amd.config import load_named

    pp, mc, tc = load_named(name)
    mc["transformer"]["encoder_layer"] = mc["transformer"]["decoder_layer"] = layers
    if not dropout:
        mc["transformer"]["encoder_dropout"] = mc["transformer"]["decoder_dropout"] = 0.0
    return pp, mc, tc


def _batches(n, B=12, seed=5):
    from speakingstyle_amd.data.synthetic import SyntheticBatches

    g = SyntheticBatches(B, device=DEV, seed=seed)
    return [g.make_batch() for _ in range(n)]


def _fresh(cfg, seed=11):
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.train.trainer import Trainer

    torch.manual_seed(seed)
    m = FastSpeech2(*cfg[:2]).to(DEV).set_compute_dtype(torch.bfloat16)
    return m, Trainer(m, cfg, seed=1234)


def _run(tr, batches):
    out = []
    for b in batches:
        losses, _, _ = tr.train_step(b)
        out.append(torch.stack([l.detach().float().reshape(()) for l in losses[:6]]))
    torch.cuda.synchronize()
    return torch.stack(out).cpu()


@pytest.mark.parametrize("name", ["LJSpeech", "BC2013", "BC2013_GST"])
def test_bitwise_deterministic_steps(name):
    cfg = _setup(name)
    bs = _batches(3)
    m1, t1 = _fresh(cfg)
    l1 = _run(t1, bs)
    p1 = t1.opt.arena.data.clone()
    n1 = t1.opt.last_grad_norm.clone()
    m2, t2 = _fresh(cfg)
    l2 = _run(t2, bs)
    assert torch.isfinite(l1).all()
    assert torch.equal(l1, l2), (l1 - l2).abs().max()
    assert torch.equal(n1, t2.opt.last_grad_norm)
    assert torch.equal(p1, t2.opt.arena.data)


def test_trainer_save_restore_continuation(tmp_path):
    from speakingstyle_amd.utils import model as mutil

    cfg = _setup("LJSpeech")
    bs = _batches(5, seed=9)
    m, tr = _fresh(cfg)
    _run(tr, bs[:3])
    path = mutil.save_checkpoint(os.path.join(tmp_path, "3.pth.tar"), m, tr.opt, 3)
    ref_losses = _run(tr, bs[3:])
    ref_params = tr.opt.arena.data.clone()

    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.train.trainer import Trainer

    torch.manual_seed(999)  # different init: everything must come from the checkpoint
    m2 = FastSpeech2(*cfg[:2]).to(DEV).set_compute_dtype(torch.bfloat16)
    ck = mutil.load_checkpoint(path)
    mutil.restore_model(m2, ck)
    tr2 = Trainer(m2, cfg, restore_step=3, seed=1234)
    tr2.opt.load_state_dict(ck["optimizer"])
    assert tr2.opt.step_count == 3 and tr2.opt.current_step == 3
    losses = _run(tr2, bs[3:])
    assert torch.equal(losses, ref_losses), (losses - ref_losses).abs().max()
    assert torch.equal(tr2.opt.arena.data, ref_params)


@pytest.mark.parametrize("name", ["LJSpeech", "BC2013"])
def test_side_stream_weight_gradients_bitwise(name):
    """Weight gradients on the side stream (default) == on the main stream, bitwise: same kernels,
    same reduction order; the joins before the optimizer order everything."""
    from speakingstyle_amd import experimental

    cfg = _setup(name)
    bs = _batches(3, seed=8)
    res = []
    for side in ("1", "0"):
        with experimental.overrides(side_wgrad=side):
            m, t = _fresh(cfg)
            l = _run(t, bs)
            res.append((l, t.opt.arena.data.clone(), float(t.opt.last_grad_norm)))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
    assert res[0][2] == res[1][2]
