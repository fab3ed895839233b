"""Golden parity against the reference's own modules (read-only oracle, fp32 CPU).

Weights are copied by identical state_dict keys; outputs and gradients must
match.  Covers: full FastSpeech2 forward with the FiLM reference encoder
(BC2013 config), loss terms, LR schedule.
"""
import contextlib
import copy
import io
import os

import pytest
import torch

from speakingstyle_amd.config import load_named
from speakingstyle_amd.data.synthetic import SyntheticBatches
from speakingstyle_amd.models.fastspeech2 import FastSpeech2
from speakingstyle_amd.models.loss import FastSpeech2Loss
from speakingstyle_amd.train.optim import ScheduledOptim

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfgs(name):
    pp, mc, tc = load_named(name)
    pp = copy.deepcopy(pp)
    pp["path"]["preprocessed_path"] = os.path.join(ROOT, "preprocessed_data", "BC2013")
    return pp, mc, tc


@pytest.fixture(scope="module")
def pair(reference_modules):
    torch.manual_seed(0)
    pp, mc, tc = _cfgs("BC2013")
    ours = FastSpeech2(pp, mc).eval()
    with contextlib.redirect_stdout(io.StringIO()):
        ref = reference_modules.model.FastSpeech2(pp, mc).eval()
    missing = ref.load_state_dict(ours.state_dict(), strict=True)
    return ours, ref, (pp, mc, tc)


def _batch(B=3, seed=3):
    g = SyntheticBatches(B, max_seq_len=1000, seed=seed, phone_counts=[12, 17, 23, 9])
    return g.make_batch()


def test_state_dict_keys_match(pair):
    ours, ref, _ = pair
    assert list(ours.state_dict().keys()) == list(ref.state_dict().keys())
    for (k, a), (_, b) in zip(ours.state_dict().items(), ref.state_dict().items()):
        assert a.shape == b.shape, k


def test_forward_matches_reference(pair):
    ours, ref, _ = pair
    b = _batch()
    with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
        o = ours(*b[2:])
        r = ref(*b[2:])
    names = ["mel", "postnet", "pitch", "energy", "log_d"]
    for i, n in enumerate(names):
        torch.testing.assert_close(o[i], r[i], rtol=1e-4, atol=1e-4, msg=n)
    assert torch.equal(o[6], r[6]) and torch.equal(o[7], r[7])


def test_inference_matches_reference(pair):
    """No targets: duration rounding + length regulation from predictions."""
    ours, ref, _ = pair
    b = _batch(B=2, seed=5)
    with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
        o = ours(b[2], b[3], b[4], b[5], b[6], b[7], b[8])
        r = ref(b[2], b[3], b[4], b[5], b[6], b[7], b[8])
    torch.testing.assert_close(o[5].float(), r[5].float())
    torch.testing.assert_close(o[9].long(), r[9].long())
    M = o[1].shape[1]
    torch.testing.assert_close(o[1], r[1][:, :M], rtol=1e-4, atol=1e-4)


def test_loss_and_grads_match(pair, reference_modules):
    ours, ref, (pp, mc, tc) = pair
    ours.train()
    ref.train()
    b = _batch(seed=7)
    # dropout off so both sides are deterministic
    for m in list(ours.modules()) + list(ref.modules()):
        if hasattr(m, "dropout") and isinstance(getattr(m, "dropout"), float):
            m.dropout = 0.0
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    import torch.nn.functional as F
    orig = F.dropout
    F.dropout = lambda x, p=0.5, training=True, inplace=False: x
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            o = ours(*b[2:])
            r = ref(*b[2:])
            lo = FastSpeech2Loss(pp, tc)(b, o, ours.film_scalars())
            named = torch.stack([p for n, p in ref.named_parameters() if "s_gamma" in n or "s_beta" in n])
            lr_ = reference_modules.loss.FastSpeech2Loss(pp, tc)(b, r, named)
    finally:
        F.dropout = orig
    for a, c in zip(lo[:6], lr_[:6]):
        torch.testing.assert_close(a, c, rtol=1e-4, atol=1e-5)
    lo[0].backward()
    lr_[0].backward()
    gp = dict(ref.named_parameters())
    for n, p in ours.named_parameters():
        if p.grad is None:
            continue
        torch.testing.assert_close(p.grad, gp[n].grad, rtol=2e-3, atol=2e-5, msg=n)
    ours.eval(); ref.eval()


def test_lr_schedule_matches_reference(pair, reference_modules):
    ours, ref, (pp, mc, tc) = pair
    ro = reference_modules.optimizer.ScheduledOptim(ref, tc, mc, 0)
    mo = ScheduledOptim(copy.deepcopy(ours), tc, mc, 0)
    for step in [0, 1, 5000, 10000, 10001, 300001, 400001, 500001]:
        ro.current_step = step
        assert abs(ro._get_lr_scale() - mo._get_lr(step)) < 1e-12, step
