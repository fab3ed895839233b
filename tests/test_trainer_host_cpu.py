"""Trainer host-side knobs (CPU): backward on the calling thread (``mi355x.backward_same_thread``,
``torch.autograd.set_multithreading_enabled``), the step-tail marks (``host_tail`` switch) and that
the calling-thread backward leaves the gradients unchanged."""
import torch

from speakingstyle_amd.benchmark import tiny_overrides
from speakingstyle_amd.config import load_named
from speakingstyle_amd.data.synthetic import SyntheticBatches
from speakingstyle_amd.models.fastspeech2 import FastSpeech2
from speakingstyle_amd.train.trainer import Trainer


def _setup(same_thread):
    pp, mc, tc = load_named("LJSpeech")
    tiny_overrides(mc)
    tc.setdefault("mi355x", {})["backward_same_thread"] = same_thread
    torch.manual_seed(0)
    model = FastSpeech2(pp, mc)
    tr = Trainer(model, (pp, mc, tc), seed=3)
    gen = SyntheticBatches(3, device="cpu", max_seq_len=mc["max_seq_len"], seed=7)
    return tr, gen.make_batch()


def test_calling_thread_backward_is_configurable_and_exact(monkeypatch):
    before = torch.autograd.is_multithreading_enabled()
    try:
        out = {}
        for same in (False, True):
            tr, b = _setup(same)
            assert torch.autograd.is_multithreading_enabled() == (not same)
            losses, _, _ = tr.train_step(b)
            assert torch.isfinite(losses[0])
            out[same] = torch.cat([p.detach().reshape(-1) for p in tr.model.parameters()])
        torch.testing.assert_close(out[False], out[True], rtol=0, atol=0)
    finally:
        torch.autograd.set_multithreading_enabled(before)


def test_host_tail_marks(monkeypatch):
    from speakingstyle_amd import experimental

    monkeypatch.setenv("SSAMD_EXPERIMENTAL", "host_tail=1")
    experimental.reset_for_tests()
    before = torch.autograd.is_multithreading_enabled()
    try:
        tr, b = _setup(True)
        for _ in range(2):
            tr.train_step(b)
        tail = tr.host_tail_summary()
        assert set(tail) == {"bwd_call->bwd_return", "bwd_return->joined", "joined->finalized",
                             "finalized->opt_launched", "opt_launched->step_end"}
        assert all(v >= 0 for v in tail.values())
    finally:
        torch.autograd.set_multithreading_enabled(before)
        monkeypatch.delenv("SSAMD_EXPERIMENTAL")
        experimental.reset_for_tests()
