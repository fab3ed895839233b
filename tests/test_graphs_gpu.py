"""HIP-graph training steps (speakingstyle_amd/train/graphs.py) against the eager step on the same padded
batches: losses, the flat-arena weights after every optimizer step and BatchNorm running statistics are
bitwise equal -- dropout on (the per-step dropout salt is device data the graph loads), FiLM reference
encoder and GST configs included."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(name, B=8):
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.train.trainer import Trainer

    pp, mc, tc = load_named(name)
    mc["transformer"]["encoder_layer"] = mc["transformer"]["decoder_layer"] = 2
    fl = pp["preprocessing"]["pitch"]["feature"] == "frame_level"
    batches = [SyntheticBatches(B, device="cuda", seed=40 + i, frame_level=fl).make_batch() for i in range(2)]
    torch.manual_seed(3)
    m = FastSpeech2(pp, mc).to("cuda").set_compute_dtype(torch.bfloat16)

    def trainer():
        tr = Trainer(copy.deepcopy(m), (pp, mc, tc), seed=77)
        tr.use_priority_stream()
        return tr
    return trainer, batches


@pytest.mark.parametrize("name", ["LJSpeech", "BC2013", "BC2013_GST"])
def test_graph_step_bitwise_equals_eager(name):
    from speakingstyle_amd.train.graphs import GraphedSteps

    make, batches = _setup(name)
    eager, tg = make(), make()
    gs = GraphedSteps(tg, warm=1)
    try:
        for i in range(6):
            b = batches[i % 2]
            pb, _ = gs.pad_batch(b)
            le, _, _ = eager.train_step(pb)
            lg, _, _ = gs.step(b)
            torch.cuda.synchronize()
            for a, c in zip(le[:6], lg[:6]):
                assert torch.equal(a.detach().float(), c.detach().float()), (i, a.item(), c.item())
            assert torch.equal(eager.opt.arena.data, tg.opt.arena.data), i
        assert gs.captures >= 1 and gs.replays >= 4, gs.stats()
        for (n, x), (_, y) in zip(eager.model.named_buffers(), tg.model.named_buffers()):
            assert torch.equal(x, y), n
        assert int(eager.opt.skipped_steps) == int(tg.opt.skipped_steps) == 0
    finally:
        torch.cuda.set_stream(torch.cuda.default_stream())


def test_graph_replays_draw_new_dropout_masks():
    """Two replays of one captured bucket on the same batch give different losses (new dropout masks from the
    device salt), while the eager step with the same (step, micro-step) salt reproduces each replay."""
    from speakingstyle_amd.train.graphs import GraphedSteps

    make, batches = _setup("LJSpeech")
    tg = make()
    gs = GraphedSteps(tg, warm=1)
    try:
        b = batches[0]
        gs.step(b)  # eager warm-up
        l1 = [x.detach().float().clone() for x in gs.step(b)[0][:6]]  # capture + replay
        l2 = [x.detach().float().clone() for x in gs.step(b)[0][:6]]
        torch.cuda.synchronize()
        assert gs.replays == 2
        assert not torch.equal(l1[1], l2[1])  # weights moved and masks changed
    finally:
        torch.cuda.set_stream(torch.cuda.default_stream())
