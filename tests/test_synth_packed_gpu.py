"""Packed synthesis (FastSpeech2.infer_packed -> Generator.infer_packed): the decoder, PostNet and vocoder run on
the valid frames only.  Each utterance must come out as its batch-1 synthesis (the padded path on that utterance
alone), and the frames away from the ends must match the padded batch (whose padded frames leak into the last
PostNet frames of the shorter utterances only)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp(min=1e-12)).item()


@pytest.fixture
def pinned_gemm():
    """The GEMM kernel choice depends on the row count (skinny kernel, fused GEMM + LayerNorm and split-K for few
    rows / tiles), so a batch-1 run and the packed batch accumulate in different orders; the bucketized pitch /
    energy embeddings turn such rounding differences into bucket flips.  The packing semantics are compared with
    one kernel family."""
    from speakingstyle_amd.ops import hip

    hip.lib().ssamd_gemm_set_skinny(0)
    hip.lib().ssamd_gemm_set_splitk(0)
    rows = hip.GEMM_ADDLN_MAX_ROWS
    hip.GEMM_ADDLN_MAX_ROWS = 0
    yield
    hip.lib().ssamd_gemm_set_skinny(1)
    hip.lib().ssamd_gemm_set_splitk(-1)
    hip.GEMM_ADDLN_MAX_ROWS = rows


@pytest.mark.parametrize("config", ["BC2013_GST", "LJSpeech"])
def test_fs2_infer_packed_equals_each_utterance_alone(config, pinned_gemm):
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.models.hifigan import Generator, default_config

    dev = torch.device("cuda", 0)
    pp, mc, tc = load_named(config)
    torch.manual_seed(0)
    model = FastSpeech2(pp, mc).to(dev)
    with torch.no_grad():  # ~8 frames per phoneme (the bench's duration head)
        lin = model.variance_adaptor.duration_predictor.linear_layer
        lin.weight.normal_(0.0, 0.005)
        lin.bias.fill_(math.log(9.1))
    model.eval().set_compute_dtype(torch.bfloat16)
    model.requires_grad_(False)
    b = SyntheticBatches(6, device=dev, seed=3, max_seq_len=mc["max_seq_len"]).make_batch()
    args = (b[2], b[3], b[4], b[5], b[6], b[7], b[8])
    assert model.packed_inference_ok(b[3])
    rows, lens, mel_len = model.infer_packed(*args)
    assert rows.shape == (sum(lens), 80) and rows.dtype == torch.float32
    with torch.no_grad():
        pad = model(*args)
    assert pad[9].tolist() == lens
    cu = [0]
    for n in lens:
        cu.append(cu[-1] + n)
    for i, n in enumerate(lens):
        # the same padded text / reference-mel inputs (style and encoder see exactly what the batch saw); the
        # length-regulated half then runs at this utterance's own length
        one = tuple(a[i:i + 1] if isinstance(a, torch.Tensor) else a for a in args)
        with torch.no_grad():
            alone = model(*one)
        assert alone[9].tolist() == [n]
        mine = rows[cu[i]:cu[i + 1]]
        assert _rel(mine, alone[1][0, :n]) < 2e-2, (i, _rel(mine, alone[1][0, :n]))
        # away from the end (the PostNet's 5 x k5 receptive field) the padded batch agrees too
        if n > 16:
            assert _rel(mine[: n - 12], pad[1][i, : n - 12]) < 2e-2
    # and the vocoder on the packed rows == on the padded mel with lengths (both length-exact paths)
    torch.manual_seed(1)
    g = Generator(default_config()).eval().fold_weight_norm().to(dev)
    w_rows = g.infer_packed(rows, lens, int16_scale=32768.0)
    w_pad = g.infer(pad[1], int16_scale=32768.0, lengths=lens)
    assert w_rows.shape == (len(lens), max(lens) * 256)
    for i, n in enumerate(lens):
        if n > 16:
            m = (n - 16) * 256
            assert _rel(w_rows[i, :m], w_pad[i, :m]) < 5e-2
        assert not w_rows[i, n * 256:].any()


def test_synth_graphs_replay_equals_eager():
    """infer/graphs.SynthGraphs: the captured packed synthesis (graph 1: style + encoder + variance adaptor +
    durations; graph 2: decoder + PostNet + vocoder for the returned lengths) replays bitwise the eager packed
    synthesis -- for new inputs of the same shapes too (replays read the static inputs) -- and new length sets
    warm / capture their own graph 2."""
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.infer.graphs import SynthGraphs
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.models.hifigan import Generator, default_config

    dev = torch.device("cuda", 0)
    pp, mc, tc = load_named("BC2013_GST")
    torch.manual_seed(0)
    model = FastSpeech2(pp, mc).to(dev)
    with torch.no_grad():
        lin = model.variance_adaptor.duration_predictor.linear_layer
        lin.weight.normal_(0.0, 0.005)
        lin.bias.fill_(math.log(9.1))
    model.eval().set_compute_dtype(torch.bfloat16)
    model.requires_grad_(False)
    torch.manual_seed(1)
    g = Generator(default_config()).eval().fold_weight_norm().to(dev)
    sg = SynthGraphs(model, g, int16_scale=32768.0, warm=1)
    import numpy as np

    for B in (1, 3):
        gen = SyntheticBatches(B, device=dev, seed=11 + B, max_seq_len=mc["max_seq_len"],
                               phone_counts=np.array([14, 14]))
        batches = [gen.make_batch() for _ in range(4)]
        r = batches[0]  # one reference mel (fixed shape), different texts
        for k, b in enumerate(batches + batches[:2]):
            args = (b[2], b[3], b[4], b[5], r[6], r[7], r[8])
            wav, lens = sg(*args)
            rows, lens_e, _ = model.infer_packed(*args)
            ref = g.infer_packed(rows, lens_e, int16_scale=32768.0)
            assert lens == lens_e and torch.equal(wav, ref), (B, k)
    assert sg.stats["captures"] >= 2 and sg.stats["replays"] >= 4, sg.stats
