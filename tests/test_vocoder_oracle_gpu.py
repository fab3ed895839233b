"""fp32 oracles for the synthesis (RTF) path on the GPU.

The vocoder's HIP inference path (``Generator._infer_hip``: channel-last bf16, fused ResBlock
layers, 3-tap ConvT GEMMs, fused conv_post/int16) and its HIP training path
(``_forward_hip_train``) share the implicit-GEMM conv kernels, so comparing one against the other
cannot catch a bug they share.  Here the oracle is the plain-PyTorch fp32 NCL forward (reference
``hifigan/models.py:149-165``) with the op backend forced to ``reference`` and the kernel library
made unreachable: the oracle provably runs no ``ssamd_`` kernel.

The end-to-end test runs FastSpeech2 (BC2013: FiLM reference encoder on a reference mel) + HiFi-GAN
to int16 samples on a bench-style synthetic batch -- durations, pitch and energy teacher-forced
from the batch so that both paths regulate to identical lengths and buckets -- HIP bf16 vs fp32."""
import contextlib

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp(min=1e-12)).item()


@contextlib.contextmanager
def torch_fp32_only():
    """Force the torch reference ops and make the HIP kernel library unreachable."""
    from speakingstyle_amd import ops
    from speakingstyle_amd.models import hifigan as H
    from speakingstyle_amd.ops import hip

    saved = (hip.lib, H._hip_train, ops._FORCED)

    def _no_kernels(*a, **k):
        raise AssertionError("an ssamd_ kernel was reached inside the fp32 oracle")

    hip.lib = _no_kernels
    H._hip_train = lambda: False
    ops.set_backend("reference")
    try:
        yield
    finally:
        hip.lib = saved[0]
        H._hip_train = saved[1]
        ops.set_backend(saved[2])


def _generator(seed):
    from speakingstyle_amd.models import hifigan as H

    torch.manual_seed(seed)
    return H.Generator(H.default_config()).eval().fold_weight_norm().to(DEV)


def test_oracle_reaches_no_kernel():
    g = _generator(1)
    mel = torch.randn(1, 80, 8, device=DEV)
    with torch_fp32_only(), torch.no_grad():
        g(mel)  # would raise inside if any op dispatched to the kernel library
    from speakingstyle_amd.ops import hip

    with torch_fp32_only():
        with pytest.raises(AssertionError):
            hip.lib()


@pytest.mark.parametrize("B,T", [(2, 24), (3, 130)])
def test_hifigan_hip_paths_vs_fp32_oracle(B, T):
    """Both HIP generator paths (RTF inference and training forward) vs the fp32 NCL oracle."""
    g = _generator(13 + T)
    mel = torch.randn(B, 80, T, device=DEV) * 2 - 5
    with torch_fp32_only(), torch.no_grad():
        ref_w = g(mel).squeeze(1)
    with torch.no_grad():
        w_inf = g.infer(mel.transpose(1, 2).contiguous().to(torch.bfloat16)).float()
        pcm = g.infer(mel.transpose(1, 2).contiguous().to(torch.bfloat16), int16_scale=32768.0)
        w_tr = g._forward_hip_train(mel).squeeze(1).float()
    assert w_inf.shape == ref_w.shape == (B, T * 256)
    # bf16 operands with fp32 accumulation through ~20 conv layers: a few % relative L2
    assert _rel(w_inf, ref_w) < 5e-2
    assert _rel(w_tr, ref_w) < 5e-2
    assert pcm.dtype == torch.int16
    assert _rel(pcm.float() / 32768.0, ref_w) < 5e-2


def test_bc2013_fs2_vocoder_int16_e2e_vs_fp32_oracle():
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2

    pp, mc, tc = load_named("BC2013")
    torch.manual_seed(0)
    model = FastSpeech2(pp, mc).to(DEV).eval()
    model.requires_grad_(False)
    voc = _generator(5)
    b = SyntheticBatches(4, device=DEV, seed=7).make_batch()
    # (speakers, texts, src_lens, max_src, ref mels, mel_lens, max_mel, pitch, energy, durations)
    args = b[2:12]
    mx = 32768.0

    with torch.no_grad():
        model.set_compute_dtype(torch.bfloat16)
        out = model(*args)
        mel_hip, len_hip = out[1], out[9]
        # the bench's synthesis path: the packed, length-exact vocoder (each utterance vocoded as if alone)
        pcm_hip = voc.infer(mel_hip, int16_scale=mx, lengths=len_hip.tolist())
    lens = len_hip.tolist()
    # fp32 oracle per utterance, alone (the reference's batch-1 synthesis: synthesize.py single mode)
    one = lambda m, i: m[i:i + 1, : lens[i]]  # noqa: E731
    with torch_fp32_only(), torch.no_grad():
        model.set_compute_dtype(torch.float32)
        out_r = model(*args)
        mel_ref, len_ref = out_r[1], out_r[9]
        wav_ref = [voc(one(mel_ref, i).transpose(1, 2)).reshape(-1) for i in range(len(lens))]
        pcm_ref = [(w * mx).clamp(-32768, 32767).to(torch.int16) for w in wav_ref]
        # the FS2 error propagated through the fp32 generator
        wav_prop = [voc(one(mel_hip, i).float().transpose(1, 2)).reshape(-1) for i in range(len(lens))]
    with torch.no_grad():
        wav_voc = [voc.infer(one(mel_ref, i).to(torch.bfloat16).contiguous()).float().reshape(-1)
                   for i in range(len(lens))]
    assert torch.equal(len_hip.cpu(), len_ref.cpu())
    assert pcm_hip.shape == (len(lens), mel_hip.shape[1] * 256)
    # Error budget per utterance (relative L2 over its valid samples).  By the triangle inequality
    #   e_total = |pcm_hip - pcm_ref| <= e_voc + e_prop + e_q (+ the vocoder's error difference between
    #   its two inputs, second order), with
    #   e_fs2  = FS2 bf16 vs fp32 mel: bf16 operands / fp32 accumulation, <= 3e-2 (model-step budget);
    #   e_voc  = HIP bf16 vocoder vs fp32 oracle on the SAME (oracle) mel, <= 5e-2 (generator-only test);
    #   e_prop = fp32 generator on the HIP mel vs on the oracle mel: the FS2 error through the generator;
    #            on these inputs the generator's relative gain e_prop / e_fs2 is ~1-2;
    #   e_q    = int16 quantisation of both sides, 2 x 0.5 LSB / RMS(wav) -- negligible at these levels.
    # The 8e-2 acceptance bound is e_voc's 5e-2 plus a 3e-2 allowance for e_prop + e_q; each term is
    # also checked on its own so a regression names its stage.
    hop = 256
    mel_err = _rel(mel_hip, mel_ref)
    assert mel_err < 3e-2
    report = []
    for i, n in enumerate(len_ref.tolist()):
        a = pcm_hip[i, : n * hop].float()
        r = pcm_ref[i].float()
        assert not pcm_hip[i, n * hop:].any()  # past its length: zero
        e_total = _rel(a, r)
        e_voc = _rel(wav_voc[i], wav_ref[i])
        e_prop = _rel(wav_prop[i], wav_ref[i])
        rms = wav_ref[i].float().pow(2).mean().sqrt().item()
        e_q = (2 * 0.5 / mx) / max(rms, 1e-12) / (12 ** 0.5)
        report.append((round(e_total, 4), round(e_voc, 4), round(e_prop, 4), round(e_q, 6)))
        assert e_voc < 5e-2, report
        assert e_prop < 3e-2 and e_q < 1e-2, report
        assert e_total <= 1.05 * (e_voc + e_prop + e_q) + 1e-3, report
        assert e_total < 8e-2, report


def test_packed_vocoding_equals_each_utterance_alone():
    """The packed, length-exact vocoder (``Generator.infer_packed``: all utterances' rows back to back, every conv
    zero-padding at its own utterance's ends through row / tile tables) against each utterance vocoded ALONE on the
    padded HIP path (B = 1, no lengths): the same samples up to fp32 summation order (the GEMM stages may pick a
    different tile / split-K variant for the smaller M; the tiled ResBlock kernels start their tiles at each
    utterance's row 0 in both) -- and zeros past each length; plus the fp32 oracle per utterance."""
    from speakingstyle_amd.models import hifigan as H

    g = _generator(9)
    assert g.packable()
    lengths = [300, 41, 170, 90, 260, 12, 1, 333]
    B, T = len(lengths), max(lengths) + 7
    torch.manual_seed(5)
    mel = torch.randn(B, T, 80, device=DEV) * 2 - 5  # fp32 in: packed to bf16 rows by the pack kernel
    with torch.no_grad():
        pk = g.infer(mel, int16_scale=32768.0, lengths=lengths)
        pkf = g.infer_packed(mel, lengths)
        assert pk.shape == (B, T * 256) and pk.dtype == torch.int16 and pkf.shape == (B, max(lengths) * 256)
        for i, n in enumerate(lengths):
            alone = g.infer(mel[i:i + 1, :n].to(torch.bfloat16).contiguous(), int16_scale=32768.0)[0]
            assert _rel(pk[i, : n * 256], alone) < 1e-2, (i, _rel(pk[i, : n * 256], alone))
            assert not pk[i, n * 256:].any()
            alone_f = g.infer(mel[i:i + 1, :n].to(torch.bfloat16).contiguous())[0]
            assert _rel(pkf[i, : n * 256], alone_f) < 1e-2, (i, _rel(pkf[i, : n * 256], alone_f))
    with torch_fp32_only(), torch.no_grad():
        refs = [g(mel[i:i + 1, :n].transpose(1, 2)).reshape(-1) for i, n in enumerate(lengths)]
    for i, n in enumerate(lengths):
        if n >= 8:
            assert _rel(pkf[i, : n * 256], refs[i]) < 5e-2, (i, _rel(pkf[i, : n * 256], refs[i]))
    # the bucketed path stays available (reference padded-batch semantics) behind the switch
    assert H._PACKED[0]


def test_packed_resblock_tile_modes_bitwise():
    """The per-layer ResBlock kernel's three packed tile heights (tall, 128-row, 64-row: hip.rb_layer_tile picks one
    from the tile count) compute every output row with the same tap / chunk order: a batch-1 utterance vocoded with
    each forced mode is bitwise the same."""
    from speakingstyle_amd.ops import hip

    g = _generator(10)
    torch.manual_seed(6)
    mel = torch.randn(1, 113, 80, device=DEV) * 2 - 5
    outs, modes = [], []
    saved = (hip._SMALL_MAX_TILES[0], hip._TALL_MIN_TILES[0])
    try:
        for small, tall in ((1 << 30, 1 << 30), (0, 1 << 30), (0, 0)):  # 64-row, 128-row, tall where instantiated
            hip._SMALL_MAX_TILES[0], hip._TALL_MIN_TILES[0] = small, tall
            modes.append(hip.rb_layer_tile(128, 7, [113], 64)[0])
            with torch.no_grad():
                outs.append(g.infer_packed(mel, [113]))
    finally:
        hip._SMALL_MAX_TILES[0], hip._TALL_MIN_TILES[0] = saved
    assert modes == [-1, 0, 1], modes
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])


def test_packed_whole_resblock_short_tile_bitwise():
    """The whole-ResBlock kernel's short tile (RF S = 1, picked by hip.rf_tile for tile-poor packed batches) and its
    regular tile recompute each tile's halo from the same inputs in the same order: a batch-1 utterance is bitwise
    the same either way, and both agree with the utterance's fp32 oracle."""
    from speakingstyle_amd.ops import hip

    g = _generator(11)
    torch.manual_seed(7)
    mel = torch.randn(1, 113, 80, device=DEV) * 2 - 5
    saved = hip._RF_SHORT_MAX_TILES[0]
    outs, picks = [], []
    try:
        for v in (1 << 30, 0):
            hip._RF_SHORT_MAX_TILES[0] = v
            picks.append(hip.rf_tile(64, 7, (1, 3, 5), [113], 128)[0])
            with torch.no_grad():
                outs.append(g.infer_packed(mel, [113]))
    finally:
        hip._RF_SHORT_MAX_TILES[0] = saved
    assert picks == [True, False], picks
    assert torch.equal(outs[0], outs[1])
    with torch_fp32_only(), torch.no_grad():
        ref = g(mel.transpose(1, 2)).reshape(-1)
    assert _rel(outs[0][0], ref) < 5e-2


def test_bucketed_vocoding_matches_padded_batch():
    """Length buckets (each group truncated at max_len + receptive radius) vs the padded batch on
    the same HIP kernels: the valid samples agree (the GEMMs are row-independent; only a different
    tile / split choice for the smaller M may reorder fp32 sums)."""
    from speakingstyle_amd.models import hifigan as H

    g = _generator(3)
    lengths = [300, 41, 170, 90, 260, 12]
    B, T = len(lengths), max(lengths)
    torch.manual_seed(4)
    mel = (torch.randn(B, T, 80, device=DEV) * 2 - 5).to(torch.bfloat16)
    with torch.no_grad():
        pad = g.infer(mel, int16_scale=32768.0)
        H._PACKED[0] = False  # the bucketed path (packed vocoding has per-utterance semantics instead)
        try:
            buck = g.infer(mel, int16_scale=32768.0, lengths=lengths, max_buckets=4, bucket_cost=0)
        finally:
            H._PACKED[0] = True
    assert len(g.length_buckets(lengths, T, g.receptive_radius(), 4, 0)) == 4
    assert buck.shape == pad.shape and buck.dtype == torch.int16
    for i, n in enumerate(lengths):
        a, r = buck[i, : n * 256].float(), pad[i, : n * 256].float()
        assert _rel(a, r) < 1e-2, (i, _rel(a, r))


def test_fs2_long_form_eval_vs_fp32_oracle():
    """Long-form synthesis: eval-mode FastSpeech2 on utterances past max_seq_len = 1000 frames (the
    reference regenerates the positional table in eval, ``transformer/Models.py:82-87,145-152``): the
    HIP bf16 path (decoder attention over ~1.8k frames, PE rows generated past the table) vs the fp32
    torch oracle, mel and PostNet output over the valid frames."""
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2

    pp, mc, tc = load_named("LJSpeech")
    torch.manual_seed(2)
    model = FastSpeech2(pp, mc).to(DEV).eval()
    model.requires_grad_(False)
    T = torch.tensor([80, 61], device=DEV)
    Tm = int(T.max())
    g = torch.Generator(device="cpu").manual_seed(3)
    texts = torch.randint(1, 360, (2, Tm), generator=g).to(DEV)
    texts[1, 61:] = 0
    dur = torch.randint(15, 30, (2, Tm), generator=g).to(DEV)
    dur[1, 61:] = 0
    mel_lens = dur.sum(1)
    M = int(mel_lens.max())
    assert M > 1000 and int(mel_lens.min()) > 1000
    pit = torch.randn(2, Tm, generator=g).to(DEV)
    ene = torch.randn(2, Tm, generator=g).to(DEV)
    spk = torch.zeros(2, dtype=torch.long, device=DEV)
    args = (spk, texts, T, Tm, None, mel_lens, M, pit, ene, dur)
    with torch.no_grad():
        model.set_compute_dtype(torch.bfloat16)
        out = model(*args)
    with torch_fp32_only(), torch.no_grad():
        model.set_compute_dtype(torch.float32)
        out_r = model(*args)
    assert out[1].shape[1] == out_r[1].shape[1] == M
    for i, n in enumerate(mel_lens.tolist()):
        assert _rel(out[0][i, :n], out_r[0][i, :n]) < 3e-2
        assert _rel(out[1][i, :n], out_r[1][i, :n]) < 3e-2
