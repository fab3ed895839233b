"""External speaker embeddings (reference ``synthesize.py:268-277``): with
``preprocessing.speaker_embedder != 'none'`` AND the opt-in ``speaker_embed_proj: true`` the per-speaker
``spker_embed/{spk}-spker_embed.npy`` vectors are loaded into a table and condition the encoder output
next to the speaker-id embedding; without the flag the model keeps the reference layout (the
reference loads the vectors and drops them)."""
import json
import os

import numpy as np
import torch


def _cfg(tmp_path, embedder, proj=True):
    from speakingstyle_amd.config import load_named

    pp, mc, tc = load_named("LJSpeech")
    root = tmp_path / "pre"
    (root / "spker_embed").mkdir(parents=True)
    spk = {"alice": 0, "bob": 1, "carol": 2}
    (root / "speakers.json").write_text(json.dumps(spk))
    rng = np.random.default_rng(0)
    for name in spk:
        np.save(root / "spker_embed" / f"{name}-spker_embed.npy", rng.standard_normal(16).astype(np.float32))
    pp["path"]["preprocessed_path"] = str(root)
    pp["preprocessing"]["speaker_embedder"] = embedder
    mc["multi_speaker"] = True
    mc["speaker_embed_proj"] = proj
    mc["transformer"].update(encoder_layer=1, decoder_layer=1, conv_filter_size=64, encoder_hidden=32,
                             decoder_hidden=32, encoder_head=2, decoder_head=2)
    mc["variance_predictor"]["filter_size"] = 32
    return pp, mc, tc


def test_speaker_embedder_table_conditions_model(tmp_path):
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2

    pp, mc, tc = _cfg(tmp_path, "DeepSpeaker")
    torch.manual_seed(0)
    m = FastSpeech2(pp, mc)
    assert m.spker_table.shape == (3, 16) and m.spker_embed_proj.in_features == 16
    assert "spker_table" not in m.state_dict()  # non-persistent: checkpoints carry only the projection
    v = np.load(os.path.join(pp["path"]["preprocessed_path"], "spker_embed", "bob-spker_embed.npy"))
    torch.testing.assert_close(m.spker_table[1], torch.from_numpy(v))
    b = SyntheticBatches(3, n_speakers=3, seed=1, phone_counts=[9, 12, 7]).make_batch()
    out = m(*b[2:])
    out[1].float().abs().mean().backward()
    assert m.spker_embed_proj.weight.grad is not None and m.spker_embed_proj.weight.grad.abs().sum() > 0
    # a different speaker id changes the output through the table as well
    m.eval()
    with torch.no_grad():
        spk = b[2].clone()
        o1 = m(spk, *b[3:6])[0]
        m.speaker_emb.weight.zero_()
        o2 = m((spk + 1) % 3, *b[3:6])[0]
        o3 = m(spk, *b[3:6])[0]
    assert o2.shape != o3.shape or not torch.allclose(o2, o3)
    assert o1.shape[0] == o3.shape[0] == 3


def test_no_embedder_keeps_reference_layout(tmp_path):
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2

    pp, mc, tc = _cfg(tmp_path, "none")
    m = FastSpeech2(pp, mc)
    assert m.spker_embed_proj is None and not any("spker" in k for k in m.state_dict())


def test_embedder_without_opt_in_keeps_reference_layout(tmp_path):
    """speaker_embedder alone (reference configs): no projection, reference state-dict keys."""
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2

    pp, mc, tc = _cfg(tmp_path, "DeepSpeaker", proj=False)
    m = FastSpeech2(pp, mc)
    assert m.spker_embed_proj is None and not any("spker" in k for k in m.state_dict())
