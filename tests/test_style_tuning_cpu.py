"""Style-token bank tuning (README research goal of the reference; ``train/style_tuning.py``)."""
import os

import numpy as np
import pytest
import torch
import yaml

from speakingstyle_amd.config import load_named
from speakingstyle_amd.models.fastspeech2 import FastSpeech2
from speakingstyle_amd.train.style_tuning import StyleTokenTuner, parse_label


def _styled_mels(n_per_class, n_classes, rng):
    """Three synthetic 'speaking styles': different spectral tilts + energy levels."""
    mels, labels = [], []
    f = np.linspace(-1, 1, 80, dtype=np.float32)
    for c in range(n_classes):
        for _ in range(n_per_class):
            T = int(rng.integers(60, 140))
            base = -6 + 2.0 * c + (c - 1) * 2.5 * f
            mels.append((base[None, :] + 0.4 * rng.standard_normal((T, 80))).astype(np.float32))
            labels.append(c)
    return mels, labels


def _gst_model(seed=0):
    pp, mc, tc = load_named("BC2013_GST")
    mc["transformer"]["encoder_layer"] = mc["transformer"]["decoder_layer"] = 1
    torch.manual_seed(seed)
    return FastSpeech2(pp, mc).eval(), (pp, mc, tc)


def test_parse_label():
    assert parse_label("2", 4).tolist() == [0, 0, 1, 0]
    np.testing.assert_allclose(parse_label("1,1,0,2", 4), [0.25, 0.25, 0, 0.5])
    with pytest.raises(ValueError):
        parse_label("7", 4)
    with pytest.raises(ValueError):
        parse_label("1,2", 4)


def test_tuner_aligns_tokens_with_annotations():
    model, _ = _gst_model()
    rng = np.random.default_rng(0)
    mels, labels = _styled_mels(6, 3, rng)
    n_tok = model.gst.embed.shape[0]
    targets = np.eye(n_tok, dtype=np.float32)[labels]
    # a random-init encoder yields near-zero, barely separable queries (|q| ~ 0.3); scale the
    # query projection to the magnitude a trained encoder produces
    with torch.no_grad():
        model.gst.w_query.weight.mul_(30.0)
    frozen = model.encoder.src_word_emb.weight.detach().clone()
    tuner = StyleTokenTuner(model, lr=5e-2, steps=150, tune_projections=True)
    res = tuner.fit(mels, targets)
    h = res["history"]
    assert h[-1]["ce"] < 0.5 * h[0]["ce"]
    assert res["accuracy"] == 1.0
    assert torch.equal(model.encoder.src_word_emb.weight, frozen)  # everything but the bank is frozen
    assert model.gst.embed.grad is None


def test_tune_style_cli(tmp_path):
    import importlib.util

    from speakingstyle_amd.utils.model import load_checkpoint, save_checkpoint

    model, (pp, mc, tc) = _gst_model(1)
    pre = tmp_path / "pre"
    (pre / "mel").mkdir(parents=True)
    rng = np.random.default_rng(1)
    mels, labels = _styled_mels(3, 2, rng)
    lines = []
    for i, (m, c) in enumerate(zip(mels, labels)):
        np.save(pre / "mel" / f"spk-mel-utt{i}.npy", m)
        lines.append(f"utt{i}|spk|{c}" if i % 2 else f"utt{i}|spk|" + ",".join("1" if k == c else "0" for k in range(10)))
    (tmp_path / "ann.txt").write_text("\n".join(lines) + "\n")
    pp["path"]["preprocessed_path"] = str(pre)
    tc["path"]["ckpt_path"] = str(tmp_path / "ckpt")
    save_checkpoint(os.path.join(tc["path"]["ckpt_path"], "5.pth.tar"), model)
    paths = []
    for name, cfg in (("p", pp), ("m", mc), ("t", tc)):
        p = tmp_path / f"{name}.yaml"
        p.write_text(yaml.safe_dump(cfg))
        paths.append(str(p))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("tune_style", os.path.join(root, "tune_style.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.main(["-p", paths[0], "-m", paths[1], "-t", paths[2], "--restore_step", "5", "--annotations",
              str(tmp_path / "ann.txt"), "--steps", "20"])
    before = load_checkpoint(os.path.join(tc["path"]["ckpt_path"], "5.pth.tar"))["model"]
    after = load_checkpoint(os.path.join(tc["path"]["ckpt_path"], "6.pth.tar"))["model"]
    changed = [k for k in before if not torch.equal(before[k], after[k])]
    assert changed == ["gst.embed"]
