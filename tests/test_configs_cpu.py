"""Every shipped config: key-by-key parity with the reference YAMLs, model construction and one
forward / backward on the CPU reference ops.

Reference: ``config/{LJSpeech,LJSpeech_paper,LibriTTS,AISHELL3,BC2013}/*.yaml``.  Allowed differences
are the machine-specific paths (the reference's point at its authors' cluster), the ``gst:`` block
(the reference ships it commented out, ``config/BC2013/model.yaml:33-39``), the ``mi355x:`` block and
``ignore_layers`` (added by this framework).  Where the reference config has unnormalised features
(LJSpeech_paper: frame-level Hz pitch with log bins) the model is built against a positive-stats
fixture, as its preprocessor would write it."""
import json
import os

import pytest
import torch
import yaml

from speakingstyle_amd.config import config_dir_triplet, load_configs, load_yaml

REF = "/root/reference/config"
REF_NAMES = ["LJSpeech", "LJSpeech_paper", "LibriTTS", "AISHELL3", "BC2013"]
ALL_NAMES = REF_NAMES + ["BC2013_GST"]


def _flat(d, p=""):
    out = {}
    if isinstance(d, dict):
        for k, v in d.items():
            out.update(_flat(v, f"{p}.{k}" if p else str(k)))
    else:
        out[p] = d
    return out


def _allowed(fname, key):
    if key.startswith("mi355x.") or key == "ignore_layers":
        return True
    if fname == "model" and key.startswith("gst."):
        return True
    if key.startswith("path.") and key != "path.lexicon_path":
        return True
    return False


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
@pytest.mark.parametrize("name", REF_NAMES)
def test_config_matches_reference(name):
    ours = config_dir_triplet(name)
    diffs = []
    for fname, path in zip(("preprocess", "model", "train"), ours):
        r = _flat(yaml.safe_load(open(os.path.join(REF, name, fname + ".yaml"))))
        o = _flat(load_yaml(path))
        for k in sorted(set(r) | set(o)):
            if r.get(k, "<absent>") != o.get(k, "<absent>") and not _allowed(fname, k):
                diffs.append(f"{fname}: {k}: reference={r.get(k, '<absent>')!r} ours={o.get(k, '<absent>')!r}")
    assert not diffs, "\n".join(diffs)


def _positive_stats(tmp_path):
    d = tmp_path / "pp"
    d.mkdir()
    # preprocessor.py output for unnormalised features: [min, max, mean, std] in Hz / energy units
    (d / "stats.json").write_text(json.dumps({"pitch": [71.0, 795.8, 207.6, 53.3],
                                              "energy": [0.017, 314.96, 21.7, 19.2]}))
    return str(d)


@pytest.mark.parametrize("name", ALL_NAMES)
def test_config_builds_and_steps(name, tmp_path, request):
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.models.loss import FastSpeech2Loss
    from speakingstyle_amd.ops import set_backend

    pp, mc, tc = load_configs(*config_dir_triplet(name))
    pcfg = pp["preprocessing"]
    norm = pcfg["pitch"]["normalization"]
    if not norm:
        pp["path"]["preprocessed_path"] = _positive_stats(tmp_path)
    frame = pcfg["pitch"]["feature"] == "frame_level"
    assert frame == (pcfg["energy"]["feature"] == "frame_level")
    n_spk = 3 if mc["multi_speaker"] else 1
    set_backend("reference")
    request.addfinalizer(lambda: set_backend(None))
    torch.manual_seed(0)
    model = FastSpeech2(pp, mc)
    if mc["multi_speaker"]:
        assert model.speaker_emb.num_embeddings > 1
    gen = SyntheticBatches(2, n_speakers=n_spk, max_seq_len=120, frames_per_phone=3.0, frame_level=frame, seed=0,
                           pitch_range=(-2.9, 11.4) if norm else (80.0, 400.0),
                           energy_range=(-1.4, 8.2) if norm else (1.0, 100.0))
    batch = gen.make_batch()
    out = model(*batch[2:])
    losses = FastSpeech2Loss(pp, tc)(batch, out, model.film_scalars())
    total = losses[0]
    assert torch.isfinite(total)
    total.backward()
    n_grad = sum(1 for p in model.parameters() if p.requires_grad and p.grad is not None)
    assert n_grad > 0
    if not norm:  # log pitch bins over Hz
        assert float(model.variance_adaptor.pitch_bins.min()) > 0
