"""Offline pipeline on a tiny generated corpus: prepare_align -> (fake MFA TextGrids)
-> Preprocessor.build_from_path -> Dataset/collate -> a real-data training step."""
import json
import os
import sys

import numpy as np
import pytest
import torch
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PHONES = ["HH", "AH0", "L", "OW1", "W", "ER1", "L", "D"]


def _textgrid(path, phones, dur_s):
    t = 0.2
    ivs = [(0.0, 0.2, "sil")]
    for p in phones:
        ivs.append((t, t + dur_s, p))
        t += dur_s
    ivs.append((t, t + 0.1, "sp"))
    xmax = t + 0.1
    lines = ['File type = "ooTextFile"', 'Object class = "TextGrid"', "", "xmin = 0", f"xmax = {xmax}", "tiers? <exists>",
             "size = 1", "item []:", "    item [1]:", '        class = "IntervalTier"', '        name = "phones"',
             "        xmin = 0", f"        xmax = {xmax}", f"        intervals: size = {len(ivs)}"]
    for i, (a, b, p) in enumerate(ivs, 1):
        lines += [f"        intervals [{i}]:", f"            xmin = {a}", f"            xmax = {b}", f'            text = "{p}"']
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return xmax


@pytest.fixture(scope="module")
def corpus(tmp_path_factory):
    from speakingstyle_amd.audio.io import write_wav

    root = tmp_path_factory.mktemp("corpus")
    corpus = root / "LJ"
    (corpus / "wavs").mkdir(parents=True)
    sr = 22050
    meta = []
    for i in range(12):
        dur = 0.2 + 8 * 0.09 + 0.1
        t = np.arange(int(sr * (dur + 0.05))) / sr
        f0 = 110 + 10 * i
        wav = 0.4 * np.sin(2 * np.pi * f0 * t) * (1 + 0.3 * np.sin(2 * np.pi * 3 * t))
        write_wav(str(corpus / "wavs" / f"LJ{i:03d}.wav"), sr, (wav * 32767).astype(np.int16))
        meta.append(f"LJ{i:03d}|Hello world {i}.|Hello world {i}.")
    (corpus / "metadata.csv").write_text("\n".join(meta) + "\n")
    from speakingstyle_amd.config import config_dir_triplet, load_yaml

    p = load_yaml(config_dir_triplet("LJSpeech")[0])
    p["path"].update(corpus_path=str(corpus), raw_path=str(root / "raw"), preprocessed_path=str(root / "pre"))
    p["preprocessing"]["val_size"] = 2
    pf = root / "preprocess.yaml"
    pf.write_text(yaml.safe_dump(p))
    return root, pf, p


def test_prepare_and_preprocess(corpus):
    root, pf, p = corpus
    import importlib.util

    def _load(name):  # by path: the session-scoped reference fixture may shadow same-named top-level modules
        spec = importlib.util.spec_from_file_location("ssamd_cli_" + name, os.path.join(ROOT, name + ".py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        return mod

    prepare_align = _load("prepare_align")
    preprocess = _load("preprocess")

    assert prepare_align.main([str(pf)]) == 12
    assert (root / "raw" / "LJSpeech" / "LJ000.lab").read_text().startswith("hello world")
    for i in range(12):
        d = root / "pre" / "TextGrid" / "LJSpeech"
        d.mkdir(parents=True, exist_ok=True)
        _textgrid(str(d / f"LJ{i:03d}.TextGrid"), PHONES, 0.09)
    out = preprocess.main(["--preprocess_config", str(pf), "--workers", "1"])
    assert len(out) == 12
    stats = json.load(open(root / "pre" / "stats.json"))
    assert len(stats["pitch"]) == 4 and stats["pitch"][0] < stats["pitch"][1]
    assert json.load(open(root / "pre" / "speakers.json")) == {"LJSpeech": 0}
    lines = (root / "pre" / "train.txt").read_text().strip().split("\n")
    assert len(lines) == 10
    base = lines[0].split("|")[0]
    dur = np.load(root / "pre" / "duration" / f"LJSpeech-duration-{base}.npy")
    mel = np.load(root / "pre" / "mel" / f"LJSpeech-mel-{base}.npy")
    pitch = np.load(root / "pre" / "pitch" / f"LJSpeech-pitch-{base}.npy")
    assert len(dur) == 8 and mel.shape == (dur.sum(), 80) and pitch.shape == (8,)


def test_dataset_and_real_data_step(corpus):
    root, pf, p = corpus
    if not (root / "pre" / "train.txt").exists():  # run alone / on another xdist worker than the preprocess test
        test_prepare_and_preprocess(corpus)
    from speakingstyle_amd.config import load_configs, load_named
    from speakingstyle_amd.data.dataset import Dataset, to_device
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.train.trainer import Trainer

    pp, mc, tc = load_named("LJSpeech")
    pp = load_configs(str(pf), mc, tc)[0]
    mc["transformer"].update(encoder_layer=1, decoder_layer=1)
    tc["optimizer"]["batch_size"] = 2
    ds = Dataset("train.txt", pp, tc, sort=True, drop_last=True)
    batches = ds.collate_fn([ds[i] for i in range(8)])
    assert len(batches) == 4 and all(len(b) == 12 for b in batches)
    b = to_device(batches[0], "cpu")
    assert b[6].shape[2] == 80 and b[10].dtype == torch.float32
    model = FastSpeech2(pp, mc)
    tr = Trainer(model, (pp, mc, tc))
    losses, _, lr = tr.train_step(b)
    assert torch.isfinite(losses[0])
    sharded = Dataset("train.txt", pp, tc, sort=True, drop_last=True, shard=(1, 2)).collate_fn([ds[i] for i in range(8)])
    assert all(len(x[0]) == 1 for x in sharded)
