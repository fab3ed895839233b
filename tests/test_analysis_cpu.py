"""Notebook tooling as library + CLI (reference notebooks/variance_control_distbn.ipynb,
notebooks/ref_encoder.ipynb) on a small synthetic preprocessed corpus."""
import json
import os
import subprocess
import sys

import numpy as np
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _corpus(tmp_path):
    pre = tmp_path / "pre"
    for k in ("mel", "pitch", "energy", "duration"):
        (pre / k).mkdir(parents=True)
    (pre / "speakers.json").write_text(json.dumps({"LJ": 0}))
    (pre / "stats.json").write_text(json.dumps({"pitch": [-2.0, 8.0, 200.0, 40.0], "energy": [-1.5, 7.0, 30.0, 20.0]}))
    rng = np.random.default_rng(0)
    lines = []
    for i in range(6):
        phones = rng.choice(["HH", "AH0", "L", "OW1", "W", "ER1", "D", "sp"], size=rng.integers(5, 12)).tolist()
        T = len(phones)
        d = rng.integers(1, 9, T)
        base = f"LJ001-{i:04d}"
        np.save(pre / "duration" / f"LJ-duration-{base}.npy", d)
        np.save(pre / "pitch" / f"LJ-pitch-{base}.npy", rng.standard_normal(T).astype(np.float32))
        np.save(pre / "energy" / f"LJ-energy-{base}.npy", rng.standard_normal(T).astype(np.float32))
        np.save(pre / "mel" / f"LJ-mel-{base}.npy", (rng.random((int(d.sum()), 80)) * 10 - 10).astype(np.float32))
        lines.append(f"{base}|LJ|{{{' '.join(phones)}}}|text {i}")
    (pre / "val.txt").write_text("\n".join(lines) + "\n")
    (pre / "train.txt").write_text("\n".join(lines * 3) + "\n")
    return pre


def _configs(tmp_path, pre):
    from speakingstyle_amd.config import config_dir_triplet, load_yaml

    p, m, t = (load_yaml(x) for x in config_dir_triplet("BC2013"))
    p["path"]["preprocessed_path"] = str(pre)
    m["transformer"].update(encoder_layer=1, decoder_layer=1, conv_filter_size=64, encoder_hidden=32,
                            decoder_hidden=32, encoder_head=2, decoder_head=2)
    m["variance_predictor"]["filter_size"] = 32
    m["reference_encoder"].update(encoder_layer=1, encoder_head=2, encoder_hidden=32, conv_layer=1,
                                  conv_filter_size=32)
    m["multi_speaker"] = False
    t["optimizer"]["batch_size"] = 2
    paths = []
    for nm, obj in (("preprocess", p), ("model", m), ("train", t)):
        f = tmp_path / f"{nm}.yaml"
        f.write_text(yaml.safe_dump(obj))
        paths.append(str(f))
    return paths


def test_remove_outlier_and_compare():
    from speakingstyle_amd.analysis.variance import compare, remove_outlier

    v = np.concatenate([np.arange(100.0), [1e6, -1e6]])
    assert remove_outlier(v).size == 100
    same = compare(np.arange(1000.0), np.arange(1000.0))
    assert abs(same["overlap"] - 1.0) < 1e-9 and same["js_bits"] < 1e-12
    far = compare(np.zeros(100), np.ones(100) * 10)
    assert far["overlap"] < 1e-9 and abs(far["js_bits"] - 1.0) < 1e-9


def test_variance_and_inspect_cli(tmp_path):
    pre = _corpus(tmp_path)
    p, m, t = _configs(tmp_path, pre)
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    out_dir = tmp_path / "ana"
    r = subprocess.run([sys.executable, "analyze.py", "variance", "-p", p, "-m", m, "-t", t, "--out_dir", str(out_dir),
                        "--pitch_control", "1.3", "--cpu"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    summ = json.loads((out_dir / "variance_summary.json").read_text())
    n_phones = sum(len(l.split("|")[2].strip("{}").split()) for l in (pre / "val.txt").read_text().splitlines())
    assert summ["pitch"]["n_true"] == n_phones == summ["pitch"]["n_pred"]
    assert abs(summ["pitch"]["mean_true"] - 200.0) < 40.0  # de-normalised with stats.json
    assert (out_dir / "pitch_true_vs_pred.png").exists()
    r = subprocess.run([sys.executable, "analyze.py", "inspect", "-p", p, "-m", m, "-t", t, "--cpu"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rep = json.loads(r.stdout)
    assert rep["source"] == "train.txt" and rep["batch_size"] == 2
    assert rep["outputs"]["mel"][0] == 2 and "style" in rep and len(rep["style"]["gamma_norm_per_utt"]) == 2
    assert np.isfinite(rep["losses"]["total"])
