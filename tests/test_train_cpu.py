"""CPU plumbing (BASELINE config #1): tiny FastSpeech2 trains through the real
CLI on synthetic data, checkpoints, resumes with weights restored (the
reference's resume silently drops the weights), evaluates, synthesizes."""
import copy
import os
import subprocess
import sys

import pytest
import torch
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tiny_configs(tmp_path, name="LJSpeech", style=None):
    from speakingstyle_amd.config import config_dir_triplet, load_yaml

    p, m, t = (load_yaml(x) for x in config_dir_triplet(name))
    p["path"]["preprocessed_path"] = os.path.join(ROOT, "preprocessed_data", "LJSpeech")
    m["transformer"].update(encoder_layer=1, decoder_layer=1, conv_filter_size=64, encoder_hidden=32, decoder_hidden=32,
                            encoder_head=2, decoder_head=2)
    m["variance_predictor"]["filter_size"] = 32
    if style == "film":
        m["reference_encoder"] = {"encoder_layer": 1, "encoder_head": 2, "encoder_hidden": 32, "conv_layer": 1,
                                  "conv_filter_size": 32, "conv_kernel_size": 3, "dropout": 0.1}
        t["loss"] = {"lambda_f": 0.001, "anneal_steps": 10}
        t["optimizer"].update(init_lr=1e-4, anneal_lr=1e-3)
    if style == "gst":
        m["gst"] = {"use_gst": True, "conv_filters": [4, 4, 8, 8, 16, 16], "gru_hidden": 16, "token_size": 16,
                    "n_style_token": 4, "attn_head": 2}
        t["loss"] = {"lambda_f": 0.001, "anneal_steps": 10}
    t["optimizer"]["batch_size"] = 3
    t["step"].update(total_step=4, log_step=2, synth_step=1000, val_step=1000, save_step=2)
    for k in ("ckpt_path", "log_path", "result_path"):
        t["path"][k] = str(tmp_path / k)
    paths = []
    for nm, obj in (("preprocess", p), ("model", m), ("train", t)):
        f = tmp_path / f"{nm}.yaml"
        f.write_text(yaml.safe_dump(obj))
        paths.append(str(f))
    return paths


def _run(args, cwd=ROOT, env_extra=None):
    env = dict(os.environ)
    env.update(env_extra or {})
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable] + args, cwd=cwd, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.mark.parametrize("style", [None, "film", "gst"])
def test_train_save_resume(tmp_path, style):
    p, m, t = _tiny_configs(tmp_path, style=style)
    out = _run(["train.py", "-p", p, "-m", m, "-t", t, "--synthetic", "--cpu", "--no_vocoder"])
    assert "Step 4/4" in out
    ck = tmp_path / "ckpt_path" / "4.pth.tar"
    assert ck.exists()
    blob = torch.load(ck, weights_only=True)
    assert set(blob) >= {"model", "optimizer"}
    # resume: weights must be the checkpoint's, LR schedule continues from step 4
    from speakingstyle_amd.config import load_configs
    from speakingstyle_amd.utils.model import get_model

    configs = load_configs(p, m, t)
    model, opt = get_model(4, configs, "cpu", train=True)
    for k, v in blob["model"].items():
        torch.testing.assert_close(model.state_dict()[k].float(), v.float())
    assert opt.current_step == 4 and opt.step_count == blob["optimizer"]["state"][next(iter(blob["optimizer"]["state"]))]["step"]
    out2 = _run(["train.py", "-p", p, "-m", m, "-t", t, "--synthetic", "--cpu", "--no_vocoder", "--restore_step", "4",
                 "--max_steps", "6"])
    assert "Step 6/6" in out2
    # TensorBoard events written with the reference tag names
    from speakingstyle_amd.utils.tb import read_scalars

    ev = [f for f in os.listdir(tmp_path / "log_path" / "train") if f.startswith("events")]
    tags = {tg for f in ev for _, tg, _ in read_scalars(str(tmp_path / "log_path" / "train" / f))}
    assert {"Loss/total_loss", "Loss/mel_loss", "Weight/learning_rate"} <= tags


def _losses(out):
    return {int(l.split("Step ")[1].split("/")[0]): l.split(", ", 1)[1] for l in out.splitlines()
            if l.startswith("Step ")}


def test_synthetic_resume_is_exact(tmp_path):
    """The synthetic stream honours the checkpoint's data position: resuming at step 4 logs the same
    step-6 losses as the uninterrupted run (weights, Adam state, LR schedule, dropout RNG and data)."""
    p, m, t = _tiny_configs(tmp_path)
    full = _losses(_run(["train.py", "-p", p, "-m", m, "-t", t, "--synthetic", "--cpu", "--no_vocoder",
                         "--max_steps", "6"]))
    res = _losses(_run(["train.py", "-p", p, "-m", m, "-t", t, "--synthetic", "--cpu", "--no_vocoder",
                        "--restore_step", "4", "--max_steps", "6"]))
    assert 6 in full and res[6] == full[6], (full, res)


def test_sigterm_checkpoint_and_fault_injection(tmp_path):
    p, m, t = _tiny_configs(tmp_path)
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "train.py", "-p", p, "-m", m, "-t", t, "--synthetic", "--cpu", "--no_vocoder",
                        "--fail_at_step", "3"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode != 0 and "fault injection at step 3" in r.stderr
    assert (tmp_path / "ckpt_path" / "2.pth.tar").exists()
    out = _run(["train.py", "-p", p, "-m", m, "-t", t, "--synthetic", "--cpu", "--no_vocoder", "--auto_resume"])
    assert "Step 4/4" in out


def test_sigterm_saves_at_step_boundary(tmp_path):
    """SIGTERM sets a flag; the loop saves at the next step boundary (with the data
    position) and exits 0 -- no exception from inside a step or a collective."""
    import signal
    import time

    p, m, t = _tiny_configs(tmp_path)
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", PYTHONUNBUFFERED="1")
    proc = subprocess.Popen([sys.executable, "train.py", "-p", p, "-m", m, "-t", t, "--synthetic", "--cpu",
                             "--no_vocoder", "--max_steps", "100000"], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE, text=True)
    try:
        deadline = time.time() + 600
        for line in proc.stdout:
            if line.startswith("Step 2/"):
                break
            assert time.time() < deadline
        proc.send_signal(signal.SIGTERM)
        out, err = proc.communicate(timeout=300)
    finally:
        if proc.poll() is None:
            proc.kill()
    assert proc.returncode == 0, err[-3000:]
    assert "SIGTERM: checkpoint saved at step" in out
    step = int(out.split("SIGTERM: checkpoint saved at step")[1].split()[0])
    blob = torch.load(tmp_path / "ckpt_path" / f"{step}.pth.tar", weights_only=True)
    assert blob["step"] == step and len(blob["data_pos"]) == 3


def test_synthesize_single_cli(tmp_path):
    p, m, t = _tiny_configs(tmp_path, style="gst")
    _run(["train.py", "-p", p, "-m", m, "-t", t, "--synthetic", "--cpu", "--no_vocoder", "--max_steps", "2"])
    out = _run(["synthesize.py", "--mode", "single", "--text", "Hello world, this is a test.", "--restore_step", "2",
                "-p", p, "-m", m, "-t", t, "--word_pitch", "1.0,1.5,1,1,0.5,1", "--style_weights", "0.5,0.2,0.2,0.1",
                "--duration_control", "1.2"])
    res = tmp_path / "result_path"
    wavs = [f for f in os.listdir(res) if f.endswith(".wav")]
    assert wavs, out
