"""HiFi-GAN vocoder side on the CPU: the HiFi-GAN mel framing (reference
``hifigan/meldataset.py:49-72``) against a numpy STFT, the training CLI (synthetic data,
validation + TensorBoard logging, checkpoints, auto-resume), fine-tuning on
ground-truth-aligned mels, and the two inference CLIs (wav -> wav, npy mel -> wav)."""
import json
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _small_cfg(tmp_path):
    from speakingstyle_amd.models.hifigan import default_config

    h = default_config()
    h.update(upsample_initial_channel=32, resblock_kernel_sizes=[3], resblock_dilation_sizes=[[1, 3, 5]],
             segment_size=2048, batch_size=2, num_workers=0)
    p = tmp_path / "config.json"
    p.write_text(json.dumps(dict(h)))
    return str(p), h


def test_hifigan_mel_framing_matches_numpy():
    from speakingstyle_amd.audio.mel import mel_filterbank
    from speakingstyle_amd.models.hifigan import default_config
    from speakingstyle_amd.vocoder.mel import mel_for

    h = default_config()
    rng = np.random.default_rng(0)
    y = (0.5 * rng.standard_normal(8192)).clip(-1, 1).astype(np.float32)
    mel = mel_for(h, torch.from_numpy(y))[0].numpy()
    assert mel.shape == (80, 8192 // 256)  # N / hop frames exactly (uncentred, (n_fft-hop)/2 reflect pad)
    p = (1024 - 256) // 2
    yp = np.pad(y, (p, p), mode="reflect").astype(np.float64)
    win = np.hanning(1025)[:-1]  # periodic hann
    basis = mel_filterbank(22050, 1024, 80, 0, 8000)
    for k in (0, 7, 31):
        X = np.fft.rfft(yp[k * 256:k * 256 + 1024] * win)
        m = np.log(np.maximum(basis @ np.sqrt(np.abs(X) ** 2 + 1e-9), 1e-5))
        np.testing.assert_allclose(mel[:, k], m, rtol=1e-3, atol=2e-3)


def _run(args, env_extra=None):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.update(env_extra or {})
    r = subprocess.run([sys.executable] + args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_train_validate_resume(tmp_path):
    cfg, _ = _small_cfg(tmp_path)
    ck = tmp_path / "ck"
    base = ["hifigan_train.py", "--synthetic", "--cpu", "--config", cfg, "--checkpoint_path", str(ck),
            "--checkpoint_interval", "1", "--validation_interval", "1", "--summary_interval", "1",
            "--stdout_interval", "1", "--num_workers", "0"]
    out = _run(base + ["--training_steps", "2"])
    assert "Steps : 1," in out
    assert (ck / "g_00000001").exists() and (ck / "do_00000001").exists()
    assert (ck / "config.json").exists()
    from speakingstyle_amd.utils.tb import read_scalars

    logs = ck / "logs"
    tags = {t for f in os.listdir(logs) if f.startswith("events") for _, t, _ in read_scalars(str(logs / f))}
    assert {"training/gen_loss_total", "training/mel_spec_error", "validation/mel_spec_error"} <= tags
    assert any(f.startswith("generated_y_hat") for f in os.listdir(logs))
    # auto-resume: continues from the saved step (do_00000001 -> step 2), no restart at 0
    out2 = _run(base + ["--training_steps", "4"])
    assert "Steps : 2," in out2 and "Steps : 0," not in out2
    blob = torch.load(ck / "do_00000003", weights_only=True)
    assert blob["steps"] == 3


def _corpus(tmp_path, h, n=3):
    from speakingstyle_amd.audio.io import write_wav

    wavs, mels = tmp_path / "wavs", tmp_path / "mels"
    wavs.mkdir()
    mels.mkdir()
    rng = np.random.default_rng(1)
    names = []
    for i in range(n):
        L = h.segment_size + 256 * (i + 2)
        t = np.arange(L) / h.sampling_rate
        w = (0.4 * np.sin(2 * np.pi * (150 + 40 * i) * t) + 0.02 * rng.standard_normal(L)).astype(np.float32)
        write_wav(str(wavs / f"utt{i}.wav"), h.sampling_rate, (w * 32767).astype(np.int16))
        np.save(mels / f"utt{i}.npy", rng.standard_normal((80, L // 256)).astype(np.float32) - 4)
        names.append(f"utt{i}")
    (tmp_path / "train.txt").write_text("\n".join(f"{n}|x" for n in names[:2]) + "\n")
    (tmp_path / "val.txt").write_text(f"{names[2]}|x\n")
    return wavs, mels, names


def test_fine_tuning_on_aligned_mels_and_inference_clis(tmp_path):
    cfg, h = _small_cfg(tmp_path)
    wavs, mels, names = _corpus(tmp_path, h)
    ck = tmp_path / "ck"
    _run(["hifigan_train.py", "--cpu", "--config", cfg, "--checkpoint_path", str(ck), "--input_wavs_dir", str(wavs),
          "--input_mels_dir", str(mels), "--input_training_file", str(tmp_path / "train.txt"),
          "--input_validation_file", str(tmp_path / "val.txt"), "--fine_tuning", "True", "--training_steps", "2",
          "--checkpoint_interval", "1", "--validation_interval", "1", "--num_workers", "0"])
    g = ck / "g_00000001"
    assert g.exists()
    # data pipeline of the fine-tuning mode: the audio crop follows the mel crop
    from speakingstyle_amd.vocoder.data import MelDataset, read_filelist

    ds = MelDataset(read_filelist(str(tmp_path / "train.txt"), str(wavs)), h, fine_tuning=True,
                    base_mels_path=str(mels))
    mel, audio, _, loss_mel = ds[0]
    assert mel.shape == (80, h.segment_size // 256) and audio.shape == (h.segment_size,)
    assert loss_mel.shape == (80, h.segment_size // 256)
    out = _run(["hifigan_inference.py", "--checkpoint_file", str(g), "--input_wavs_dir", str(wavs),
                "--output_dir", str(tmp_path / "gen")])
    assert len([l for l in out.splitlines() if l.endswith("_generated.wav")]) == len(names)
    out = _run(["hifigan_inference_e2e.py", "--checkpoint_file", str(g), "--input_mels_dir", str(mels),
                "--output_dir", str(tmp_path / "gen_e2e")])
    files = sorted(os.listdir(tmp_path / "gen_e2e"))
    assert files == [f"{n}_generated_e2e.wav" for n in names]
    from speakingstyle_amd.audio.io import read_wav

    w, sr = read_wav(str(tmp_path / "gen_e2e" / files[1]))
    assert sr == h.sampling_rate and len(w) == np.load(mels / "utt1.npy").shape[1] * 256
