"""Logging / plotting / sample synthesis helpers (reference ``utils/tools.py:82-282``).

TensorBoard tag names are unchanged (``Loss/total_loss`` ... ``Weight/lambda_f``)."""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from .tools import expand


def log_scalars(logger, step=None, losses=None, lr=None, lambdas=None, fig=None, audio=None, sampling_rate=22050, tag=""):
    if logger is None:
        return
    if losses is not None:
        names = ["total_loss", "mel_loss", "mel_postnet_loss", "pitch_loss", "energy_loss", "duration_loss"]
        for n, v in zip(names, losses):
            logger.add_scalar(f"Loss/{n}", float(v), step)
    if lr is not None:
        logger.add_scalar("Weight/learning_rate", float(lr), step)
    if lambdas is not None:
        logger.add_scalar("Weight/lambda_f", float(lambdas), step)
    if fig is not None:
        logger.add_figure(tag, fig)
    if audio is not None:
        a = np.asarray(audio, dtype=np.float32)
        logger.add_audio(tag, a / max(1e-8, float(np.abs(a).max())), sample_rate=sampling_rate)


def _stats(preprocess_config):
    p = os.path.join(preprocess_config["path"]["preprocessed_path"], "stats.json")
    with open(p) as f:
        s = json.load(f)
    return s["pitch"] + s["energy"][:2]


def plot_mel(data, stats, titles):
    import matplotlib

    matplotlib.use("Agg")
    from matplotlib import pyplot as plt

    fig, axes = plt.subplots(len(data), 1, squeeze=False)
    titles = titles or [None] * len(data)
    p_min, p_max, p_mean, p_std, e_min, e_max = stats
    p_max = p_max * p_std + p_mean
    for i, (mel, pitch, energy) in enumerate(data):
        pitch = np.asarray(pitch) * p_std + p_mean
        ax = axes[i][0]
        ax.imshow(mel, origin="lower", aspect="auto")
        ax.set_title(titles[i], fontsize="medium")
        ax.tick_params(labelsize="x-small", left=False, labelleft=False)
        ax1 = fig.add_axes(ax.get_position(), anchor="W")
        ax1.set_facecolor("None")
        ax1.plot(pitch, color="tomato")
        ax1.set_xlim(0, mel.shape[1])
        ax1.set_ylim(0, p_max)
        ax1.tick_params(labelsize="x-small", colors="tomato", bottom=False, labelbottom=False)
        ax2 = fig.add_axes(ax.get_position(), anchor="W")
        ax2.set_facecolor("None")
        ax2.plot(energy, color="darkviolet")
        ax2.set_xlim(0, mel.shape[1])
        ax2.set_ylim(e_min, e_max)
        ax2.tick_params(labelsize="x-small", colors="darkviolet", bottom=False, labelbottom=False, left=False,
                        labelleft=False, right=True, labelright=True)
    return fig


def _feature_curve(values, durations, level):
    return expand(values, durations) if level == "phoneme_level" else values


def synth_one_sample(targets, predictions, vocoder, model_config, preprocess_config, logger=None, step=0, prefix="Training"):
    """GT vs predicted mel plot + vocoded audio of the first utterance (``utils/tools.py:128-180``)."""
    from .model import vocoder_infer

    basename = targets[0][0]
    src_len = int(predictions[8][0])
    mel_len = int(predictions[9][0])
    mel_len = min(mel_len, predictions[1].shape[1])
    mel_target = targets[6][0, :mel_len].detach().float().transpose(0, 1)
    mel_pred = predictions[1][0, :mel_len].detach().float().transpose(0, 1)
    dur = targets[11][0, :src_len].detach().cpu().numpy()
    pp = preprocess_config["preprocessing"]
    pitch = targets[9][0, : (src_len if pp["pitch"]["feature"] == "phoneme_level" else mel_len)].detach().cpu().numpy()
    energy = targets[10][0, : (src_len if pp["energy"]["feature"] == "phoneme_level" else mel_len)].detach().cpu().numpy()
    pitch = _feature_curve(pitch, dur, pp["pitch"]["feature"])
    energy = _feature_curve(energy, dur, pp["energy"]["feature"])
    fig = None
    try:
        fig = plot_mel([(mel_pred.cpu().numpy(), pitch, energy), (mel_target.cpu().numpy(), pitch, energy)],
                       _stats(preprocess_config), ["Synthetized Spectrogram", "Ground-Truth Spectrogram"])
    except (OSError, KeyError):
        pass
    wav_rec = wav_pred = None
    if vocoder is not None:
        wav_rec = vocoder_infer(mel_target.unsqueeze(0), vocoder, model_config, preprocess_config)[0]
        wav_pred = vocoder_infer(mel_pred.unsqueeze(0), vocoder, model_config, preprocess_config)[0]
    if logger is not None:
        tag = f"{prefix}/step_{step}_{basename}"
        if fig is not None:
            log_scalars(logger, fig=fig, tag=tag)
        sr = pp["audio"]["sampling_rate"]
        if wav_rec is not None:
            log_scalars(logger, audio=wav_rec, sampling_rate=sr, tag=tag + "_reconstructed")
            log_scalars(logger, audio=wav_pred, sampling_rate=sr, tag=tag + "_synthesized")
    if fig is not None:
        import matplotlib.pyplot as plt

        plt.close(fig)
    return fig, wav_rec, wav_pred, basename


def synth_samples(targets, predictions, vocoder, model_config, preprocess_config, path, plot=False):
    """Write ``{basename}.wav`` (+ ``.png``) for every utterance (``utils/tools.py:183-230``)."""
    from ..audio.io import write_wav
    from .model import vocoder_infer

    os.makedirs(path, exist_ok=True)
    basenames = targets[0]
    pp = preprocess_config["preprocessing"]
    if plot:
        import matplotlib.pyplot as plt

        stats = _stats(preprocess_config)
        for i in range(len(predictions[0])):
            src_len = int(predictions[8][i])
            mel_len = int(predictions[9][i])
            mel_pred = predictions[1][i, :mel_len].detach().float().transpose(0, 1).cpu().numpy()
            dur = predictions[5][i, :src_len].detach().cpu().numpy()
            pitch = predictions[2][i, : (src_len if pp["pitch"]["feature"] == "phoneme_level" else mel_len)].detach().cpu().numpy()
            energy = predictions[3][i, : (src_len if pp["energy"]["feature"] == "phoneme_level" else mel_len)].detach().cpu().numpy()
            fig = plot_mel([(mel_pred, _feature_curve(pitch, dur, pp["pitch"]["feature"]),
                             _feature_curve(energy, dur, pp["energy"]["feature"]))], stats, ["Synthetized Spectrogram"])
            plt.savefig(os.path.join(path, f"{basenames[i]}.png"))
            plt.close(fig)
    lengths = predictions[9] * pp["stft"]["hop_length"]
    wavs = vocoder_infer(predictions[1].float(), vocoder, model_config, preprocess_config, lengths=lengths,
                         channel_last=True)
    for wav, name in zip(wavs, basenames):
        write_wav(os.path.join(path, f"{name}.wav"), pp["audio"]["sampling_rate"], wav)
    return wavs
