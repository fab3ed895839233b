"""Model / optimizer / vocoder factories and checkpoint I/O.

Reference: ``utils/model.py:11-115``.  Checkpoint layout is unchanged --
``{ckpt_path}/{step}.pth.tar`` = ``{"model": state_dict, "optimizer": Adam
state_dict}`` (``train.py:155-165``) -- with optional extra keys (``step``,
``rng``) that older loaders ignore.  Fixed: restore now actually loads the model
weights (the reference passes the whole checkpoint dict to
``load_state_dict(strict=False)``) and honours ``ignore_layers`` by
key substring; ``requires_grad_(False)`` for inference (D6); checkpoints are
written atomically (tmp + rename) and loaded with ``weights_only=True``.
"""
from __future__ import annotations

import glob
import json
import os
import re
from typing import Iterable, Optional

import numpy as np
import torch

from ..models.fastspeech2 import FastSpeech2
from ..models.hifigan import AttrDict, Generator, default_config

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ckpt_file(train_config, step: int) -> str:
    return os.path.join(train_config["path"]["ckpt_path"], f"{step}.pth.tar")


def latest_step(train_config) -> int:
    files = glob.glob(os.path.join(train_config["path"]["ckpt_path"], "*.pth.tar"))
    steps = [int(m.group(1)) for f in files if (m := re.match(r"(\d+)\.pth\.tar$", os.path.basename(f)))]
    return max(steps) if steps else 0


def load_checkpoint(path: str, device="cpu"):
    return torch.load(path, map_location=device, weights_only=True)


def save_checkpoint(path: str, model, optimizer=None, step: Optional[int] = None, extra: Optional[dict] = None):
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    sd = {k: v.detach().clone().cpu() for k, v in model.state_dict().items()}
    blob = {"model": sd}
    if optimizer is not None:
        blob["optimizer"] = optimizer.state_dict()
    if step is not None:
        blob["step"] = int(step)
    if extra:
        blob.update(extra)
    tmp = path + ".tmp"
    torch.save(blob, tmp)
    os.replace(tmp, path)
    return path


def filter_ignored(state: dict, ignore_layers: Iterable[str]) -> dict:
    ignore = list(ignore_layers or [])
    return {k: v for k, v in state.items() if not any(s in k for s in ignore)}


def restore_model(model, ckpt: dict, ignore_layers=()):
    state = ckpt.get("model", ckpt)
    state = filter_ignored(state, ignore_layers)
    own = model.state_dict()
    usable = {k: v for k, v in state.items() if k in own and own[k].shape == v.shape}
    missing, unexpected = model.load_state_dict(usable, strict=False)
    skipped = sorted(set(state) - set(usable))
    return missing, skipped


def get_model(restore_step: int, configs, device, train: bool = False, ignore_layers=(), compute_dtype=None):
    """-> model (eval) or (model, ScheduledOptim) when ``train``."""
    preprocess_config, model_config, train_config = configs
    model = FastSpeech2(preprocess_config, model_config).to(device)
    ckpt = None
    if restore_step:
        ckpt = load_checkpoint(ckpt_file(train_config, restore_step), device="cpu")
        restore_model(model, ckpt, ignore_layers)
    if compute_dtype is None:
        compute_dtype = torch.bfloat16 if torch.device(device).type == "cuda" else torch.float32
    model.set_compute_dtype(compute_dtype)
    if train:
        from ..train.optim import ScheduledOptim

        opt = ScheduledOptim(model, train_config, model_config, restore_step)
        if ckpt is not None and "optimizer" in ckpt:
            opt.load_state_dict(ckpt["optimizer"])
        model.train()
        return model, opt
    model.eval()
    model.requires_grad_(False)
    return model


def get_param_num(model) -> int:
    return sum(p.numel() for p in model.parameters())


def get_named_param(model, tags=("s_gamma", "s_beta")):
    ps = [p for n, p in model.named_parameters() if any(t in n for t in tags)]
    return torch.cat([p.reshape(-1) for p in ps]) if ps else torch.zeros(0)


# ------------------------------------------------------------------ vocoder
def vocoder_config(path: Optional[str] = None) -> AttrDict:
    path = path or os.path.join(ROOT, "config", "hifigan", "config.json")
    if os.path.exists(path):
        with open(path) as f:
            return AttrDict(json.load(f))
    return default_config()


def get_vocoder(model_config, device, ckpt_dir: Optional[str] = None, allow_random: bool = True):
    """HiFi-GAN generator; loads ``generator_{LJSpeech,universal}.pth.tar`` when
    present (weights_only), otherwise random init (benchmarks).  MelGAN via
    torch.hub is not supported (network download)."""
    name = model_config["vocoder"]["model"]
    if name != "HiFi-GAN":
        raise ValueError(f"vocoder {name!r} not supported (HiFi-GAN only)")
    speaker = model_config["vocoder"]["speaker"]
    gen = Generator(vocoder_config())
    ckpt_dir = ckpt_dir or os.path.join(ROOT, "hifigan")
    path = os.path.join(ckpt_dir, f"generator_{speaker}.pth.tar")
    if os.path.exists(path):
        ck = load_checkpoint(path)
        gen.load_state_dict(ck["generator"])
    elif not allow_random:
        raise FileNotFoundError(path)
    gen.eval().fold_weight_norm().to(device)
    gen.requires_grad_(False)
    return gen


@torch.no_grad()
def vocoder_infer(mels, vocoder, model_config, preprocess_config, lengths=None, channel_last: bool = False):
    """mels [B, n_mel, T] (reference layout) or [B, T, n_mel] with ``channel_last``
    -> list of int16 numpy wavs trimmed to ``lengths`` samples (``utils/model.py:97-115``)."""
    x = mels if channel_last else mels.transpose(1, 2)
    mx = preprocess_config["preprocessing"]["audio"]["max_wav_value"]
    if x.is_cuda:
        x = x.to(torch.bfloat16).contiguous()
        hop = preprocess_config["preprocessing"]["stft"]["hop_length"]
        frames = None if lengths is None else [-(-int(n) // hop) for n in lengths]
        # int16 written by the conv_post kernel; length-bucketed when the lengths are known
        wavs = vocoder.infer(x, int16_scale=mx, lengths=frames).cpu().numpy()
    else:
        wavs = vocoder(x.transpose(1, 2).float()).squeeze(1)
        wavs = (wavs * mx).clamp(-32768, 32767).cpu().numpy().astype(np.int16)
    out = [w for w in wavs]
    if lengths is not None:
        out = [w[: int(n)] for w, n in zip(out, lengths)]
    return out
