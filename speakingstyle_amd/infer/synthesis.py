"""Text -> mel -> waveform synthesis (reference ``synthesize.py:26-292``).

Modes (same as the reference): ``single`` (one text + optional reference wav for
the speaking style) and ``batch`` (a metadata file through ``TextDataset``, each
utterance's own mel as the style reference).  Added:

* word-level prosody control (the reference notebook ``control.ipynb``'s
  ``ControlledVarianceAdapter``): per-word pitch / energy / duration factors are
  expanded to per-phoneme control tensors,
* GST token weights as a style source without reference audio,
* neutral style when no reference is given (the reference crashes),
* ``bench_durations``: fixed injected durations for throughput benchmarks with
  random-init weights (random duration predictors emit ~0 frames).
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..audio.io import read_wav
from ..audio.stft import TacotronSTFT, get_mel_from_wav
from ..data.dataset import to_device
from ..text import g2p
from ..utils.logging import synth_samples


def reference_mel(preprocess_config, wav_path: str) -> np.ndarray:
    """Reference-audio featurizer (``synthesize.py:93-125``) -> [T, n_mel] float32."""
    pp = preprocess_config["preprocessing"]
    wav, _ = read_wav(wav_path, pp["audio"]["sampling_rate"])
    stft = TacotronSTFT(pp["stft"]["filter_length"], pp["stft"]["hop_length"], pp["stft"]["win_length"],
                        pp["mel"]["n_mel_channels"], pp["audio"]["sampling_rate"], pp["mel"]["mel_fmin"],
                        pp["mel"]["mel_fmax"])
    mel, _ = get_mel_from_wav(np.clip(wav, -1, 1), stft)
    return mel.T.astype(np.float32)


def word_level_controls(groups, per_word: Optional[Sequence[float]], default: float = 1.0) -> np.ndarray:
    """Expand per-word factors to per-phoneme factors (punctuation 'sp' keeps the default)."""
    out: List[float] = []
    wi = 0
    for word, phones in groups:
        is_word = not (len(phones) == 1 and phones[0] == "sp" and not word.isalnum())
        f = default
        if is_word and per_word is not None:
            f = float(per_word[wi]) if wi < len(per_word) else default
            wi += 1
        out += [f] * len(phones)
    return np.asarray(out, dtype=np.float32)


def single_batch(text: str, preprocess_config, speaker_id: int = 0, ref_audio: Optional[str] = None,
                 lexicon: Optional[dict] = None):
    pp = preprocess_config["preprocessing"]
    cleaners = pp["text"]["text_cleaners"]
    if pp["text"].get("language", "en") == "zh":
        seq, phones = g2p.preprocess_mandarin(text.split(), cleaners, lexicon)
    else:
        seq, phones = g2p.preprocess_english(text, cleaners, lexicon)
    ids = [text[:100]]
    texts = np.asarray([seq], dtype=np.int64)
    text_lens = np.asarray([len(seq)], dtype=np.int64)
    if ref_audio:
        mel = reference_mel(preprocess_config, ref_audio)[None]
    else:
        mel = np.zeros((1, 1, pp["mel"]["n_mel_channels"]), np.float32)
    mel_lens = np.asarray([mel.shape[1]], dtype=np.int64)
    batch = (ids, [text], np.asarray([speaker_id], dtype=np.int64), texts, text_lens, int(text_lens.max()), mel,
             mel_lens, int(mel_lens.max()))
    return batch, phones, (ref_audio is not None)


@torch.no_grad()
def synthesize(model, configs, vocoder, batchs, control_values, result_path, plot=False, use_ref=True,
               style_weights=None, bench_durations=None):
    preprocess_config, model_config, _ = configs
    p_ctl, e_ctl, d_ctl = control_values
    device = next(model.parameters()).device
    outputs = []
    for batch in batchs:
        batch = to_device(batch, device)
        mels = batch[6] if use_ref else None
        mel_lens = batch[7] if use_ref else None
        sw = None if style_weights is None else torch.as_tensor(style_weights, device=device).float().view(1, -1).expand(
            batch[3].shape[0], -1)
        d_t = None
        if bench_durations is not None:
            d_t = torch.full_like(batch[3], int(bench_durations)).masked_fill(
                torch.arange(batch[3].shape[1], device=device)[None] >= batch[4][:, None], 0)
        ctl = [torch.as_tensor(c, device=device).view(1, -1) if isinstance(c, (list, np.ndarray)) else c
               for c in (p_ctl, e_ctl, d_ctl)]
        out = model(batch[2], batch[3], batch[4], batch[5], mels=mels, mel_lens=mel_lens,
                    max_mel_len=batch[8] if use_ref else None, d_targets=d_t,
                    p_control=ctl[0], e_control=ctl[1], d_control=ctl[2], style_weights=sw)
        if vocoder is not None and result_path is not None:
            synth_samples(batch, out, vocoder, model_config, preprocess_config, result_path, plot=plot)
        outputs.append(out)
    return outputs
