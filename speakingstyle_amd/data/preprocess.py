"""Offline feature extraction (reference ``preprocessor/preprocessor.py``,
``preprocessor/{ljspeech,libritts,aishell3,bc_2013}.py``, ``prepare_align.py``).

Pipeline: ``prepare_align`` (resample + peak-normalise wavs, write ``.lab``
transcripts) -> Montreal Forced Aligner (external) -> ``Preprocessor.build_from_path``:
TextGrid phones + frame durations (leading/trailing silence trimmed), F0,
mel + energy (TacotronSTFT), optional phoneme-level averaging, outlier-robust
z-normalisation, ``stats.json`` / ``speakers.json`` / ``train.txt`` / ``val.txt``.
Output layout is the reference's.

Offline-image substitutions: TextGrids are parsed here (no ``tgt``); F0 is
pyworld's algorithm pair DIO + StoneMask re-implemented in the native host
runtime (``csrc/host_f0.cpp``, ``utils/native.dio/stonemask``), same frame period
(hop / sr) and 0 = unvoiced convention; numerical parity with pyworld itself is
unpinned (the library is not installable here).  ``preprocessing.pitch.extractor:
yin`` selects the vectorised YIN tracker below instead.
Utterances are processed by a multiprocessing pool (the reference uses
joblib+dask, ``preprocessor/bc_2013.py:62-73``).
"""
from __future__ import annotations

import json
import os
import random
import re
from multiprocessing import Pool
from typing import List, Optional, Tuple

import numpy as np

from ..audio.io import read_wav, write_wav
from ..audio.stft import TacotronSTFT, get_mel_from_wav
from ..text import cleaners as _cleaners

SIL_PHONES = ("sil", "sp", "spn", "")


# ------------------------------------------------------------------ TextGrid
def parse_textgrid(path: str):
    """-> {tier_name: [(start, end, text), ...]} for interval tiers.

    Both Praat formats reduce to the same value sequence -- long format: the values
    right of every ``=``; short format: every quoted string / number -- namely
    file-type, object-class, xmin, xmax, n_tiers, then per tier: class, name, xmin,
    xmax, n, and n (xmin, xmax, text) triples (point tiers: n (time, mark) pairs).
    """
    with open(path, encoding="utf-8") as f:
        raw = f.read()
    tok_re = r'"(?:[^"]|"")*"|[-+]?\d*\.?\d+(?:[eE][-+]?\d+)?'
    if re.search(r"^\s*xmin\s*=", raw, re.M):
        vals = re.findall(r"=\s*(" + tok_re + ")", raw)
    else:
        vals = re.findall(tok_re, raw)

    def unq(t):
        return t[1:-1].replace('""', '"') if t.startswith('"') else t

    vals = [unq(v) if v.startswith('"') else v for v in vals]
    i = 5  # skip header: type, class, xmin, xmax, n_tiers
    n_tiers = int(float(vals[4])) if len(vals) > 4 else 0
    tiers = {}
    for _ in range(n_tiers):
        cls, name = vals[i], vals[i + 1]
        n = int(float(vals[i + 4]))
        i += 5
        if cls == "IntervalTier":
            tiers[name] = [(float(vals[i + 3 * k]), float(vals[i + 3 * k + 1]), vals[i + 3 * k + 2]) for k in range(n)]
            i += 3 * n
        else:
            i += 2 * n
    return tiers


def get_alignment(intervals, sampling_rate: int, hop_length: int):
    """Phones + frame durations, trimming leading/trailing silences (``preprocessor.py:253-291``)."""
    phones: List[str] = []
    durations: List[int] = []
    start_time = end_time = 0.0
    end_idx = 0
    for s, e, p in intervals:
        if not phones:
            if p in SIL_PHONES:
                continue
            start_time = s
        if p not in SIL_PHONES:
            phones.append(p)
            end_time = e
            end_idx = len(phones)
        else:
            phones.append(p if p else "sp")
        durations.append(int(np.round(e * sampling_rate / hop_length) - np.round(s * sampling_rate / hop_length)))
    return phones[:end_idx], durations[:end_idx], start_time, end_time


# ------------------------------------------------------------------ F0 (YIN)
def yin_f0(wav: np.ndarray, sr: int, hop: int, fmin: float = 71.0, fmax: float = 800.0, frame: int = 1024,
           threshold: float = 0.15) -> np.ndarray:
    """Frame-synchronous F0 (Hz, 0 = unvoiced) with center padding like the STFT."""
    x = np.pad(wav.astype(np.float64), (frame // 2, frame // 2), mode="reflect")
    n_frames = 1 + (len(x) - frame) // hop
    tau_min = max(2, int(sr / fmax))
    tau_max = min(frame // 2, int(sr / fmin) + 1)
    idx = np.arange(frame)[None, :] + hop * np.arange(n_frames)[:, None]
    frames = x[idx]
    frames = frames - frames.mean(axis=1, keepdims=True)
    W = frame // 2
    # difference function via FFT autocorrelation: d(tau) = r(0)_t + r(0)_{t+tau} - 2 r(tau)
    fft_n = 1 << int(np.ceil(np.log2(2 * frame)))
    F = np.fft.rfft(frames, fft_n, axis=1)
    acf = np.fft.irfft(F * np.conj(np.fft.rfft(frames[:, :W], fft_n, axis=1)), fft_n, axis=1)[:, : W + 1]
    sq = np.cumsum(frames ** 2, axis=1)
    e0 = sq[:, W - 1:W]
    taus = np.arange(1, W + 1)
    e_tau = sq[:, taus + W - 1] - sq[:, taus - 1]
    d = np.concatenate([np.zeros((n_frames, 1)), e0 + e_tau - 2 * acf[:, 1:]], axis=1)
    cmnd = d.copy()
    csum = np.cumsum(d[:, 1:], axis=1)
    cmnd[:, 1:] = d[:, 1:] * taus[None, :] / np.maximum(csum, 1e-12)
    cmnd[:, 0] = 1.0
    f0 = np.zeros(n_frames)
    region = cmnd[:, tau_min:tau_max]
    below = region < threshold
    has = below.any(axis=1)
    first = np.argmax(below, axis=1)
    for i in np.nonzero(has)[0]:
        t = first[i] + tau_min
        while t + 1 < tau_max and cmnd[i, t + 1] < cmnd[i, t]:
            t += 1
        if 1 <= t < W:  # parabolic interpolation
            a, b, c = cmnd[i, t - 1], cmnd[i, t], cmnd[i, t + 1]
            den = a - 2 * b + c
            t = t + (0.5 * (a - c) / den if abs(den) > 1e-12 else 0.0)
        f0[i] = sr / t
    energy_gate = np.sqrt(e0[:, 0] / W) > 1e-4
    return (f0 * energy_gate).astype(np.float64)


def extract_f0(wav: np.ndarray, sr: int, hop: int, method: str = "dio") -> np.ndarray:
    """Frame F0 (Hz, 0 = unvoiced) on the hop grid.  ``dio``: DIO + StoneMask exactly as
    the reference calls pyworld (``preprocessor/preprocessor.py:182-187``: float64 wav,
    frame_period = hop / sr * 1000 ms, default floor/ceil 71/800 Hz)."""
    if method == "dio":
        from ..utils import native

        x = wav.astype(np.float64)
        f0, t = native.dio(x, sr, frame_period=hop / sr * 1000)
        return native.stonemask(x, f0, t, sr)
    if method == "yin":
        return yin_f0(wav, sr, hop)
    raise ValueError(f"unknown pitch extractor {method!r} (dio | yin)")


def interpolate_unvoiced(pitch: np.ndarray) -> np.ndarray:
    nz = np.nonzero(pitch)[0]
    if len(nz) == 0:
        return pitch
    return np.interp(np.arange(len(pitch)), nz, pitch[nz])


def phoneme_average(values: np.ndarray, durations: List[int]) -> np.ndarray:
    out = np.zeros(len(durations))
    pos = 0
    for i, d in enumerate(durations):
        out[i] = np.mean(values[pos:pos + d]) if d > 0 else 0.0
        pos += d
    return out


def remove_outlier(values: np.ndarray) -> np.ndarray:
    values = np.asarray(values)
    if values.size == 0:
        return values
    p25, p75 = np.percentile(values, [25, 75])
    lo, hi = p25 - 1.5 * (p75 - p25), p75 + 1.5 * (p75 - p25)
    return values[(values > lo) & (values < hi)]


class RunningMoments:
    """StandardScaler.partial_fit equivalent (Chan's parallel update)."""

    def __init__(self):
        self.n, self.mean, self.m2 = 0, 0.0, 0.0

    def update(self, x):
        x = np.asarray(x, dtype=np.float64).reshape(-1)
        if x.size == 0:
            return
        n_b, mean_b = x.size, float(x.mean())
        m2_b = float(((x - mean_b) ** 2).sum())
        n = self.n + n_b
        delta = mean_b - self.mean
        self.mean += delta * n_b / n
        self.m2 += m2_b + delta * delta * self.n * n_b / n
        self.n = n

    @property
    def std(self):
        return float(np.sqrt(self.m2 / self.n)) if self.n else 1.0


# ------------------------------------------------------------------ Preprocessor
class Preprocessor:
    def __init__(self, config, model_config=None):  # second arg accepted for CLI compatibility
        self.config = config
        pp = config["preprocessing"]
        self.in_dir = config["path"]["raw_path"]
        self.out_dir = config["path"]["preprocessed_path"]
        self.val_size = pp["val_size"]
        self.sampling_rate = pp["audio"]["sampling_rate"]
        self.hop_length = pp["stft"]["hop_length"]
        self.pitch_phoneme = pp["pitch"]["feature"] == "phoneme_level"
        self.energy_phoneme = pp["energy"]["feature"] == "phoneme_level"
        self.pitch_norm = pp["pitch"]["normalization"]
        self.energy_norm = pp["energy"]["normalization"]
        self.f0_method = pp["pitch"].get("extractor", "dio")
        self.stft = TacotronSTFT(pp["stft"]["filter_length"], self.hop_length, pp["stft"]["win_length"],
                                 pp["mel"]["n_mel_channels"], self.sampling_rate, pp["mel"]["mel_fmin"],
                                 pp["mel"]["mel_fmax"])

    def process_utterance(self, speaker: str, basename: str):
        wav_path = os.path.join(self.in_dir, speaker, f"{basename}.wav")
        lab_path = os.path.join(self.in_dir, speaker, f"{basename}.lab")
        tg_path = os.path.join(self.out_dir, "TextGrid", speaker, f"{basename}.TextGrid")
        tiers = parse_textgrid(tg_path)
        phone, duration, start, end = get_alignment(tiers.get("phones", []), self.sampling_rate, self.hop_length)
        if start >= end or not phone:
            return None
        text = "{" + " ".join(phone) + "}"
        wav, _ = read_wav(wav_path, self.sampling_rate)
        wav = wav[int(self.sampling_rate * start): int(self.sampling_rate * end)].astype(np.float32)
        with open(lab_path, encoding="utf-8") as f:
            raw_text = f.readline().strip("\n")
        pitch = extract_f0(wav, self.sampling_rate, self.hop_length, self.f0_method)
        mel, energy = get_mel_from_wav(np.clip(wav, -1, 1), self.stft)
        T = sum(duration)
        pitch, mel, energy = pitch[:T], mel[:, :T], energy[:T]
        if pitch.shape[0] < T or np.sum(pitch != 0) <= 1:
            return None
        if self.pitch_phoneme:
            pitch = phoneme_average(interpolate_unvoiced(pitch), duration)
        if self.energy_phoneme:
            energy = phoneme_average(energy, duration)
        for kind, arr in (("duration", np.asarray(duration)), ("pitch", pitch), ("energy", energy), ("mel", mel.T)):
            np.save(os.path.join(self.out_dir, kind, f"{speaker}-{kind}-{basename}.npy"), arr)
        return "|".join([basename, speaker, text, raw_text]), remove_outlier(pitch), remove_outlier(energy), mel.shape[1]

    def build_from_path(self, workers: int = 4):
        for kind in ("mel", "pitch", "energy", "duration"):
            os.makedirs(os.path.join(self.out_dir, kind), exist_ok=True)
        speakers = {}
        jobs: List[Tuple[str, str]] = []
        for i, spk in enumerate(sorted(os.listdir(self.in_dir))):
            spk_dir = os.path.join(self.in_dir, spk)
            if not os.path.isdir(spk_dir):
                continue
            speakers[spk] = len(speakers)
            for fn in sorted(os.listdir(spk_dir)):
                if fn.endswith(".wav"):
                    base = fn[:-4]
                    if os.path.exists(os.path.join(self.out_dir, "TextGrid", spk, f"{base}.TextGrid")):
                        jobs.append((spk, base))
        if workers > 1:
            with Pool(workers) as pool:
                results = pool.starmap(self.process_utterance, jobs)
        else:
            results = [self.process_utterance(s, b) for s, b in jobs]
        out, pm, em = [], RunningMoments(), RunningMoments()
        n_frames = 0
        for r in results:
            if r is None:
                continue
            info, p, e, n = r
            out.append(info)
            pm.update(p)
            em.update(e)
            n_frames += n
        p_mean, p_std = (pm.mean, pm.std) if self.pitch_norm else (0.0, 1.0)
        e_mean, e_std = (em.mean, em.std) if self.energy_norm else (0.0, 1.0)
        p_min, p_max = self.normalize(os.path.join(self.out_dir, "pitch"), p_mean, p_std)
        e_min, e_max = self.normalize(os.path.join(self.out_dir, "energy"), e_mean, e_std)
        with open(os.path.join(self.out_dir, "speakers.json"), "w") as f:
            json.dump(speakers, f)
        with open(os.path.join(self.out_dir, "stats.json"), "w") as f:
            json.dump({"pitch": [p_min, p_max, p_mean, p_std], "energy": [e_min, e_max, e_mean, e_std]}, f)
        random.Random(1234).shuffle(out)
        val = out[: self.val_size]
        train = out[self.val_size:]
        with open(os.path.join(self.out_dir, "train.txt"), "w", encoding="utf-8") as f:
            f.write("".join(x + "\n" for x in train))
        with open(os.path.join(self.out_dir, "val.txt"), "w", encoding="utf-8") as f:
            f.write("".join(x + "\n" for x in val))
        print("Total time: {:.2f} hours".format(n_frames * self.hop_length / self.sampling_rate / 3600))
        return out

    @staticmethod
    def normalize(in_dir, mean, std):
        lo, hi = np.finfo(np.float64).max, np.finfo(np.float64).min
        for fn in os.listdir(in_dir):
            p = os.path.join(in_dir, fn)
            v = (np.load(p) - mean) / std
            np.save(p, v)
            if v.size:
                lo, hi = min(lo, float(v.min())), max(hi, float(v.max()))
        return lo, hi


# ------------------------------------------------------------------ prepare_align
def _write_pair(out_dir, speaker, base, wav, sr_in, sr, max_wav_value, text):
    os.makedirs(os.path.join(out_dir, speaker), exist_ok=True)
    wav = np.asarray(wav, dtype=np.float64)
    if sr_in != sr:
        from math import gcd

        from scipy.signal import resample_poly

        g = gcd(sr_in, sr)
        wav = resample_poly(wav, sr // g, sr_in // g)
    wav = wav / max(np.abs(wav).max(), 1e-8) * max_wav_value
    write_wav(os.path.join(out_dir, speaker, f"{base}.wav"), sr, wav.astype(np.int16))
    with open(os.path.join(out_dir, speaker, f"{base}.lab"), "w", encoding="utf-8") as f:
        f.write(text)


def _clean(text, names):
    for n in names:
        text = getattr(_cleaners, n)(text)
    return text


def prepare_align(config):
    """Dataset dispatcher (reference ``prepare_align.py:8-17``)."""
    ds = config["dataset"]
    in_dir = config["path"]["corpus_path"]
    out_dir = config["path"]["raw_path"]
    sr = config["preprocessing"]["audio"]["sampling_rate"]
    mx = config["preprocessing"]["audio"]["max_wav_value"] - 1  # stay inside int16
    names = config["preprocessing"]["text"]["text_cleaners"]
    n = 0
    if ds in ("LJSpeech", "BC2013"):
        meta = os.path.join(in_dir, "metadata.csv")
        spk = ds
        with open(meta, encoding="utf-8") as f:
            for line in f:
                parts = line.strip().split("|")
                if len(parts) < 2:
                    continue
                base, text = parts[0], parts[-1]
                wp = os.path.join(in_dir, "wavs", f"{base}.wav")
                if os.path.exists(wp):
                    wav, sr_in = read_wav(wp)
                    _write_pair(out_dir, spk, base, wav, sr_in, sr, mx, _clean(text, names))
                    n += 1
    elif ds == "LibriTTS":
        for spk in sorted(os.listdir(in_dir)):
            for chap in sorted(os.listdir(os.path.join(in_dir, spk))):
                d = os.path.join(in_dir, spk, chap)
                for fn in sorted(os.listdir(d)):
                    if not fn.endswith(".wav"):
                        continue
                    base = fn[:-4]
                    tp = os.path.join(d, f"{base}.normalized.txt")
                    if not os.path.exists(tp):
                        continue
                    with open(tp, encoding="utf-8") as f:
                        text = _clean(f.readline().strip(), names)
                    wav, sr_in = read_wav(os.path.join(d, fn))
                    _write_pair(out_dir, spk, base, wav, sr_in, sr, mx, text)
                    n += 1
    elif ds == "AISHELL3":
        for split in ("train", "test"):
            content = os.path.join(in_dir, split, "content.txt")
            if not os.path.exists(content):
                continue
            with open(content, encoding="utf-8") as f:
                for line in f:
                    wav_name, text = line.strip("\n").split("\t")
                    spk = wav_name[:7]
                    text = " ".join(text.split(" ")[1::2])  # pinyin tokens
                    wp = os.path.join(in_dir, split, "wav", spk, wav_name)
                    if os.path.exists(wp):
                        wav, sr_in = read_wav(wp)
                        _write_pair(out_dir, spk, wav_name[:-4], wav, sr_in, sr, mx, text)
                        n += 1
    else:
        raise ValueError(f"unknown dataset {ds!r}")
    return n
