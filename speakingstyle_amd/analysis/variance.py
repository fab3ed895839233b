"""Variance-distribution analysis (reference ``notebooks/variance_control_distbn.ipynb``
cells 2-35): ground-truth pitch / energy (de-normalised with ``stats.json``) and durations of
a metadata list, the model's predictions on the same texts (optionally under p/e/d control),
IQR outlier removal, and true-vs-predicted histograms with overlap / distance summaries.

Differences from the notebook: no dask / joblib cluster (files are read sequentially, the
model runs batched on the GPU through the HIP kernels), the duration predictions are the
rounded frame counts the length regulator uses, and results are returned as arrays + a JSON
summary (and PNG overlays when ``out_dir`` is given) instead of inline plots.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch


def remove_outlier(values, k: float = 3.0) -> np.ndarray:
    """Keep values strictly inside [p25 - k*IQR, p75 + k*IQR] (notebook cells 14 / 33: k = 3, 6)."""
    v = np.asarray(values, dtype=np.float64)
    if v.size == 0:
        return v
    p25, p75 = np.percentile(v, 25), np.percentile(v, 75)
    lo, hi = p25 - k * (p75 - p25), p75 + k * (p75 - p25)
    return v[(v > lo) & (v < hi)]


def read_basenames(list_path: str) -> List[str]:
    with open(list_path, encoding="utf-8") as f:
        return [ln.split("|")[0] for ln in f if ln.strip()]


def _stats(preprocessed_path: str) -> Dict[str, Sequence[float]]:
    with open(os.path.join(preprocessed_path, "stats.json")) as f:
        return json.load(f)


def ground_truth(preprocessed_path: str, basenames: Iterable[str]) -> Dict[str, np.ndarray]:
    """De-normalised pitch / energy and integer durations of the given utterances
    (``{kind}/{speaker}-{kind}-{basename}.npy``; speaker-agnostic match on the basename)."""
    st = _stats(preprocessed_path)
    want = set(basenames)
    out = {}
    for kind in ("pitch", "energy", "duration"):
        d = os.path.join(preprocessed_path, kind)
        vals: List[np.ndarray] = []
        for fn in sorted(os.listdir(d)) if os.path.isdir(d) else []:
            stem = os.path.splitext(fn)[0]
            parts = stem.split("-")
            base = "-".join(parts[2:]) if len(parts) > 2 and parts[1] == kind else stem
            if base not in want:
                continue
            x = np.load(os.path.join(d, fn), allow_pickle=False).astype(np.float64).reshape(-1)
            if kind != "duration":
                x = x * st[kind][3] + st[kind][2]
            vals.append(x)
        out[kind] = np.concatenate(vals) if vals else np.zeros(0)
    return out


@torch.no_grad()
def predicted(model, batches, stats: Dict[str, Sequence[float]], device, controls=(1.0, 1.0, 1.0)) -> Dict[str, np.ndarray]:
    """Model predictions over the valid phonemes of ``batches`` (TextDataset-style tuples, reference
    ``synthesize.py`` forward): de-normalised pitch / energy and rounded durations (frames)."""
    from ..data.dataset import to_device

    model.eval()
    p_all, e_all, d_all = [], [], []
    for b in batches:
        b = to_device(b, device)
        # reference mels (when the list has them) drive the style encoder, as in synthesize.py batch mode
        out = model(*b[2:], p_control=controls[0], e_control=controls[1], d_control=controls[2])
        p, e, d, src_mask = out[2], out[3], out[5], out[6]
        valid = ~src_mask
        if p is not None and p.shape == valid.shape:
            p_all.append(p[valid].float().cpu().numpy())
        if e is not None and e.shape == valid.shape:
            e_all.append(e[valid].float().cpu().numpy())
        d_all.append(d[valid].float().cpu().numpy())
    cat = lambda xs: np.concatenate(xs).astype(np.float64) if xs else np.zeros(0)  # noqa: E731
    return {"pitch": cat(p_all) * stats["pitch"][3] + stats["pitch"][2],
            "energy": cat(e_all) * stats["energy"][3] + stats["energy"][2],
            "duration": cat(d_all)}


def compare(true: np.ndarray, pred: np.ndarray, bins: int = 50) -> Dict[str, float]:
    """Histogram overlap (sum of min of the two densities x bin width, 1 = identical), Jensen-Shannon
    divergence (bits) and the first two moments of both samples."""
    true, pred = np.asarray(true, np.float64), np.asarray(pred, np.float64)
    if true.size == 0 or pred.size == 0:
        return {"n_true": int(true.size), "n_pred": int(pred.size)}
    lo, hi = min(true.min(), pred.min()), max(true.max(), pred.max())
    if hi <= lo:
        hi = lo + 1e-6
    edges = np.linspace(lo, hi, bins + 1)
    ht, _ = np.histogram(true, edges, density=True)
    hp, _ = np.histogram(pred, edges, density=True)
    w = edges[1] - edges[0]
    pt, pp = ht * w, hp * w
    m = 0.5 * (pt + pp)

    def kl(a, b):
        nz = a > 0
        return float(np.sum(a[nz] * np.log2(a[nz] / b[nz])))

    return {"n_true": int(true.size), "n_pred": int(pred.size), "overlap": float(np.minimum(pt, pp).sum()),
            "js_bits": 0.5 * kl(pt, m) + 0.5 * kl(pp, m), "mean_true": float(true.mean()),
            "mean_pred": float(pred.mean()), "std_true": float(true.std()), "std_pred": float(pred.std())}


def plot_overlay(true, pred, label: str, path: str, bins: int = 50):
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    fig, ax = plt.subplots(figsize=(6, 4))
    ax.hist(true, bins=bins, alpha=0.5, label="true", density=True)
    ax.hist(pred, bins=bins, alpha=0.5, label="pred", density=True)
    ax.legend(loc="upper right")
    ax.set_xlabel(label)
    fig.tight_layout()
    fig.savefig(path)
    plt.close(fig)


def analyze(model, configs, source: str, device, controls=(1.0, 1.0, 1.0), out_dir: Optional[str] = None,
            batch_size: int = 8, outlier_k: float = 3.0) -> Dict[str, Dict[str, float]]:
    """Full notebook flow on ``source`` (a ``val.txt``-style list): ground truth vs predictions."""
    from torch.utils.data import DataLoader

    from ..data.dataset import TextDataset

    pp = configs[0]
    root = pp["path"]["preprocessed_path"]
    st = _stats(root)
    gt = ground_truth(root, read_basenames(source))
    ds = TextDataset(source, pp)
    pr = predicted(model, DataLoader(ds, batch_size=batch_size, collate_fn=ds.collate_fn), st, device, controls)
    summary = {}
    for kind, label in (("pitch", "F0"), ("energy", "Energy"), ("duration", "Duration")):
        t, p = gt[kind], pr[kind]
        if kind == "duration":
            t, p = remove_outlier(t, outlier_k), remove_outlier(p, outlier_k)
        summary[kind] = compare(t, p)
        if out_dir and t.size and p.size:
            os.makedirs(out_dir, exist_ok=True)
            plot_overlay(t, p, label, os.path.join(out_dir, f"{kind}_true_vs_pred.png"))
    if out_dir:
        with open(os.path.join(out_dir, "variance_summary.json"), "w") as f:
            json.dump(summary, f, indent=2)
    return summary
