"""One-batch forward inspection on the training data (reference ``notebooks/ref_encoder.ipynb``
cells 2-11: the notebook re-declares the Dataset with speaker-embedding loading, builds the
loader exactly like ``train.py`` and pushes one batch through the model to debug the
reference encoder).

``inspect_batch`` does the same with the framework's own loader (``ShardedGroupSampler``
grouping, speaker-embedding table when configured) and returns a report: output shapes,
the loss terms, the style encoder's FiLM conditioning statistics (gamma / beta mean, std,
per-utterance norms) and the learnable FiLM scalars.  Synthetic batches of the
configured shape are used when the preprocessed corpus is absent.
"""
from __future__ import annotations

from typing import Dict

import torch


@torch.no_grad()
def inspect_batch(model, configs, device, split: str = "train.txt", synthetic: bool = False, seed: int = 1234) -> Dict:
    import os

    from ..data.dataset import Dataset, ShardedGroupSampler, to_device
    from ..data.synthetic import SyntheticBatches
    from ..models.loss import FastSpeech2Loss

    pp, mc, tc = configs
    root = pp["path"]["preprocessed_path"]
    if synthetic or not os.path.exists(os.path.join(root, split)):
        batch = SyntheticBatches(int(tc["optimizer"]["batch_size"]), device=device, seed=seed,
                                 max_seq_len=mc["max_seq_len"]).make_batch()
        source = "synthetic"
    else:
        ds = Dataset(split, pp, tc, sort=True, drop_last=True)
        sampler = ShardedGroupSampler(ds, int(tc["optimizer"]["batch_size"]), 4, 0, 1, seed=seed)
        idx = next(iter(sampler))
        batch = to_device(ds.collate_local([ds[i] for i in idx])[0], device)
        source = split
    model.eval()
    out = model(*batch[2:])
    losses = FastSpeech2Loss(pp, tc)(batch, out, model.film_scalars())
    names = ["total", "mel", "postnet", "pitch", "energy", "duration"]
    rep = {"source": source, "batch_size": int(batch[2].shape[0]), "max_src_len": int(batch[5]),
           "max_mel_len": int(batch[8]),
           "outputs": {k: (None if v is None else list(v.shape)) for k, v in zip(
               ["mel", "postnet", "pitch", "energy", "log_duration", "duration_rounded", "src_masks", "mel_masks",
                "src_lens", "mel_lens"], out)},
           "losses": {n: float(v) for n, v in zip(names, losses[:6])}}
    mels, mel_lens, max_mel = batch[6], batch[7], batch[8]
    style = model.compute_style(mels, mel_lens, max_mel, batch[3].shape[0], mels.device)
    if style is not None:
        g, b = (t.float() for t in style)
        rep["style"] = {"gamma_mean": float(g.mean()), "gamma_std": float(g.std()), "beta_mean": float(b.mean()),
                        "beta_std": float(b.std()), "gamma_norm_per_utt": g.norm(dim=1).cpu().tolist(),
                        "beta_norm_per_utt": b.norm(dim=1).cpu().tolist()}
    fs = model.film_scalars()
    if fs is not None:
        rep["film_scalars"] = fs.float().cpu().tolist()
    return rep
