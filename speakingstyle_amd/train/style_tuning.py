"""Style-token bank tuning from human-annotated, re-embedded utterances.

The reference states this as its research goal (``README.md:3-7``: tune a fixed bank of style
tokens using human-annotated utterances) but implements none of it; SURVEY §2.6 scopes an API
in.  The procedure here:

1. **Re-embed** every annotated utterance once through the frozen GST reference encoder
   (``GlobalStyleTokens.reference_embedding`` -> ``w_query``): one query vector per utterance.
2. **Tune** only the token bank (``gst.embed``; optionally also the key / value projections)
   with two terms per utterance i with annotation distribution t_i over the tokens:

   * ``CE``: cross-entropy between t_i and the head-averaged attention weights of q_i over
     the bank -- the utterance should attend to the tokens the annotator chose;
   * ``MSE``: || style(t_i) - style(q_i) ||^2, where style(t) is the token mixture
     ``from_token_weights`` uses at synthesis and style(q) the attention output -- choosing
     the annotated token(s) by weight at synthesis reproduces that utterance's style.

Everything else in the model stays frozen (requires_grad restored afterwards).  On the GPU the
encoder and the token attention run on the HIP kernels (``csrc/k_gst.hip``).

Annotation file (``parse_annotations``): one utterance per line, ``basename|speaker|label``
where ``label`` is a token index (``3``) or a comma-separated weight vector over the tokens
(``0,0.5,0.5,0,...``); the mel is read from ``{preprocessed_path}/mel/{speaker}-mel-{basename}.npy``.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from ..utils.tools import pad_2d


def parse_label(label: str, n_tokens: int) -> np.ndarray:
    label = label.strip()
    if "," in label:
        w = np.asarray([float(x) for x in label.split(",") if x.strip()], dtype=np.float32)
        if w.shape[0] != n_tokens:
            raise ValueError(f"weight label has {w.shape[0]} entries, the bank has {n_tokens} tokens")
    else:
        k = int(label)
        if not 0 <= k < n_tokens:
            raise ValueError(f"token index {k} out of range [0, {n_tokens})")
        w = np.zeros(n_tokens, dtype=np.float32)
        w[k] = 1.0
    s = float(w.sum())
    if s <= 0 or (w < 0).any():
        raise ValueError(f"label {label!r}: weights must be non-negative with a positive sum")
    return w / s


def parse_annotations(path: str, preprocessed_path: str, n_tokens: int) -> Tuple[List[str], List[np.ndarray], np.ndarray]:
    """-> (basenames, mels [T, n_mel] f32, targets [N, n_tokens])."""
    names, mels, targets = [], [], []
    with open(path, encoding="utf-8") as f:
        for ln, line in enumerate(f, 1):
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            parts = line.split("|")
            if len(parts) != 3:
                raise ValueError(f"{path}:{ln}: expected basename|speaker|label")
            base, spk, label = parts
            mel = np.load(os.path.join(preprocessed_path, "mel", f"{spk}-mel-{base}.npy")).astype(np.float32)
            names.append(base)
            mels.append(mel)
            targets.append(parse_label(label, n_tokens))
    if not names:
        raise ValueError(f"{path}: no annotations")
    return names, mels, np.stack(targets)


class StyleTokenTuner:
    def __init__(self, model, lr: float = 1e-2, steps: int = 300, mse_weight: float = 1.0,
                 tune_projections: bool = False, batch_size: int = 64):
        gst = getattr(model, "gst", None)
        if gst is None:
            raise ValueError("style-token tuning needs a GST model (model.yaml `gst: use_gst: true`)")
        self.model, self.gst = model, gst
        self.lr, self.steps, self.mse_weight = lr, steps, mse_weight
        self.batch_size = batch_size
        self.tuned = [gst.embed] + ([gst.w_key.weight, gst.w_value.weight] if tune_projections else [])

    @property
    def device(self):
        return self.gst.embed.device

    @torch.no_grad()
    def embed_queries(self, mels: Sequence[np.ndarray]) -> torch.Tensor:
        """Re-embedding: [N, token_size] queries of the frozen reference encoder (eval mode)."""
        was = self.gst.training
        self.gst.eval()
        cd = self.model.compute_dtype
        out = []
        try:
            for i in range(0, len(mels), self.batch_size):
                chunk = mels[i:i + self.batch_size]
                lens = torch.tensor([m.shape[0] for m in chunk], device=self.device)
                x = torch.from_numpy(pad_2d(chunk)).to(self.device, cd)
                ref = self.gst.reference_embedding(x, lens)
                out.append(F.linear(ref.float(), self.gst.w_query.weight.float()))
        finally:
            self.gst.train(was)
        return torch.cat(out)

    def losses(self, q: torch.Tensor, targets: torch.Tensor) -> Dict[str, torch.Tensor]:
        style_q, w = self.gst.token_attention(q)
        p = w.float().mean(1).clamp_min(1e-8)                     # head-averaged weights [N, n_tok]
        ce = -(targets * p.log()).sum(1).mean()
        k, v = self.gst.token_bank()                               # [heads, n_tok, d]
        style_t = torch.einsum("bn,hnd->bhd", targets, v.float()).reshape(targets.shape[0], -1)
        mse = (style_t - style_q.float()).pow(2).sum(1).mean()
        return {"ce": ce, "mse": mse, "total": ce + self.mse_weight * mse, "weights": p.detach()}

    def fit(self, mels: Sequence[np.ndarray], targets, log_every: int = 0) -> dict:
        targets = torch.as_tensor(np.asarray(targets), dtype=torch.float32, device=self.device)
        q = self.embed_queries(mels)
        saved = {id(p): p.requires_grad for p in self.model.parameters()}
        self.model.requires_grad_(False)
        for p in self.tuned:
            p.requires_grad_(True)
        opt = torch.optim.Adam(self.tuned, lr=self.lr)
        history = []
        try:
            for step in range(self.steps):
                opt.zero_grad(set_to_none=True)
                lo = self.losses(q, targets)
                lo["total"].backward()
                opt.step()
                history.append({k: float(lo[k].detach()) for k in ("total", "ce", "mse")})
                if log_every and (step % log_every == 0 or step == self.steps - 1):
                    print(f"step {step}: " + ", ".join(f"{k} {v:.4f}" for k, v in history[-1].items()))
            with torch.no_grad():
                p = self.losses(q, targets)["weights"]
        finally:
            for prm in self.model.parameters():
                prm.requires_grad_(saved.get(id(prm), True))
            for prm in self.tuned:
                prm.grad = None
        if self.device.type == "cuda":
            from ..ops import hip  # the bank changed in place: cached bf16 images must be rebuilt

            hip.bump_weight_generation()
        acc = float((p.argmax(1) == targets.argmax(1)).float().mean())
        return {"history": history, "accuracy": acc, "weights": p.cpu().numpy()}
