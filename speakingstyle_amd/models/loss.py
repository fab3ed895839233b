"""FastSpeech2 loss (reference ``model/loss.py:5-99``).

Same five masked terms + ``lambda_f * sum(s^2)`` over the FiLM scalars and the
same 7-tuple output.  Implementation differences:

* no ``masked_select`` compaction -- masked sums / valid counts; on the GPU two
  fused deterministic HIP kernel pairs (L1 mel + postnet; MSE pitch + energy +
  log-duration) instead of ~30 elementwise/reduction launches;
* optional *global* valid counts for data parallelism: each rank divides its
  masked sums by the counts of the whole global batch (all-reduced), so summed
  gradients equal the single-process full-batch gradient (the reference computes
  the loss on the DataParallel-gathered full batch, ``train.py:86-88``).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from .. import ops


class FastSpeech2Loss(nn.Module):
    def __init__(self, preprocess_config, train_config):
        super().__init__()
        pp = preprocess_config["preprocessing"]
        self.pitch_feature_level = pp["pitch"]["feature"]
        self.energy_feature_level = pp["energy"]["feature"]
        loss_cfg = train_config.get("loss") or {}
        self.lambda_f = float(loss_cfg.get("lambda_f", 0.0))

    @staticmethod
    def local_counts(batch, predictions, n_mel):
        """[mel elements, pitch elements, energy elements, phonemes] valid in this batch."""
        src_masks, mel_masks = predictions[6], predictions[7]
        n_src = (~src_masks).sum()
        n_mel_frames = (~mel_masks).sum()
        return torch.stack([n_mel_frames * n_mel, n_src, n_mel_frames]).float()

    def forward(self, inputs, predictions, named_param: Optional[torch.Tensor] = None,
                global_counts: Optional[torch.Tensor] = None):
        mel_t, _, _, p_t, e_t, d_t = inputs[6:12]
        mel_p, post_p, p_p, e_p, logd_p, _, src_masks, mel_masks, _, _ = predictions
        M = mel_masks.shape[1]
        mel_t = mel_t[:, :M]
        n_mel = mel_t.shape[-1]
        phon_p = self.pitch_feature_level == "phoneme_level"
        phon_e = self.energy_feature_level == "phoneme_level"
        if mel_p.is_cuda and ops.use_hip(mel_p):
            # GPU: two fused deterministic kernel pairs (L1 mel/postnet, MSE pitch/energy/duration)
            from ..ops import hip

            # one autograd node: both fused kernel pairs + a finalize kernel that counts the valid mel
            # elements from the lengths (mel_masks = t >= min(len, M)) and forms the total
            if global_counts is not None:
                c_mel = global_counts[0]
                gc = global_counts[[1 if phon_p else 2, 1 if phon_e else 2, 1]]
            else:
                c_mel, gc = None, None  # the kernels count the unmasked elements themselves
            total, mel_l, post_l, pitch_l, energy_l, dur_l = hip.fs2_losses(
                mel_p, post_p, mel_t, inputs[7], p_p, p_t, src_masks if phon_p else mel_masks, e_p, e_t,
                src_masks if phon_e else mel_masks, logd_p, d_t, src_masks, mel_count=c_mel, var_counts=gc)
            if named_param is not None and self.lambda_f > 0:
                total = total + self.lambda_f * torch.sum(torch.square(named_param))
            return total, mel_l, post_l, pitch_l, energy_l, dur_l, self.lambda_f
        else:
            src_valid = ~src_masks
            mel_valid = ~mel_masks
            p_valid = src_valid if phon_p else mel_valid
            e_valid = src_valid if phon_e else mel_valid
            if not phon_p:
                p_t, p_p = p_t[:, :M], p_p[:, :M]
            if not phon_e:
                e_t, e_p = e_t[:, :M], e_p[:, :M]
            if global_counts is not None:
                c_mel, c_src, c_frame = global_counts[0], global_counts[1], global_counts[2]
            else:
                c_mel = (mel_valid.sum() * n_mel).float()
                c_src = src_valid.sum().float()
                c_frame = mel_valid.sum().float()
            c_p = c_src if phon_p else c_frame
            c_e = c_src if phon_e else c_frame
            mv = mel_valid.unsqueeze(-1)
            mel_l = ((mel_p - mel_t.float()).abs() * mv).sum() / c_mel.clamp(min=1)
            post_l = ((post_p - mel_t.float()).abs() * mv).sum() / c_mel.clamp(min=1)
            pitch_l = _mse(p_p, p_t, p_valid, c_p)
            energy_l = _mse(e_p, e_t, e_valid, c_e)
            dur_l = _mse(logd_p, torch.log(d_t.float() + 1.0), src_valid, c_src)
        total = mel_l + post_l + dur_l + pitch_l + energy_l
        if named_param is not None and self.lambda_f > 0:
            total = total + self.lambda_f * torch.sum(torch.square(named_param))
        return total, mel_l, post_l, pitch_l, energy_l, dur_l, self.lambda_f


def _mse(pred, target, valid, count):
    diff = (pred.float() - target.float()) * valid
    return (diff * diff).sum() / count.clamp(min=1)
