"""HIP-graph training steps: the forward + loss + backward of a step captured once per padded-shape bucket
and replayed (reference ``train.py:79-101``: one optimizer step per batch; this changes how the step is
launched, not what it computes).

Why: a FastSpeech2 step is ~700 kernel launches driven from Python and autograd (~12-14 ms of host time).
With a large per-GPU batch (LJSpeech, 200 utterances) the GPU takes longer than that and the host runs
ahead; with the reference's small per-GPU batches -- LibriTTS 16, BC2013 75 split over 8 GPUs = ~10 -- the
step is entirely host-bound.  A replay costs the host ~0.1 ms, so the step takes what the GPU takes.

What is captured, per bucket (B, T_b, M_b):
  * the dropout-salt loads (``hip.load_dropout_salt``: the step-dependent part of every dropout mask is
    device data, written before each replay by ``Trainer._step_seed``, so replays draw the masks of the
    step they stand for -- bit-identical to the eager step on the same padded batch, tests/test_graphs_gpu.py);
  * ``Trainer.forward_backward``: forward, loss, backward (side-stream weight gradients included: the side
    stream forks from and joins back into the capture stream through events), every gradient left in its
    flat-arena slot.
Outside the graph, per step: the copy of the batch into the bucket's static input tensors, clip + Adam +
LR schedule (``Trainer.step_tail``: its lr / Adam step are host values), zero_grad, the loss read-out.

Buckets: the batch is padded to T_b = ceil(T / t_quant) * t_quant phonemes and M_b = ceil(M / m_quant) *
m_quant frames (masks come from the lengths, so the padded positions behave as the batch's own padding),
and the decoder / reference encoder run on the padded layout (the packed decoder's row count R varies per
batch; a graph needs fixed shapes).  Note: the PostNet BatchNorm statistics include padded frames (as in the
reference, ``model/modules.py`` PostNet over the padded batch), so their count is the bucket's M_b instead of
the batch maximum -- the same effect as a batch whose longest utterance is up to m_quant - 1 frames longer.
A bucket is captured after ``warm`` eager steps on it (workspaces, weight images and the side-stream
decisions settle first); a batch of another size (e.g. the last partial batch of an epoch) runs eagerly.
Single process only (world size 1): a multi-rank step runs eagerly (its collectives are issued from
autograd hooks).
"""
from __future__ import annotations

import time
from typing import Dict

import torch
import torch.nn.functional as F


def _ceil(x: int, q: int) -> int:
    return (int(x) + q - 1) // q * q


class GraphedSteps:
    def __init__(self, trainer, t_quant: int = 16, m_quant: int = 32, warm: int = 2, max_buckets: int = 64):
        self.tr = trainer
        self.t_quant, self.m_quant, self.warm = int(t_quant), int(m_quant), int(warm)
        self.max_buckets = int(max_buckets)
        self.buckets: Dict[tuple, dict] = {}
        self.pool = None
        self.captures = 0
        self.replays = 0
        self.eager_steps = 0
        self.capture_s = 0.0

    @staticmethod
    def supported(trainer) -> bool:
        return trainer.opt.arena.data.is_cuda and trainer.world == 1 and trainer.grad_acc == 1

    # ------------------------------------------------------------------ batch padding
    def pad_batch(self, batch):
        """-> (padded batch without host lengths -- the padded decoder / reference-encoder path --, bucket key)."""
        (ids, raw, spk, texts, src_lens, T, mels, mel_lens, M, pitch, energy, dur) = batch
        max_seq = self.tr.max_seq_len
        Tb = _ceil(T, self.t_quant)
        Mb = min(_ceil(M, self.m_quant), max(int(M), max_seq))
        dT, dM = Tb - texts.shape[1], Mb - mels.shape[1]
        texts = F.pad(texts, (0, dT)) if dT else texts
        dur = F.pad(dur, (0, dT)) if dT else dur
        mels = F.pad(mels, (0, 0, 0, dM)) if dM else mels
        # the feature level comes from the preprocess config (a shape test cannot tell when M == T)
        pre = self.tr.configs[0]["preprocessing"]
        frame_level = pre["pitch"]["feature"] == "frame_level"
        assert pre["energy"]["feature"] == pre["pitch"]["feature"], "graph steps: mixed pitch / energy levels"
        dp = dM if frame_level else dT
        if dp:
            pitch, energy = F.pad(pitch, (0, dp)), F.pad(energy, (0, dp))
        ml = mel_lens.detach().clone()  # no host_lengths attribute: the padded (unpacked) path
        key = (len(ids), Tb, Mb, frame_level)
        return (ids, raw, spk, texts, src_lens, Tb, mels, ml, Mb, pitch, energy, dur), key

    # ------------------------------------------------------------------ step
    def step(self, batch):
        tr = self.tr
        pb, key = self.pad_batch(batch)
        ent = self.buckets.get(key)
        if ent is None:
            if len(self.buckets) >= self.max_buckets:
                self.eager_steps += 1
                return tr.train_step(pb)
            ent = self.buckets[key] = {"seen": 0, "graph": None}
        if ent["graph"] is None and ent["seen"] < self.warm:
            ent["seen"] += 1
            self.eager_steps += 1
            return tr.train_step(pb)
        if not tr.model.training:
            tr.model.train()
        tr._step_seed()  # host per-op seeds (constant) + this step's device dropout salt
        from ..ops import hip

        hip.refresh_stale_images(tr.opt.arena.data.device)
        if ent["graph"] is None:
            self._capture(ent, pb)
        for dst, src in zip(ent["static"], pb):
            if isinstance(dst, torch.Tensor):
                dst.copy_(src, non_blocking=True)
        ent["graph"].replay()
        self.replays += 1
        lr = tr.step_tail(batch, True, graphed=True)
        # the static outputs live in the graph pool and the next replay of this bucket overwrites them: callers
        # get clones (a few small tensors) so nothing they keep aliases graph memory
        clone = lambda t: t.clone() if isinstance(t, torch.Tensor) else t  # noqa: E731
        return [clone(t) for t in ent["losses"]], [clone(t) for t in ent["output"]], lr

    def _capture(self, ent, pb):
        tr = self.tr
        t0 = time.perf_counter()
        static = [t.clone() if isinstance(t, torch.Tensor) else t for t in pb]
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        stream = getattr(tr, "compute_stream", None)  # None: torch's own capture stream
        from ..ops import hip

        hip.graphs_live()  # from now on grown workspaces are retired, never freed (ops/hip.py)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        # the capture stream is the trainer's compute stream (priority, side-stream forks / joins)
        with torch.cuda.graph(g, pool=self.pool, stream=stream):
            losses, output = tr.forward_backward(tuple(static))
        torch.cuda.synchronize()
        ent.update(graph=g, static=static, losses=losses, output=output)
        self.captures += 1
        self.capture_s += time.perf_counter() - t0

    def stats(self) -> dict:
        return {"buckets": len(self.buckets), "captures": self.captures, "replays": self.replays,
                "eager_steps": self.eager_steps, "capture_s": round(self.capture_s, 3)}
