"""Training step / loop shared by ``train.py`` and ``bench.py``.

Per step (reference ``train.py:79-101``): forward -> loss -> (loss / grad_acc)
backward -> every ``grad_acc_step``: clip + Adam + LR schedule + zero_grad.
MI355X-specific structure:

* multi-process DP (``parallel/ddp.py``): the global valid-element counts are
  all-reduced asynchronously at the start of the step (overlapping the forward)
  and the loss divides by them; gradient buckets are all-reduced during
  backward; the fused clip+Adam kernel runs once ``finish()`` has ordered the
  compute stream after the last bucket.
* no host synchronisation inside the step: lengths needed for allocation come
  with the batch (``max_src_len``, ``max_mel_len``), loss values stay on the
  device until a ``log_step``.
* non-finite guard without sync: a non-finite global gradient norm makes the
  Adam kernel skip the update (``optimizer.skipped_steps`` counts them).
"""
from __future__ import annotations

import os
import time
from typing import Optional

import numpy as np
import torch

from ..models.loss import FastSpeech2Loss
from ..parallel import ddp
from .optim import ScheduledOptim


def side_wgrad_wanted(host_lengths, max_seq_len: int):
    """The ``experimental.side_wgrad`` decision for a step with these host mel lengths: True / False, or None
    (auto without host lengths: keep the current setting rather than sync to find out)."""
    from .. import experimental

    mode = experimental.get("side_wgrad")
    if mode != "auto":
        return mode == "1"
    if host_lengths is None:
        return None
    return int(np.minimum(host_lengths, max_seq_len).sum()) >= experimental.get("side_wgrad_min_frames")


class Trainer:
    def __init__(self, model, configs, restore_step: int = 0, bucket_mb: Optional[float] = None,
                 seed: Optional[int] = None):
        preprocess_config, model_config, train_config = configs
        self.model = model
        self.configs = configs
        self.loss_fn = FastSpeech2Loss(preprocess_config, train_config)
        self.opt = ScheduledOptim(model, train_config, model_config, restore_step)
        self.grad_acc = int(train_config["optimizer"]["grad_acc_step"])
        self.world = ddp.world_size()
        bm = bucket_mb if bucket_mb is not None else train_config.get("mi355x", {}).get("bucket_mb", 32)
        self.buckets_mb = bm
        self.buckets = ddp.GradBuckets(self.opt.arena, bm)
        self.n_mel = preprocess_config["preprocessing"]["mel"]["n_mel_channels"]
        self.max_seq_len = model_config["max_seq_len"]
        self.micro = 0
        self.last_lr = self.opt._get_lr()
        self.frames = torch.zeros((), dtype=torch.int64, device=self.opt.arena.data.device)
        self.frames_host = 0
        # dropout masks (counter-hash RNG in the HIP kernels) are seeded per micro-step from
        # (seed, rank, optimizer step, micro-step): a resumed run reproduces the masks of an
        # uninterrupted one bit for bit, with nothing extra stored in the checkpoint
        self.seed = seed
        self.rank = ddp.rank()
        import os

        from ..utils.timing import PhaseTimer

        from .. import experimental

        mi = train_config.get("mi355x", {}) or {}
        experimental.configure(mi.get("experimental"))  # also pushes the kernel-library switches
        # host timestamps of the step tail (backward return .. optimizer launch): diagnostics only
        self._host_tail = [] if experimental.get("host_tail") else None
        self._defer = experimental.get("defer_release")
        self._held = None
        # backward on the calling thread instead of autograd's per-device worker thread: no thread
        # hand-off per backward and less engine bookkeeping -- host enqueue per step 15.7 -> 12.1 ms
        # (BC2013_GST), 18.6 -> 15.1 (BC2013), 12.2 -> 10.3 (LJSpeech); profiles/r3_v10_host_lead.txt
        same = bool(mi.get("backward_same_thread", True))
        torch.autograd.set_multithreading_enabled(not same)
        self.timer = PhaseTimer(bool(mi.get("phase_timing", False)) or experimental.get("phase_timing"))

    def use_priority_stream(self, enabled: bool = True, wgrad_cu_frac: Optional[float] = None):
        """Run the step's main chain on a HIGH-priority HIP stream (made the current stream of this
        thread).  The weight gradients go to a normal-priority side stream (``ops/hip.py::wgrad_async``)
        and only fill the CUs the data-gradient chain leaves idle; with both at one priority the
        dispatcher splits CUs between them and the critical-path kernels run slower.  Call before the
        first step; tensors made earlier on the old stream are synchronised once here.

        The weight-gradient split plan is also sized for ``wgrad_cu_frac`` of the CUs: its 256x256
        blocks hold a CU's whole LDS, so a plan for every CU locks the data-gradient GEMMs out of the
        GPU until its blocks drain (LJSpeech +0.5 % at 3/4, ``profiles/r3_v10_wgrad_cus_ab.txt``).  The
        plan (and with it the split-M count, i.e. the fp32 reduction order) applies to every stream, so a
        weight gradient reduces identically whether it runs on the side stream or on the main stream (the
        first step after a resume, before the single-contribution flags are known): a resumed run
        continues bit for bit (tests/test_train_gpu.py).  Bitwise reproduction across runs therefore
        needs the same ``mi355x.stream_priority`` / ``wgrad_cu_frac`` setting; ``ssamd_wgrad_set_cus``
        can also scope the plan to one stream (switch ``wgrad_cus_all=0``)."""
        dev = self.opt.arena.data.device
        if not (enabled and dev.type == "cuda"):
            return None
        lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
        torch.cuda.synchronize(dev)
        s = torch.cuda.Stream(device=dev, priority=hi)
        torch.cuda.set_stream(s)
        self.compute_stream = s
        from .. import experimental
        from ..ops import hip

        frac = experimental.get("wgrad_cu_frac") if wgrad_cu_frac is None else wgrad_cu_frac
        if frac and frac < 1.0:
            cus = torch.cuda.get_device_properties(dev).multi_processor_count
            stream = -1 if experimental.get("wgrad_cus_all") else hip.side_stream_handle(dev)
            hip.lib().ssamd_wgrad_set_cus(stream, max(1, int(cus * frac)))
        return s

    def take_frames(self) -> int:
        """Valid mel frames consumed since the last call, summed over ranks (host sync: log steps only)."""
        f = self.frames.clone() + self.frames_host
        self.frames.zero_()
        self.frames_host = 0
        if self.world > 1:
            import torch.distributed as dist

            dist.all_reduce(f)
        return int(f)

    def reduce_losses(self, losses):
        """Host floats of the 6 loss terms of the *global* batch.

        Each rank's masked terms are its share of the global mean (they divide by the
        all-reduced valid counts), so the global value is their SUM over ranks; the
        ``lambda_f * sum(s^2)`` FiLM term is identical on every rank and is added once."""
        terms = torch.stack([l.detach().float().reshape(()) for l in losses[1:6]])
        if self.world > 1:
            import torch.distributed as dist

            dist.all_reduce(terms)
        vals = [float(v) for v in terms]
        total = sum(vals)
        named = self.model.film_scalars()
        if named is not None and self.loss_fn.lambda_f > 0:
            total += float(self.loss_fn.lambda_f * torch.sum(torch.square(named.detach().float())))
        return [total] + vals

    def _global_counts(self, batch):
        """[mel elements, phonemes, mel frames] valid in this rank's batch (device, fp32)."""
        src_lens, mel_lens = batch[4], batch[7]
        frames = mel_lens.clamp(max=self.max_seq_len).sum()
        c = torch.stack([frames * self.n_mel, src_lens.sum(), frames]).float()
        work = ddp.all_reduce_async(c)
        return c, work

    def _step_seed(self):
        """Dropout randomness of this micro-step: the per-op seeds (host LCG) start from a per-(seed, rank)
        value that does not change between steps, and the step-dependent part -- (optimizer step, micro-step)
        -- is the device dropout salt (``hip.set_dropout_salt``), so a step captured in a HIP graph
        (a captured step) replays with the masks of the step it stands for, bit-identical to the eager
        step, and a resumed run reproduces the masks of an uninterrupted one."""
        if self.seed is None or not self.opt.arena.data.is_cuda:
            return
        from ..ops import hip

        hip.set_seed((self.seed * 1000003 + self.rank) * 0x9E3779B97F4A7C15)
        hip.set_dropout_salt((self.opt.current_step * 64 + self.micro % self.grad_acc) + 1,
                             self.opt.arena.data.device)

    def _side_policy(self, batch):
        """Side-stream weight gradients for this step (``experimental.side_wgrad``): on for device-bound steps,
        off for small host-bound ones (LibriTTS batch 16: +9-11 %, BC2013 batch 10: +17 %,
        ``profiles/r5_side_stream_policy.txt``).  The split-M plan of a weight gradient does not depend on the
        stream it runs on, so the switch changes no value."""
        from .. import experimental
        from ..ops import hip

        if not self.opt.arena.data.is_cuda:
            return
        on = side_wgrad_wanted(getattr(batch[7], "host_lengths", None), self.max_seq_len)
        if on is not None:
            hip.set_wgrad_stream(on)

    def train_step(self, batch):
        tm = self.timer
        tm.phase("setup")
        if not self.model.training:  # module.train() walks every submodule: only when needed
            self.model.train()
        self._side_policy(batch)
        self._step_seed()
        counts, work = self._global_counts(batch) if self.world > 1 else (None, None)
        last_micro = (self.micro + 1) % self.grad_acc == 0
        tm.phase("forward")
        losses, output = self.forward_backward(batch, counts, work, last_micro)
        lr = self.step_tail(batch, last_micro)
        tm.stop()
        return losses, output, lr

    def forward_backward(self, batch, counts=None, work=None, last_micro=True):
        """Forward + loss + backward of one micro-step, every gradient in its arena slot at return (side
        streams joined).  Device work only after ``_step_seed``: the part a HIP graph captures
        (a captured step)."""
        tm = self.timer
        if self.opt.arena.data.is_cuda and self.seed is not None:
            from ..ops import hip

            hip.load_dropout_salt(self.opt.arena.data.device)
        output = self.model(*batch[2:])
        self._held = None  # defer_release: the previous backward's side-stream inputs
        if work is not None:
            work.wait()
        tm.phase("loss")
        named = self.model.film_scalars()
        losses = self.loss_fn(batch, output, named, global_counts=counts)
        total = losses[0]
        if self.world > 1 and named is not None and self.loss_fn.lambda_f > 0:
            # the FiLM L2 term is identical on every rank: scale so the SUM all-reduce counts it once
            total = total - (1.0 - 1.0 / self.world) * self.loss_fn.lambda_f * torch.sum(torch.square(named))
        tm.phase("backward")
        ht = self._host_tail
        if ht is not None:
            ht.append(("bwd_call", time.perf_counter()))
        if last_micro or self.world == 1:
            (total / self.grad_acc).backward()
        else:
            with self.buckets.no_sync():
                (total / self.grad_acc).backward()
        if ht is not None:
            ht.append(("bwd_return", time.perf_counter()))
        cuda = self.opt.arena.data.is_cuda
        if cuda:
            from ..ops import hip

            # weight gradients computed on the side stream; their inputs are released here (holding them
            # into the next forward measured within noise and would raise the peak by a step's activations)
            self._held = hip.join_side_streams(defer_release=self._defer)
        if ht is not None:
            ht.append(("joined", time.perf_counter()))
        self.opt.arena.finalize_grads()
        if ht is not None:
            ht.append(("finalized", time.perf_counter()))
        return losses, output

    def step_tail(self, batch, last_micro=True, graphed=False):
        """Host bookkeeping + (on the last micro-step) bucket wait, clip + Adam + LR schedule, zero_grad.
        ``graphed``: the backward was a graph replay -- its parameters' p.grad views and slot decisions are
        those of the capture, so the single-contribution bookkeeping is skipped."""
        tm = self.timer
        ht = self._host_tail
        cuda = self.opt.arena.data.is_cuda
        self.micro += 1
        hl = getattr(batch[7], "host_lengths", None)
        if hl is not None:  # host copy from the loader: no device work
            self.frames_host += int(np.minimum(hl, self.max_seq_len).sum())
        else:
            self.frames += batch[7].clamp(max=self.max_seq_len).sum()
        lr = None
        if last_micro:
            tm.phase("allreduce_wait")
            self.buckets.finish()
            tm.phase("optimizer")
            lr = self.opt.step_and_update_lr()
            if ht is not None:
                ht.append(("opt_launched", time.perf_counter()))
        if cuda and not graphed:
            # host bookkeeping for the next step AFTER the optimizer launch: the GPU runs clip + Adam
            # meanwhile instead of idling at the end of the step
            from ..ops import gradslots

            gradslots.note_contributions(self.opt.arena)  # which parameters may use their slot next step
        if last_micro:
            self.opt.zero_grad()
            self.last_lr = lr
        if ht is not None:
            ht.append(("step_end", time.perf_counter()))
        return lr

    def host_tail_summary(self):
        """Mean host ms between consecutive step-tail marks (``host_tail`` diagnostics switch), or None."""
        ht = self._host_tail
        if not ht:
            return None
        acc, n = {}, {}
        for (a, ta), (b, tb) in zip(ht, ht[1:]):
            if b == "bwd_call":
                continue  # forward + loss of the next step
            k = f"{a}->{b}"
            acc[k] = acc.get(k, 0.0) + (tb - ta) * 1e3
            n[k] = n.get(k, 0) + 1
        return {k: round(acc[k] / n[k], 3) for k in acc}
