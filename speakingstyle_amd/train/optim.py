"""Optimizer: flat fp32 parameter/gradient arenas + fused Adam + the reference LR schedules.

MI355X design:

* All trainable parameters live in ONE contiguous fp32 arena (``FlatArena``);
  each ``p.data`` / ``p.grad`` is a view into it.  That makes gradient clipping
  one reduction kernel, Adam one element-wise kernel, and DDP bucketing a set of
  contiguous slices of the gradient arena (``parallel/ddp.py``).  Parameters are
  laid out in *reverse registration order* so that the gradients produced first
  in backward sit at the start of the arena -> the first DDP bucket fills first.
* Clip + Adam run without any host synchronisation: the global norm stays on the
  device, the clip coefficient and the non-finite guard are applied inside the
  Adam kernel.
* ``state_dict()`` emits / ``load_state_dict()`` accepts the exact
  ``torch.optim.Adam`` layout indexed over ``model.parameters()`` (the reference
  checkpoint's ``"optimizer"`` entry, ``train.py:155-165``), so reference
  checkpoints resume.

LR schedule (``ScheduledOptim._get_lr``): when ``optimizer.init_lr`` is set, the
reference's linear warm-up ``init_lr -> anneal_lr`` over ``loss.anneal_steps``
followed by ``anneal_rate`` steps (``model/optimizer.py:35-44``); otherwise the
upstream FastSpeech2 Noam schedule ``d^-0.5 * min(s^-0.5, s * warm^-1.5)`` with the
same anneal steps (the reference configs without init_lr crash).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn as nn


class FlatArena:
    """Packs the given parameters into contiguous fp32 data / grad buffers.

    ``groups``: lists of parameters to place back to back in the given order (e.g.
    the Q/K/V projections of an attention layer, so the fused QKV weight and its
    gradient are views).  Each group takes the position of its first member.
    Gradients are written in place by the backward kernels (``ops/gradslots.py``);
    between steps ``p.grad`` is None.
    """

    def __init__(self, params: List[nn.Parameter], device=None, align: int = 64, groups=None):
        from ..ops import gradslots

        params = list(params)
        if groups:
            member = {}
            for gi, g in enumerate(groups):
                if all(any(q is p for p in params) for q in g):
                    for q in g:
                        member[id(q)] = gi
            ordered, done = [], set()
            for p in params:
                gi = member.get(id(p))
                if gi is None:
                    ordered.append(p)
                elif gi not in done:
                    done.add(gi)
                    ordered.extend(groups[gi])
            params = ordered
        self.params = params
        device = device or (self.params[0].device if self.params else "cpu")
        offs, n = [], 0
        for p in self.params:
            offs.append(n)
            n += (p.numel() + align - 1) // align * align  # 256-B aligned slices for vector kernels
        self.offsets = offs
        self.numel = n
        self.data = torch.zeros(n, dtype=torch.float32, device=device)
        self.grad = torch.zeros(n, dtype=torch.float32, device=device)
        self._slot_ptr = {}
        self.copied = 0  # gradients that did not arrive in their slot (diagnostics)
        self.copied_ids = set()  # this step's parameters whose gradient had to be copied into the slot
        for p, o in zip(self.params, offs):
            k = p.numel()
            self.data[o:o + k].copy_(p.detach().reshape(-1).float())
            p.data = self.data[o:o + k].view_as(p)
            p.grad = None
            gradslots.register(p, self, o)
            self._slot_ptr[id(p)] = self.grad[o:o + k].data_ptr()
        gradslots.reset()

    def slice(self, i):
        o = self.offsets[i]
        return o, o + self.params[i].numel()

    def grad_view(self, i):
        o = self.offsets[i]
        p = self.params[i]
        return self.grad[o:o + p.numel()].view_as(p)

    def zero_grad(self):
        from ..ops import gradslots

        self.grad.zero_()
        for p in self.params:
            p.grad = None
        self.copied_ids.clear()
        gradslots.reset()

    def ensure_slot(self, p, i=None):
        """Make ``p.grad`` the arena slot (copying a gradient produced outside it).

        A parameter whose weight gradient WAS written by the side stream this step
        (``gradslots.side_issued``, recorded by ``hip.wgrad_async``) but that arrives here with a gradient
        that is NOT its slot view received a second contribution summed on the main stream -- possibly
        while the side stream was still writing the slot.  Its slot is poisoned with NaN instead: the
        global-norm guard of the fused clip + Adam kernel then skips this step on the device (on every rank
        under DP: the slot is poisoned before its bucket is all-reduced), and the flag flip in
        ``note_contributions`` keeps the parameter on the main stream from the next step on.  A parameter
        whose gradient stayed on the main stream cannot have raced: its gradient is copied.  The race path
        inside a HIP-graph capture is an error (the poison would be baked into every replay)."""
        from ..ops import gradslots

        g = p.grad
        if g is None or g.data_ptr() == self._slot_ptr[id(p)]:
            return
        if i is None:
            i = next(j for j, q in enumerate(self.params) if q is p)
        slot = self.grad_view(i)
        if gradslots.side_issued(p):
            if g.is_cuda and torch.cuda.is_current_stream_capturing():
                raise RuntimeError(f"gradslots: parameter {i} raced the weight-gradient side stream during a HIP-graph "
                                   "capture; capture only after eager warm-up steps have settled the side-stream flags")
            slot.fill_(float("nan"))
            gradslots.report_race(i)
        else:
            slot.copy_(g)
        p.grad = slot
        self.copied += 1
        self.copied_ids.add(id(p))

    def finalize_grads(self):
        """After backward: every produced gradient lives in the arena."""
        sp = self._slot_ptr
        for i, p in enumerate(self.params):
            g = p.grad
            if g is not None and g.data_ptr() != sp[id(p)]:
                self.ensure_slot(p, i)

    def rebind_grads(self):
        """Re-point p.grad at the arena (e.g. before reading gradients of every parameter)."""
        self.finalize_grads()
        for i, p in enumerate(self.params):
            if p.grad is None:
                p.grad = self.grad_view(i)


class ScheduledOptim:
    def __init__(self, model: nn.Module, train_config, model_config, current_step: int = 0):
        opt = train_config["optimizer"]
        self.model = model
        self.betas = tuple(opt["betas"])
        self.eps = float(opt["eps"])
        self.weight_decay = float(opt["weight_decay"])
        self.anneal_steps = list(opt["anneal_steps"])
        self.anneal_rate = float(opt["anneal_rate"])
        self.l_anneal_steps = int(train_config["loss"]["anneal_steps"])
        self.init_lr = opt.get("init_lr")
        self.anneal_lr = opt.get("anneal_lr")
        self.n_warmup = int(opt.get("warm_up_step", 4000))
        self.noam_scale = float(model_config["transformer"]["encoder_hidden"]) ** -0.5
        self.current_step = int(current_step)
        self.grad_clip = float(opt.get("grad_clip_thresh", 0.0) or 0.0)

        self.all_params = list(model.parameters())  # torch.optim index space
        trainable = [p for p in self.all_params if p.requires_grad]
        groups = model.fused_param_groups() if hasattr(model, "fused_param_groups") else None
        self.arena = FlatArena(list(reversed(trainable)), groups=groups)
        self._index = {id(p): i for i, p in enumerate(self.all_params)}
        self.exp_avg = torch.zeros_like(self.arena.data)
        self.exp_avg_sq = torch.zeros_like(self.arena.data)
        self.step_count = 0  # Adam's t (per-parameter steps are uniform here)
        dev = self.arena.data.device
        self.last_grad_norm = torch.zeros((), device=dev)
        self.skipped_steps = torch.zeros((), device=dev, dtype=torch.int64)

    # -------------------------------------------------------------- schedule
    def _get_lr(self, step: Optional[int] = None) -> float:
        s = self.current_step if step is None else step
        if self.init_lr is not None:
            if s > self.l_anneal_steps:
                lr = float(self.anneal_lr)
                for a in self.anneal_steps:
                    if s > a:
                        lr *= self.anneal_rate
            else:
                lr = float(self.init_lr) + (s / max(self.l_anneal_steps, 1)) * (float(self.anneal_lr) - float(self.init_lr))
            return lr
        s = max(s, 1)
        lr = self.noam_scale * min(s ** -0.5, s * self.n_warmup ** -1.5)
        for a in self.anneal_steps:
            if s > a:
                lr *= self.anneal_rate
        return lr

    # -------------------------------------------------------------- API
    def zero_grad(self):
        self.arena.zero_grad()

    def step_and_update_lr(self) -> float:
        self.current_step += 1
        lr = self._get_lr()
        self.step_count += 1
        fused_adam_step(self, lr)
        return lr

    # -------------------------------------------------------------- checkpoint
    def state_dict(self) -> Dict:
        state = {}
        for p, o in zip(self.arena.params, self.arena.offsets):
            k = p.numel()
            state[self._index[id(p)]] = {
                "step": torch.tensor(float(self.step_count)),
                "exp_avg": self.exp_avg[o:o + k].view_as(p).detach().clone().cpu(),
                "exp_avg_sq": self.exp_avg_sq[o:o + k].view_as(p).detach().clone().cpu(),
            }
        group = {
            "lr": self._get_lr(), "betas": self.betas, "eps": self.eps, "weight_decay": self.weight_decay,
            "amsgrad": False, "maximize": False, "foreach": None, "capturable": False,
            "differentiable": False, "fused": None, "params": list(range(len(self.all_params))),
        }
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd: Dict):
        st = sd.get("state", {})
        steps = []
        for p, o in zip(self.arena.params, self.arena.offsets):
            s = st.get(self._index[id(p)])
            if s is None:
                continue
            k = p.numel()
            if s["exp_avg"].numel() != k:
                continue
            self.exp_avg[o:o + k].copy_(s["exp_avg"].reshape(-1).float())
            self.exp_avg_sq[o:o + k].copy_(s["exp_avg_sq"].reshape(-1).float())
            steps.append(float(s["step"]))
        if steps:
            self.step_count = int(max(steps))


def fused_adam_step(opt: ScheduledOptim, lr: float):
    """Global-norm clip + Adam over the flat arena; no host sync."""
    a = opt.arena
    if a.data.is_cuda:
        from ..ops import hip

        fresh = hip.clip_adam_step(a.data, a.grad, opt.exp_avg, opt.exp_avg_sq, lr, opt.betas, opt.eps,
                                   opt.weight_decay, opt.step_count, opt.grad_clip, opt.last_grad_norm,
                                   opt.skipped_steps)
        hip.bump_weight_generation()  # raw-pointer writes: torch version counters do not move
        hip.stamp_images(fresh)  # images rewritten by the same launch: no weight_prep refresh
        return
    g = a.grad
    norm = torch.linalg.vector_norm(g)
    opt.last_grad_norm.copy_(norm)
    finite = torch.isfinite(norm)
    if not bool(finite):
        opt.skipped_steps += 1
        return
    if opt.grad_clip > 0:
        coef = torch.clamp(opt.grad_clip / (norm + 1e-6), max=1.0)
        g = g * coef
    if opt.weight_decay:
        g = g + opt.weight_decay * a.data
    b1, b2 = opt.betas
    t = opt.step_count
    opt.exp_avg.mul_(b1).add_(g, alpha=1 - b1)
    opt.exp_avg_sq.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - b1 ** t
    bc2 = 1 - b2 ** t
    denom = (opt.exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(opt.eps)
    a.data.addcdiv_(opt.exp_avg, denom, value=-lr / bc1)
