"""Gradient slots: backward kernels write parameter gradients straight into the flat fp32 arena.

Without this, every fused op returns a freshly allocated weight gradient and
autograd's AccumulateGrad adds it into ``p.grad`` (the arena view): ~230 extra
fp32 add kernels + allocations per FastSpeech2 step.  With slots:

* ``FlatArena.zero_grad()`` zeroes the arena and sets every ``p.grad = None``,
  then ``reset()`` forgets the claims of the previous step;
* a backward kernel ``claim()``-s the slot of its parameter (only possible while
  ``p.grad is None`` and nobody else claimed it this step -- a parameter used
  twice in one graph gets its slot once, the second use allocates), writes the
  gradient in place (zeroed slots also serve as atomic accumulators for the
  LayerNorm / embedding reductions) and returns a fresh *view* of the slot;
* AccumulateGrad, seeing ``p.grad is None`` and a sole-owner gradient of the
  parameter's layout, adopts that view as ``p.grad`` without copying;
* ``FlatArena.finalize_grads()`` (or the DDP hook, per parameter) copies the
  few gradients that did not come from a slot (plain-torch ops) into the arena.

Contiguous parameter groups (the Q/K/V projections of one attention layer) are
laid out back to back in the arena, so the fused [3*H*dk, d] weight and its
gradient are plain views -- no ``torch.cat`` in forward, no split in backward.
"""
from __future__ import annotations

import weakref
from typing import List, Optional, Sequence

import torch

_slots = {}      # id(p) -> (weakref(p), arena, offset)
_claimed = set()


def register(p: torch.nn.Parameter, arena, offset: int):
    _slots[id(p)] = (weakref.ref(p), arena, offset)


def unregister(p: torch.nn.Parameter):
    _slots.pop(id(p), None)


def reset():
    _claimed.clear()


def _entry(p):
    e = _slots.get(id(p))
    if e is None or e[0]() is not p:
        return None
    return e


def claim(p: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """Fresh view of ``p``'s (zeroed) arena gradient slot, or None when it cannot be written in place."""
    if p is None or not isinstance(p, torch.nn.Parameter):
        return None
    e = _entry(p)
    if e is None or p.grad is not None or id(p) in _claimed:
        return None
    _claimed.add(id(p))
    arena, o = e[1], e[2]
    return arena.grad[o:o + p.numel()].view(p.shape)


def _contiguous(params: Sequence[torch.Tensor]):
    es = [_entry(p) if isinstance(p, torch.nn.Parameter) else None for p in params]
    if any(e is None for e in es) or any(e[1] is not es[0][1] for e in es):
        return None
    o = es[0][2]
    for p, e in zip(params, es):
        if e[2] != o:
            return None
        o += p.numel()
    return es[0][1], es[0][2], o - es[0][2]


def fused_data(params: Sequence[torch.Tensor]) -> Optional[torch.Tensor]:
    """[sum(rows), ...] view of the arena data spanning ``params`` (concatenated along dim 0), or None."""
    c = _contiguous(params)
    if c is None:
        return None
    arena, o, n = c
    rows = sum(p.shape[0] for p in params)
    return arena.data[o:o + n].view(rows, *params[0].shape[1:])


def claim_fused(params: Sequence[torch.Tensor]) -> Optional[torch.Tensor]:
    """Claim the slots of a contiguous group at once (all or nothing)."""
    c = _contiguous(params)
    if c is None or any(p.grad is not None or id(p) in _claimed for p in params):
        return None
    for p in params:
        _claimed.add(id(p))
    arena, o, n = c
    rows = sum(p.shape[0] for p in params)
    return arena.grad[o:o + n].view(rows, *params[0].shape[1:])


def split_rows(g: torch.Tensor, params: Sequence[torch.Tensor]) -> List[torch.Tensor]:
    out, r = [], 0
    for p in params:
        out.append(g[r:r + p.shape[0]].view(p.shape))
        r += p.shape[0]
    return out
