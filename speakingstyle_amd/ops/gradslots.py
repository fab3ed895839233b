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
_single = {}     # id(p) -> True when the last backward ended with p.grad == its slot view (one contribution)
_film_holders = {}  # tuple(id(p) of the FiLM scalars) -> FilmL2Holder
_film_of = {}       # id(scalar) -> FilmL2Holder


class FilmL2Holder:
    """Rendezvous between the concat of the FiLM scalars (s_gamma / s_beta of every LayerNorm
    site, fed to the ``lambda_f * sum(s^2)`` loss term) and the LayerNorm sites that own them.

    Each scalar has two gradient sources: the L2 term and its site.  Left to autograd that is a
    fresh gradient + an add + a copy into the arena slot per scalar (~80 tiny kernels for the 26
    scalars of a styled model).  Instead the concat's backward -- which runs first: it was recorded
    after the whole model forward -- parks the L2 gradient here and returns None, and each site's
    FiLM-gradient kernel adds its two entries while writing the scalar gradients straight into
    their slots.  Should a site run first (any other order), the concat returns plain gradients."""

    def __init__(self, params):
        self.index = {id(p): i for i, p in enumerate(params)}
        self.grad = None            # fp32 [n] L2-term gradient of this step, or None
        self.sites_started = False
        self.pending = set()        # ids of the scalars a site used in this step's forward

    def reset(self):
        self.grad = None
        self.sites_started = False

    def register_site(self, p):
        """Forward of a LayerNorm site using scalar ``p`` (grad enabled): its backward will fold the
        L2 entry in.  Scalars no site used (pitch / energy predictors run without style) get their
        L2 gradient from the concat as usual."""
        if id(p) in self.index:
            self.pending.add(id(p))

    def entry(self, p):
        """This step's L2 gradient entry of scalar ``p`` (a [1] view), or None."""
        self.sites_started = True
        if self.grad is None or p is None:
            return None
        i = self.index.get(id(p))
        return None if i is None else self.grad[i:i + 1]


def film_holder_for(params) -> FilmL2Holder:
    key = tuple(id(p) for p in params)
    h = _film_holders.get(key)
    if h is None:
        h = FilmL2Holder(params)
        _film_holders[key] = h
        for p in params:
            _film_of[id(p)] = h
    return h


def film_holder(p) -> Optional[FilmL2Holder]:
    return None if p is None else _film_of.get(id(p))


def register(p: torch.nn.Parameter, arena, offset: int):
    _slots[id(p)] = (weakref.ref(p), arena, offset)


def unregister(p: torch.nn.Parameter):
    _slots.pop(id(p), None)


_side_issued = set()  # ids of parameters whose weight gradient went to the side stream this step (hip.wgrad_async)


def mark_side(params):
    for p in params:
        if p is not None:
            _side_issued.add(id(p))


def side_issued(p) -> bool:
    """True when ``p``'s weight gradient was issued on the side stream since the last reset: only then can a
    second, main-stream contribution have raced the slot write."""
    return p is not None and id(p) in _side_issued


def reset():
    _claimed.clear()
    _side_issued.clear()
    for h in _film_holders.values():  # no L2 gradient / site registration survives into the next step
        h.reset()
        h.pending.clear()


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


def single_contribution(p) -> bool:
    """True when ``p``'s gradient was its slot view after the previous backward: autograd adopted the
    slot without summing it with another contribution (a parameter used twice -- e.g. the mel_linear
    bias, also the padded-frame fill -- gets an InputBuffer add on the main stream, which must not
    read a slot a side-stream kernel is still writing).  Unknown (first step) counts as False."""
    return p is not None and _single.get(id(p), False)


race_suspects = [0]  # steps skipped because a side-stream-eligible parameter lost its single slot view


def report_race(index: int):
    """Called by ``FlatArena.ensure_slot`` when it poisoned a possibly raced slot (step skipped on device)."""
    import warnings

    race_suspects[0] += 1
    warnings.warn(f"gradslots: parameter {index} received a second gradient contribution after being scheduled for "
                  "the weight-gradient side stream (graph changed between steps); its gradient may have raced the "
                  "side stream, so this optimizer step is skipped (non-finite guard)", RuntimeWarning)


def note_contributions(arena):
    """After a backward (all streams joined): record which parameters ended with their slot view.

    A parameter marked single here may have its next weight gradient written by the side stream.  The
    race case -- it then ends a backward with a gradient that is NOT its slot view -- is caught before the
    optimizer by ``FlatArena.ensure_slot`` (the step is skipped); this only updates the flags."""
    sp = arena._slot_ptr
    copied = getattr(arena, "copied_ids", ())
    for p in arena.params:
        g = p.grad
        _single[id(p)] = g is not None and g.data_ptr() == sp[id(p)] and id(p) not in copied


def split_rows(g: torch.Tensor, params: Sequence[torch.Tensor]) -> List[torch.Tensor]:
    out, r = [], 0
    for p in params:
        out.append(g[r:r + p.shape[0]].view(p.shape))
        r += p.shape[0]
    return out
