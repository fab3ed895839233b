"""Data parallelism: one process per GPU, RCCL all-reduce over xGMI of contiguous
gradient buckets, overlapped with backward.

Replaces the reference's single-process ``nn.DataParallel`` (``train.py:45``:
scatter / replicate-broadcast / gather + reduce to cuda:0 every step, SURVEY
§2.5 C1-C4) and HiFi-GAN's DDP (``hifigan/train.py:58-61``).

Design (MI355X-first):

* Gradients already live in one flat fp32 arena (``train/optim.py``), laid out
  in reverse registration order ~= backward production order.  A bucket is a
  contiguous slice of that arena -- no copy-in/copy-out, the collective runs on
  the arena memory directly.
* Each parameter carries a post-accumulate-grad hook; when the last parameter of
  a bucket has its gradient, the bucket's ``all_reduce(SUM)`` is issued
  asynchronously.  With the ``nccl`` backend (= RCCL on ROCm) the collective runs
  on RCCL's internal stream after an event wait on the compute stream, so it
  overlaps the rest of backward.  ``finish()`` makes the compute stream wait for
  all buckets before the fused clip+Adam kernel reads the arena.
* Buckets default to 32 MiB: the LJSpeech model's 140 MB of fp32 gradients
  become 5 buckets -- large enough that each ring all-reduce runs near the
  per-link xGMI bandwidth, small enough that the first bucket launches early
  in backward (the decoder/PostNet grads arrive first).
* Parameters that receive no gradient in a step (e.g. the pitch/energy FiLM
  scalars, which the reference never applies -- SURVEY D7) leave their bucket
  incomplete; ``finish()`` launches any such bucket at the end.
* Loss normalisation uses *global* valid-element counts (all-reduced at step
  start, see ``models/loss.py``), so summed gradients equal the single-process
  full-batch gradient exactly; no 1/world rescale is needed.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist


def init_distributed(backend: Optional[str] = None):
    """torchrun-style env init.  Returns (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local_rank


def world_size() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def barrier():
    if world_size() > 1:
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


class GradBuckets:
    """Bucketed, backward-overlapped gradient all-reduce over a FlatArena."""

    def __init__(self, arena, bucket_mb: float = 32.0, group=None):
        self.arena = arena
        self.group = group
        self.world = world_size()
        cap = max(1, int(bucket_mb * 1024 * 1024 // 4))
        self.buckets: List[tuple] = []  # (start, end, n_params)
        self.param_bucket = {}
        self.param_index = {id(p): i for i, p in enumerate(arena.params)}
        start = 0
        members = 0
        cur_end = 0
        for i, p in enumerate(arena.params):
            s, e = arena.slice(i)
            e_al = arena.offsets[i + 1] if i + 1 < len(arena.params) else arena.numel
            if members and (e_al - start) > cap:
                self.buckets.append([start, cur_end, members])
                start, members = s, 0
            self.param_bucket[id(p)] = len(self.buckets)
            members += 1
            cur_end = e_al
        if members:
            self.buckets.append([start, cur_end, members])
        self.pending = [b[2] for b in self.buckets]
        self.works: List[Optional[object]] = [None] * len(self.buckets)
        self.enabled = True
        self._handles = []
        if self.world > 1:
            for p in arena.params:
                self._handles.append(p.register_post_accumulate_grad_hook(self._hook))

    def _launch(self, bi):
        s, e, _ = self.buckets[bi]
        self.works[bi] = dist.all_reduce(self.arena.grad[s:e], op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def _hook(self, p):
        if not self.enabled:
            return
        self.arena.ensure_slot(p, self.param_index[id(p)])  # gradients from plain-torch ops: into the bucket
        bi = self.param_bucket[id(p)]
        self.pending[bi] -= 1
        if self.pending[bi] == 0 and self.works[bi] is None:
            self._launch(bi)

    def finish(self):
        """Launch stragglers, make the current stream wait for every bucket, reset."""
        if self.world <= 1:
            return
        for bi in range(len(self.buckets)):
            if self.works[bi] is None:
                self._launch(bi)
        for w in self.works:
            w.wait()
        self.works = [None] * len(self.buckets)
        self.pending = [b[2] for b in self.buckets]

    def no_sync(self):
        """Context for gradient-accumulation micro-steps (no collectives)."""
        outer = self

        class _Ctx:
            def __enter__(self):
                outer.enabled = False

            def __exit__(self, *a):
                outer.enabled = True
                outer.pending = [b[2] for b in outer.buckets]

        return _Ctx()


def broadcast_module_state(module: torch.nn.Module, src: int = 0):
    """Make every rank start from rank ``src``'s parameters and buffers."""
    if world_size() <= 1:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src)
    from ..ops import hip  # ``.data`` writes bypass version counters: cached bf16 images are stale

    hip.bump_weight_generation()


def all_reduce_async(t: torch.Tensor):
    if world_size() <= 1:
        return None
    return dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)
