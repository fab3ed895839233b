#!/usr/bin/env python
"""Headline benchmark: FastSpeech2 training throughput in mel-frames/s (node).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it
is launched by torch.distributed.run with one rank per GPU (RCCL over xGMI).
W untimed warm-up steps, then exactly K full training steps (forward + loss +
backward + bucketed gradient all-reduce + clip + Adam + LR schedule) bracketed
by barrier + device synchronise on both sides; the time is the MAX over ranks;
rank 0 prints one JSON line.

Config = BASELINE.json's headline: LJSpeech FastSpeech2 (model.yaml shape: 4+6
FFT blocks, d=256, no style encoder), bf16 compute with fp32 master weights /
Adam state, synthetic LJSpeech-shaped data (phoneme counts drawn from the real
LJSpeech metadata, ~8.1 frames per phoneme, groups of 4 batches sorted by text
length exactly like the reference loader), random-init weights.  Scaling is
weak: every rank runs ``--batch`` utterances (default: the config's
``optimizer.batch_size`` = 200), so the global batch is N*200.
``value`` = total valid mel frames consumed by the K timed steps over all ranks
divided by the max-over-ranks wall time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_FRAMES_PER_S = 2.5e4  # derived GTX-1080Ti lower bound (train mel-frames/s)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="LJSpeech")
    ap.add_argument("--batch", type=int, default=None, help="utterances per GPU (default: config batch_size)")
    ap.add_argument("--pool", type=int, default=8, help="distinct synthetic batches cycled through")
    ap.add_argument("--backend", default=None, choices=[None, "hip", "reference"])
    ap.add_argument("--profile-steps", type=int, default=0)
    args = ap.parse_args()
    # variable-shape batches: let the caching allocator grow segments instead of re-mallocing
    os.environ.setdefault("PYTORCH_HIP_ALLOC_CONF", "expandable_segments:True")
    os.environ.setdefault("PYTORCH_CUDA_ALLOC_CONF", "expandable_segments:True")

    import torch

    from speakingstyle_amd import ops
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.parallel import ddp
    from speakingstyle_amd.train.trainer import Trainer

    if args.backend:
        ops.set_backend(args.backend)
    rank, world, local_rank = ddp.init_distributed()
    cuda = torch.cuda.is_available()
    device = torch.device("cuda", local_rank) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(device)
    pp, mc, tc = load_named(args.config)
    batch = args.batch or int(tc["optimizer"]["batch_size"])
    torch.manual_seed(1234)
    model = FastSpeech2(pp, mc).to(device)
    model.set_compute_dtype(torch.bfloat16 if cuda else torch.float32)
    ddp.broadcast_module_state(model)
    trainer = Trainer(model, (pp, mc, tc))

    gen = SyntheticBatches(batch, device=device, max_seq_len=mc["max_seq_len"], seed=1000 + rank,
                           frame_level=pp["preprocessing"]["pitch"]["feature"] == "frame_level")
    pool = []
    for _ in range(args.pool):
        b = gen.make_batch()
        pool.append((b, gen.last_valid_frames))
    # largest padded batch first: the first warm-up step sizes the allocator for all others
    pool.sort(key=lambda e: -(e[0][0].__len__() * e[0][8]))

    def step(i):
        b, frames = pool[i % len(pool)]
        trainer.train_step(b)
        return frames

    for i in range(args.warmup):
        step(i)
    if cuda:
        torch.cuda.synchronize()
    ddp.barrier()
    if cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    frames = 0
    for i in range(args.steps):
        frames += step(args.warmup + i)
    if cuda:
        torch.cuda.synchronize()
    ddp.barrier()
    if cuda:
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    stats = torch.tensor([elapsed, float(frames)], dtype=torch.float64, device=device)
    if world > 1:
        import torch.distributed as dist

        t_max = stats[0:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        f_sum = stats[1:2].clone()
        dist.all_reduce(f_sum, op=dist.ReduceOp.SUM)
        elapsed, frames = float(t_max.item()), float(f_sum.item())
    value = frames / elapsed
    if rank == 0:
        print(json.dumps({
            "metric": "train mel-frames/sec (node)",
            "value": round(value, 1),
            "unit": "mel-frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_FRAMES_PER_S, 3),
            "dtype": "bf16" if cuda else "fp32",
            "data": "synthetic (LJSpeech-shaped lengths, random-init weights)",
            "config": {
                "model": f"FastSpeech2 ({args.config} model.yaml)",
                "global_batch": batch * world,
                "seq_len": "T~LJSpeech phonemes, M<=1000 mel frames",
                "parallelism": f"dp{world}",
            },
        }), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
