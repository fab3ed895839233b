"""Training loop (reference ``train.py:21-173``) on top of ``Trainer``.

Same cadence and outputs as the reference: ``log_step`` -> ``log/train/log.txt`` +
TensorBoard scalars ``Loss/*``, ``Weight/learning_rate``, ``Weight/lambda_f``;
``synth_step`` -> mel figure + reconstructed / synthesized audio; ``val_step`` ->
``evaluate``; ``save_step`` -> ``{step}.pth.tar``; stop at ``total_step``.

Added: one process per GPU (torchrun env), per-phase throughput
scalars (``Perf/mel_frames_per_s``, ``Perf/step_ms``), SIGTERM -> checkpoint
(SLURM preemption), ``--auto_resume`` from the latest checkpoint (HiFi-GAN-style),
non-finite steps skipped on the device and reported, synthetic-data mode for
plumbing runs without a preprocessed corpus, fault injection for resume tests.
"""
from __future__ import annotations

import os
import signal
import sys
import time
from typing import Optional

import numpy as np
import torch
from torch.utils.data import DataLoader

from ..data.dataset import Dataset, to_device
from ..data.synthetic import SyntheticBatches
from ..parallel import ddp
from ..utils import model as mutil
from ..utils.logging import log_scalars, synth_one_sample
from ..utils.tb import SummaryWriter
from .trainer import Trainer


def _batches(configs, device, rank, world, synthetic: bool, seed: int, pos=None):
    """Yields (epoch, group_index, [batches]); one item = one global group of
    ``group`` length-sorted batches, this rank's shard of each.  ``pos`` =
    (epoch, groups consumed) resumes the data order exactly where a checkpoint left it.

    Batch semantics (``mi355x.frames_per_gpu``):
    * unset (reference ``train.py:27-45``): ``optimizer.batch_size`` is the GLOBAL batch, split
      over the ranks (each gets ``batch_size / world`` utterances of every sorted batch);
    * set: every rank gets its own batch of up to ``frames_per_gpu`` padded mel frames
      (``FrameBudgetSampler``), so the per-GPU shape is sized for HBM and the global batch grows
      with the world size; one item = one global step."""
    preprocess_config, model_config, train_config = configs
    bs = int(train_config["optimizer"]["batch_size"])
    mi = train_config.get("mi355x", {}) or {}
    budget = mi.get("frames_per_gpu")
    max_len = int(model_config["max_seq_len"])
    if synthetic:
        if not budget and bs < world:
            raise ValueError(f"batch_size={bs} < world size {world}: set mi355x.frames_per_gpu or a larger batch")
        per_rank = max(1, bs // world)
        gen = SyntheticBatches(per_rank, device=device, max_seq_len=max_len, seed=seed + rank,
                               n_speakers=_n_speakers(preprocess_config), frames_per_batch=budget or None,
                               frame_level=preprocess_config["preprocessing"]["pitch"]["feature"] == "frame_level")
        # one group = one batch; every group re-seeds the stream from (seed + rank, group index), so a
        # resume at the checkpoint's data position continues with exactly the batches that were next
        gi = int(pos[1]) if pos else 0
        while True:
            gen.seek(gi)
            yield 0, gi, [gen.make_batch()]
            gi += 1
    from ..data.dataset import FrameBudgetSampler, ShardedGroupSampler

    dataset = Dataset("train.txt", preprocess_config, train_config, sort=True, drop_last=True)
    group = 4
    if not budget:
        assert bs * group < len(dataset), "batch_size * group_size must be < dataset size"
    epoch, start = pos if pos else (0, 0)
    while True:
        if budget:
            sampler = FrameBudgetSampler(dataset, int(budget), rank, world, seed=seed, epoch=epoch, start=start,
                                         max_seq_len=max_len, max_batch=mi.get("max_batch_per_gpu"))
        else:
            sampler = ShardedGroupSampler(dataset, bs, group, rank, world, seed=seed, epoch=epoch, start=start)
        loader = DataLoader(dataset, batch_sampler=sampler, collate_fn=dataset.collate_local,
                            num_workers=int(mi.get("num_workers", 4)),
                            pin_memory=torch.cuda.is_available())
        for gi, batchs in enumerate(loader, start=start):
            yield epoch, gi, [to_device(b, device) for b in batchs]
        epoch, start = epoch + 1, 0


def _n_speakers(preprocess_config):
    import json

    p = os.path.join(preprocess_config["path"]["preprocessed_path"], "speakers.json")
    if os.path.exists(p):
        with open(p) as f:
            return len(json.load(f))
    return 1


def train(args, configs):
    preprocess_config, model_config, train_config = configs
    rank, world, local_rank = ddp.init_distributed()
    cuda = torch.cuda.is_available() and not getattr(args, "cpu", False)
    device = torch.device("cuda", local_rank) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(device)
    seed = int(getattr(args, "seed", None) or train_config.get("mi355x", {}).get("seed", 1234))
    torch.manual_seed(seed)
    np.random.seed(seed)
    if cuda:
        from ..ops import hip

        hip.set_seed(seed * 1000003 + rank)

    restore = int(args.restore_step or 0)
    if getattr(args, "auto_resume", False) and not restore:
        restore = mutil.latest_step(train_config)
    mi = train_config.get("mi355x", {}) or {}
    if cuda and (not mi.get("hip_kernels", True) or mi.get("dtype", "bf16") == "fp32"):
        from .. import ops

        ops.set_backend("reference")  # torch ops on the GPU (fp32 oracle runs / A-B debugging)
    model = mutil.FastSpeech2(preprocess_config, model_config).to(device)
    model.set_compute_dtype(torch.bfloat16 if (cuda and mi.get("dtype", "bf16") == "bf16") else torch.float32)
    ckpt = None
    if restore:
        ckpt = mutil.load_checkpoint(mutil.ckpt_file(train_config, restore))
        mutil.restore_model(model, ckpt, train_config.get("ignore_layers", []))
    ddp.broadcast_module_state(model)
    trainer = Trainer(model, configs, restore_step=restore, seed=seed)
    trainer.use_priority_stream(cuda and (train_config.get("mi355x", {}) or {}).get("stream_priority", "high") == "high")
    if ckpt is not None and "optimizer" in ckpt:
        trainer.opt.load_state_dict(ckpt["optimizer"])
    if ckpt is not None and isinstance(ckpt.get("rng"), torch.Tensor) and not cuda:
        torch.set_rng_state(ckpt["rng"])  # CPU dropout (torch RNG); the GPU masks are step-seeded
    if rank == 0:
        print("Number of FastSpeech2 Parameters:", mutil.get_param_num(model), flush=True)

    vocoder = None
    if rank == 0 and not getattr(args, "no_vocoder", False):
        vocoder = mutil.get_vocoder(model_config, device)

    paths = train_config["path"]
    train_log_path = os.path.join(paths["log_path"], "train")
    val_log_path = os.path.join(paths["log_path"], "val")
    train_logger = val_logger = None
    if rank == 0:
        for p in paths.values():
            os.makedirs(p, exist_ok=True)
        os.makedirs(train_log_path, exist_ok=True)
        os.makedirs(val_log_path, exist_ok=True)
        train_logger = SummaryWriter(train_log_path)
        val_logger = SummaryWriter(val_log_path)

    st = train_config["step"]
    total_step = int(getattr(args, "max_steps", None) or st["total_step"])
    log_step, save_step, synth_step, val_step = st["log_step"], st["save_step"], st["synth_step"], st["val_step"]
    fail_at = int(getattr(args, "fail_at_step", 0) or 0)

    state = {"step": restore}
    pos0 = ckpt.get("data_pos") if ckpt is not None else None  # (epoch, group, batches done in group)
    check_every = int(train_config.get("mi355x", {}).get("preempt_check_steps", 10))

    def save(step, pos):
        if rank == 0:
            mutil.save_checkpoint(mutil.ckpt_file(train_config, step), model, trainer.opt, step,
                                  extra={"rng": torch.get_rng_state(), "data_pos": list(pos)})

    # SIGTERM (SLURM preemption) on ANY rank sets a flag; ranks agree on it at a step
    # boundary (every ``preempt_check_steps`` under DP: one tiny all-reduce), then rank 0
    # saves and everybody leaves the loop together -- no rank is left inside a collective.
    flag = {"term": False}

    def on_term(signum, frame):
        flag["term"] = True

    prev = signal.signal(signal.SIGTERM, on_term)

    def preempted(step):
        if world == 1:
            return flag["term"]
        if step % check_every:
            return False
        t = torch.tensor([1.0 if flag["term"] else 0.0], device=device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        return bool(t.item() > 0)

    step = restore + 1
    bs_global = int(train_config["optimizer"]["batch_size"])
    t_last = time.perf_counter()
    synthetic = getattr(args, "synthetic", False) or not os.path.exists(
        os.path.join(preprocess_config["path"]["preprocessed_path"], "train.txt"))
    start_pos = (pos0[0], pos0[1]) if pos0 else None
    skip = int(pos0[2]) if pos0 else 0
    try:
        for epoch, gi, batchs in _batches(configs, device, rank, world, synthetic, seed, start_pos):
            for k, batch in enumerate(batchs):
                if skip:  # resumed inside a group: these batches were consumed before the checkpoint
                    skip -= 1
                    continue
                if fail_at and step == fail_at:
                    raise RuntimeError(f"fault injection at step {step}")
                losses, output, lr = trainer.train_step(batch)
                if step == restore + 1:  # per-rank batch shape of the first step (DP batch semantics)
                    budget = (train_config.get("mi355x") or {}).get("frames_per_gpu")
                    rule = f"frames_per_gpu={budget}" if budget else f"batch_size/world={bs_global}/{world}"
                    print(f"[rank {rank}] first batch: {len(batch[0])} utterances, {len(batch[0]) * int(batch[8])} "
                          f"padded mel frames ({rule})", flush=True)
                # position AFTER this batch: the next run starts at the following batch
                pos = (epoch, gi + 1, 0) if k + 1 == len(batchs) else (epoch, gi, k + 1)
                if step % log_step == 0:
                    vals = trainer.reduce_losses(losses)  # collective on every rank
                    frames = trainer.take_frames()
                    dt = time.perf_counter() - t_last
                    t_last = time.perf_counter()
                    if rank == 0:
                        msg1 = "Step {}/{}, ".format(step, total_step)
                        msg2 = ("Total Loss: {:.4f}, Mel Loss: {:.4f}, Mel PostNet Loss: {:.4f}, Pitch Loss: {:.4f}, "
                                "Energy Loss: {:.4f}, Duration Loss: {:.4f}").format(*vals)
                        with open(os.path.join(train_log_path, "log.txt"), "a") as f:
                            f.write(msg1 + msg2 + "\n")
                        print(msg1 + msg2, flush=True)
                        log_scalars(train_logger, step, losses=vals, lr=trainer.last_lr, lambdas=losses[-1])
                        train_logger.add_scalar("Perf/step_ms", 1000.0 * dt / log_step, step)
                        train_logger.add_scalar("Perf/mel_frames_per_s", frames / max(dt, 1e-9), step)
                        train_logger.add_scalar("Perf/skipped_steps", float(trainer.opt.skipped_steps), step)
                        for ph, v in trainer.timer.summary().items():  # empty unless phase timing is on
                            train_logger.add_scalar(f"Perf/phase_{ph}_host_ms", v["host_ms"], step)
                            train_logger.add_scalar(f"Perf/phase_{ph}_device_ms", v["device_ms"], step)
                if rank == 0 and synth_step and step % synth_step == 0:
                    synth_one_sample(batch, output, vocoder, model_config, preprocess_config, train_logger, step, "Training")
                if val_step and step % val_step == 0 and not synthetic:
                    from ..train.evaluate import evaluate

                    model.eval()
                    msg = evaluate(model, step, configs, val_logger if rank == 0 else None, vocoder)
                    if rank == 0:
                        with open(os.path.join(val_log_path, "log.txt"), "a") as f:
                            f.write(msg + "\n")
                        print(msg, flush=True)
                    model.train()
                if save_step and step % save_step == 0:
                    save(step, pos)
                state["step"] = step
                if step >= total_step:
                    return step
                if preempted(step):
                    save(step, pos)
                    if rank == 0:
                        print(f"SIGTERM: checkpoint saved at step {step}", flush=True)
                    return step
                step += 1
    finally:
        signal.signal(signal.SIGTERM, prev)
        for lg in (train_logger, val_logger):
            if lg is not None:
                lg.close()
