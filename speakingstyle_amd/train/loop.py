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


class _Preempted(Exception):
    pass


def _batches(configs, device, rank, world, synthetic: bool, seed: int):
    """Yields lists of batches (one DataLoader item = group_size sorted batches)."""
    preprocess_config, model_config, train_config = configs
    bs = int(train_config["optimizer"]["batch_size"])
    if synthetic:
        per_rank = max(1, bs // world)
        gen = SyntheticBatches(per_rank, device=device, max_seq_len=model_config["max_seq_len"], seed=seed + rank,
                               n_speakers=_n_speakers(preprocess_config),
                               frame_level=preprocess_config["preprocessing"]["pitch"]["feature"] == "frame_level")
        while True:
            yield [gen.make_batch()]
    dataset = Dataset("train.txt", preprocess_config, train_config, sort=True, drop_last=True, shard=(rank, world))
    group = 4
    assert bs * group < len(dataset), "batch_size * group_size must be < dataset size"
    epoch = 0
    while True:
        g = torch.Generator().manual_seed(seed + epoch)  # identical shuffle on every rank
        loader = DataLoader(dataset, batch_size=bs * group, shuffle=True, generator=g, collate_fn=dataset.collate_fn,
                            num_workers=int(train_config.get("mi355x", {}).get("num_workers", 4)),
                            pin_memory=torch.cuda.is_available(), drop_last=True)
        for batchs in loader:
            yield [to_device(b, device) for b in batchs]
        epoch += 1


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
    model, _opt_unused = None, None
    model = mutil.FastSpeech2(preprocess_config, model_config).to(device)
    model.set_compute_dtype(torch.bfloat16 if cuda else torch.float32)
    ckpt = None
    if restore:
        ckpt = mutil.load_checkpoint(mutil.ckpt_file(train_config, restore))
        mutil.restore_model(model, ckpt, train_config.get("ignore_layers", []))
    ddp.broadcast_module_state(model)
    trainer = Trainer(model, configs, restore_step=restore)
    if ckpt is not None and "optimizer" in ckpt:
        trainer.opt.load_state_dict(ckpt["optimizer"])
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

    def save(step):
        if rank == 0:
            mutil.save_checkpoint(mutil.ckpt_file(train_config, step), model, trainer.opt, step,
                                  extra={"rng": torch.get_rng_state()})

    def on_term(signum, frame):
        raise _Preempted()

    prev = signal.signal(signal.SIGTERM, on_term) if rank == 0 or world == 1 else None
    step = restore + 1
    frames_acc = 0
    t_last = time.perf_counter()
    synthetic = getattr(args, "synthetic", False) or not os.path.exists(
        os.path.join(preprocess_config["path"]["preprocessed_path"], "train.txt"))
    try:
        for batchs in _batches(configs, device, rank, world, synthetic, seed):
            for batch in batchs:
                if fail_at and step == fail_at:
                    raise RuntimeError(f"fault injection at step {step}")
                losses, output, lr = trainer.train_step(batch)
                frames_acc += int(batch[7].clamp(max=model_config["max_seq_len"]).sum()) if step % log_step == 0 else 0
                if rank == 0 and step % log_step == 0:
                    vals = [float(l) for l in losses[:-1]]
                    dt = time.perf_counter() - t_last
                    t_last = time.perf_counter()
                    msg1 = "Step {}/{}, ".format(step, total_step)
                    msg2 = ("Total Loss: {:.4f}, Mel Loss: {:.4f}, Mel PostNet Loss: {:.4f}, Pitch Loss: {:.4f}, "
                            "Energy Loss: {:.4f}, Duration Loss: {:.4f}").format(*vals)
                    with open(os.path.join(train_log_path, "log.txt"), "a") as f:
                        f.write(msg1 + msg2 + "\n")
                    print(msg1 + msg2, flush=True)
                    log_scalars(train_logger, step, losses=vals, lr=trainer.last_lr, lambdas=losses[-1])
                    train_logger.add_scalar("Perf/step_ms", 1000.0 * dt / log_step, step)
                    train_logger.add_scalar("Perf/skipped_steps", float(trainer.opt.skipped_steps), step)
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
                    save(step)
                state["step"] = step
                if step >= total_step:
                    return step
                step += 1
    except _Preempted:
        save(state["step"])
        print(f"SIGTERM: checkpoint saved at step {state['step']}", flush=True)
        return state["step"]
    finally:
        if prev is not None:
            signal.signal(signal.SIGTERM, prev)
        for lg in (train_logger, val_logger):
            if lg is not None:
                lg.close()
