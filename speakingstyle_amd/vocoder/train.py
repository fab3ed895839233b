"""HiFi-GAN vocoder training (reference ``hifigan/train.py:23-233``).

One process per GPU (torchrun env; RCCL all-reduce via torch DDP over the generator and both
discriminators, as the reference), AdamW + ExponentialLR per epoch, loss = mel-L1 x45 +
feature matching + LSGAN (reference ``hifigan/models.py:234-264``), checkpoints
``g_{steps:08d}`` / ``do_{steps:08d}`` with auto-resume from the latest pair, the run's
``config.json`` copied into the checkpoint directory (reference ``env.py`` build_env).

Logging (rank 0): stdout every ``stdout_interval`` steps (gen loss, mel error, s/b);
TensorBoard ``training/gen_loss_total``, ``training/mel_spec_error`` every
``summary_interval``; validation every ``validation_interval`` steps over the validation
list (whole utterances, batch 1): ``validation/mel_spec_error`` plus audio / spectrogram
figures of the first 5 items (``gt/*`` at step 0, ``generated/*``).

``fine_tuning``: inputs are ground-truth-aligned mels from ``input_mels_dir`` (the acoustic
model's teacher-forced output), reference ``meldataset.py:142-159``.
"""
from __future__ import annotations

import glob
import itertools
import json
import os
import shutil
import time

import torch
import torch.nn.functional as F

from ..models import hifigan as H
from ..parallel import ddp
from ..utils.model import vocoder_config
from ..utils.tb import SummaryWriter
from .data import MelDataset, get_dataset_filelist
from .mel import mel_for


def latest(path: str, prefix: str):
    cps = sorted(glob.glob(os.path.join(path, prefix + "????????")))
    return cps[-1] if cps else None


def _log_spec(sw, tag, spec, step):
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    fig, ax = plt.subplots(figsize=(10, 2))
    ax.imshow(spec, aspect="auto", origin="lower", interpolation="none")
    fig.tight_layout()
    sw.add_figure(tag, fig, step)
    plt.close(fig)


def _unwrap(m):
    return m.module if hasattr(m, "module") else m


def train(a):
    h = vocoder_config(a.config)
    if a.batch_size:
        h.batch_size = a.batch_size
    rank, world, local_rank = ddp.init_distributed()
    cuda = torch.cuda.is_available() and not getattr(a, "cpu", False)
    dev = torch.device("cuda", local_rank) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(dev)
    torch.manual_seed(h.seed + rank)
    os.makedirs(a.checkpoint_path, exist_ok=True)
    if rank == 0:
        cfg_out = os.path.join(a.checkpoint_path, "config.json")
        if a.config and os.path.abspath(a.config) != os.path.abspath(cfg_out):
            shutil.copyfile(a.config, cfg_out)
        elif not os.path.exists(cfg_out):
            with open(cfg_out, "w") as f:
                json.dump(dict(h), f, indent=2)

    gen = H.Generator(h).to(dev)
    mpd = H.MultiPeriodDiscriminator().to(dev)
    msd = H.MultiScaleDiscriminator().to(dev)
    steps, last_epoch = 0, -1
    cp_g, cp_do = latest(a.checkpoint_path, "g_"), latest(a.checkpoint_path, "do_")
    state_do = None
    if cp_g and cp_do:
        gen.load_state_dict(torch.load(cp_g, map_location=dev, weights_only=True)["generator"])
        state_do = torch.load(cp_do, map_location=dev, weights_only=True)
        mpd.load_state_dict(state_do["mpd"])
        msd.load_state_dict(state_do["msd"])
        steps, last_epoch = state_do["steps"] + 1, state_do["epoch"]
    # GPU: the discriminators, losses and STFT run on the HIP kernels (vocoder/hip_train.py, explicit
    # forward + backward); torch modules otherwise
    use_hip = cuda and H._hip_train() and not getattr(a, "torch_losses", False)
    if world > 1:
        ids = [local_rank] if cuda else None
        gen = torch.nn.parallel.DistributedDataParallel(gen, device_ids=ids)
        if not use_hip:  # HIP path: the discriminator gradients are all-reduced as one flat buffer
            mpd = torch.nn.parallel.DistributedDataParallel(mpd, device_ids=ids)
            msd = torch.nn.parallel.DistributedDataParallel(msd, device_ids=ids)
    opt_g = torch.optim.AdamW(gen.parameters(), h.learning_rate, betas=(h.adam_b1, h.adam_b2))
    opt_d = torch.optim.AdamW(itertools.chain(msd.parameters(), mpd.parameters()), h.learning_rate,
                              betas=(h.adam_b1, h.adam_b2))
    if state_do is not None:
        opt_g.load_state_dict(state_do["optim_g"])
        opt_d.load_state_dict(state_do["optim_d"])
    sch_g = torch.optim.lr_scheduler.ExponentialLR(opt_g, gamma=h.lr_decay, last_epoch=last_epoch)
    sch_d = torch.optim.lr_scheduler.ExponentialLR(opt_d, gamma=h.lr_decay, last_epoch=last_epoch)

    synthetic = a.synthetic or not (os.path.exists(a.input_training_file) and os.path.isdir(a.input_wavs_dir))
    if synthetic:
        train_files, valid_files = [], []
    else:
        train_files, valid_files = get_dataset_filelist(a.input_training_file, a.input_validation_file,
                                                        a.input_wavs_dir)
    trainset = MelDataset(train_files, h, shuffle=world == 1, fine_tuning=a.fine_tuning,
                          base_mels_path=a.input_mels_dir, synthetic_n=64 if synthetic else 0, seed=h.seed)
    sampler = torch.utils.data.distributed.DistributedSampler(trainset) if world > 1 else None
    bs = max(1, int(h.batch_size) // world)  # reference: global batch split over the GPUs
    loader = torch.utils.data.DataLoader(trainset, batch_size=bs, shuffle=False, sampler=sampler, drop_last=True,
                                         num_workers=int(a.num_workers), pin_memory=cuda)
    sw = valid_loader = None
    if rank == 0:
        validset = MelDataset(valid_files, h, split=False, shuffle=False, fine_tuning=a.fine_tuning,
                              base_mels_path=a.input_mels_dir, synthetic_n=4 if synthetic else 0)
        valid_loader = torch.utils.data.DataLoader(validset, batch_size=1, shuffle=False, num_workers=0)
        sw = SummaryWriter(os.path.join(a.checkpoint_path, "logs"))

    gen.train(); mpd.train(); msd.train()
    try:
        # the checkpoint's epoch is the one it was written in: resume INSIDE it (reference
        # ``hifigan/train.py:105``), so the ExponentialLR decay stays aligned with an uninterrupted run
        for epoch in range(max(0, last_epoch), a.training_epochs):
            t_ep = time.time()
            if sampler is not None:
                sampler.set_epoch(epoch)
            for x, y, _, y_mel in loader:
                t_b = time.time()
                x, y, y_mel = x.to(dev, non_blocking=True), y.to(dev, non_blocking=True), y_mel.to(dev, non_blocking=True)
                y = y.unsqueeze(1)
                y_g = gen(x)
                if use_hip:
                    loss_g, loss_mel = hip_step(h, mpd, msd, opt_d, opt_g, y.squeeze(1), y_g.squeeze(1), y_mel, world)
                else:
                    loss_g, loss_mel = torch_step(h, mpd, msd, opt_d, opt_g, y, y_g, y_mel)
                if rank == 0:
                    mel_err = float(loss_mel) / 45
                    if steps % a.stdout_interval == 0:
                        print(f"Steps : {steps:d}, Gen Loss Total : {float(loss_g):4.3f}, Mel-Spec. Error : "
                              f"{mel_err:4.3f}, s/b : {time.time() - t_b:4.3f}", flush=True)
                    if steps % a.checkpoint_interval == 0 and steps:
                        torch.save({"generator": _unwrap(gen).state_dict()},
                                   os.path.join(a.checkpoint_path, f"g_{steps:08d}"))
                        torch.save({"mpd": _unwrap(mpd).state_dict(), "msd": _unwrap(msd).state_dict(),
                                    "optim_g": opt_g.state_dict(), "optim_d": opt_d.state_dict(), "steps": steps,
                                    "epoch": epoch}, os.path.join(a.checkpoint_path, f"do_{steps:08d}"))
                    if steps % a.summary_interval == 0:
                        sw.add_scalar("training/gen_loss_total", float(loss_g), steps)
                        sw.add_scalar("training/mel_spec_error", mel_err, steps)
                    if steps % a.validation_interval == 0:
                        validate(gen, valid_loader, h, sw, steps, dev)
                steps += 1
                if a.training_steps and steps >= a.training_steps:
                    return steps
            sch_g.step()
            sch_d.step()
            if rank == 0:
                print(f"Time taken for epoch {epoch + 1} is {int(time.time() - t_ep)} sec", flush=True)
    finally:
        if sw is not None:
            sw.close()
    return steps


def torch_step(h, mpd, msd, opt_d, opt_g, y, y_g, y_mel):
    """One D + G update on the torch modules (reference ``hifigan/train.py:113-160``)."""
    y_g_mel = mel_for(h, y_g.squeeze(1), loss=True)
    T = min(y_mel.shape[-1], y_g_mel.shape[-1])
    opt_d.zero_grad()
    r, g_, _, _ = mpd(y, y_g.detach())
    r2, g2, _, _ = msd(y, y_g.detach())
    loss_d = H.discriminator_loss(r, g_)[0] + H.discriminator_loss(r2, g2)[0]
    loss_d.backward()
    opt_d.step()
    opt_g.zero_grad()
    loss_mel = F.l1_loss(y_mel[..., :T], y_g_mel[..., :T]) * 45
    _, g_, fr, fg = mpd(y, y_g)
    _, g2, fr2, fg2 = msd(y, y_g)
    loss_g = (H.generator_loss(g_)[0] + H.generator_loss(g2)[0] + H.feature_loss(fr, fg) + H.feature_loss(fr2, fg2)
              + loss_mel)
    loss_g.backward()
    opt_g.step()
    return loss_g, loss_mel


def hip_step(h, mpd, msd, opt_d, opt_g, y, y_g, y_mel, world=1):
    """The same update on the HIP kernels: D loss + gradient into the discriminators (``hip_train.d_step``), then
    the mel-L1 x45 and adversarial + feature-matching gradients accumulated into ONE d loss / d y_g buffer and a
    single backward through the generator.  y, y_g: [B, T]."""
    from . import hip_train as HT

    mpd_m, msd_m = _unwrap(mpd), _unwrap(msd)
    opt_d.zero_grad()
    HT.d_step(mpd_m, msd_m, y, y_g.detach())
    if world > 1:
        ddp.allreduce_grads_flat(list(mpd_m.parameters()) + list(msd_m.parameters()))
    opt_d.step()
    opt_g.zero_grad()
    dy = torch.zeros(y_g.shape, device=y_g.device, dtype=torch.float32)
    loss_mel = HT.mel_l1(h, y_g, y_mel, 45.0, dy)
    loss_adv = HT.g_adv(mpd_m, msd_m, y, y_g, dy)
    torch.autograd.backward(y_g, dy.to(y_g.dtype))
    opt_g.step()
    return loss_mel + loss_adv, loss_mel


@torch.no_grad()
def validate(gen, loader, h, sw, steps, dev):
    g = _unwrap(gen)
    g.eval()
    err, n = 0.0, 0
    for j, (x, y, _, y_mel) in enumerate(loader):
        y_g = g(x.to(dev))
        y_g_mel = mel_for(h, y_g.squeeze(1), loss=True)
        ym = y_mel.to(dev)
        T = min(ym.shape[-1], y_g_mel.shape[-1])
        err += F.l1_loss(ym[..., :T], y_g_mel[..., :T]).item()
        n += 1
        if j <= 4:
            if steps == 0:
                sw.add_audio(f"gt/y_{j}", y[0].numpy(), steps, h.sampling_rate)
                _log_spec(sw, f"gt/y_spec_{j}", x[0].numpy(), steps)
            sw.add_audio(f"generated/y_hat_{j}", y_g[0, 0].float().cpu().numpy(), steps, h.sampling_rate)
            _log_spec(sw, f"generated/y_hat_spec_{j}", mel_for(h, y_g.squeeze(1))[0].cpu().numpy(), steps)
    if n:
        sw.add_scalar("validation/mel_spec_error", err / n, steps)
    g.train()
    return err / max(n, 1)
