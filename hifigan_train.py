#!/usr/bin/env python
"""HiFi-GAN vocoder training (reference ``hifigan/train.py``) -- one process per GPU
(torchrun), DDP over RCCL for G / MPD / MSD, AdamW + ExponentialLR, mel-L1 x45 +
feature matching + LSGAN losses, auto-resume from the latest ``g_########`` /
``do_########`` checkpoints.  The reference script cannot run (MPD undefined);
this one implements both discriminators.

  torchrun --standalone --nproc-per-node 8 hifigan_train.py --input_wavs_dir wavs --checkpoint_path ckpt
  python hifigan_train.py --synthetic --training_steps 2     (plumbing, CPU or GPU)
"""
import argparse
import glob
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from torch.nn.parallel import DistributedDataParallel  # noqa: E402

from speakingstyle_amd.audio.stft import TacotronSTFT  # noqa: E402
from speakingstyle_amd.models import hifigan as H  # noqa: E402
from speakingstyle_amd.parallel import ddp  # noqa: E402
from speakingstyle_amd.utils.model import vocoder_config  # noqa: E402


class MelDataset(torch.utils.data.Dataset):
    """Random ``segment_size`` crops of wavs + their mels (reference ``hifigan/meldataset.py:86-168``)."""

    def __init__(self, files, h, synthetic_n=0):
        self.files, self.h, self.synthetic_n = files, h, synthetic_n
        self.stft = TacotronSTFT(h.n_fft, h.hop_size, h.win_size, h.num_mels, h.sampling_rate, h.fmin, h.fmax)

    def __len__(self):
        return self.synthetic_n or len(self.files)

    def __getitem__(self, i):
        from speakingstyle_amd.audio.io import read_wav

        seg = self.h.segment_size
        if self.synthetic_n:
            t = np.arange(seg) / self.h.sampling_rate
            wav = 0.3 * np.sin(2 * np.pi * (110 + 30 * (i % 7)) * t) + 0.01 * np.random.randn(seg)
        else:
            wav, _ = read_wav(self.files[i], self.h.sampling_rate)
            wav = 0.95 * wav / max(1e-6, np.abs(wav).max())
            if len(wav) >= seg:
                s = np.random.randint(0, len(wav) - seg + 1)
                wav = wav[s:s + seg]
            else:
                wav = np.pad(wav, (0, seg - len(wav)))
        y = torch.from_numpy(wav.astype(np.float32)).clamp(-1, 1)
        mel, _ = self.stft.mel_spectrogram(y.unsqueeze(0))
        return mel[0, :, : seg // self.h.hop_size], y  # frames * hop == segment_size


def latest(path, prefix):
    cps = sorted(glob.glob(os.path.join(path, prefix + "????????")))
    return cps[-1] if cps else None


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--input_wavs_dir", default="LJSpeech-1.1/wavs")
    ap.add_argument("--checkpoint_path", default="output/hifigan")
    ap.add_argument("--config", default=None)
    ap.add_argument("--training_epochs", type=int, default=3100)
    ap.add_argument("--training_steps", type=int, default=0, help="stop after N steps (0 = epochs)")
    ap.add_argument("--checkpoint_interval", type=int, default=5000)
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--batch_size", type=int, default=None)
    a = ap.parse_args(argv)
    h = vocoder_config(a.config)
    rank, world, local_rank = ddp.init_distributed()
    cuda = torch.cuda.is_available()
    dev = torch.device("cuda", local_rank) if cuda else torch.device("cpu")
    torch.manual_seed(h.seed + rank)
    gen = H.Generator(h).to(dev)
    mpd = H.MultiPeriodDiscriminator().to(dev)
    msd = H.MultiScaleDiscriminator().to(dev)
    os.makedirs(a.checkpoint_path, exist_ok=True)
    steps, last_epoch = 0, -1
    cp_g, cp_do = latest(a.checkpoint_path, "g_"), latest(a.checkpoint_path, "do_")
    state_do = None
    if cp_g and cp_do:
        gen.load_state_dict(torch.load(cp_g, map_location=dev, weights_only=True)["generator"])
        state_do = torch.load(cp_do, map_location=dev, weights_only=True)
        mpd.load_state_dict(state_do["mpd"])
        msd.load_state_dict(state_do["msd"])
        steps, last_epoch = state_do["steps"] + 1, state_do["epoch"]
    if world > 1:
        gen = DistributedDataParallel(gen, device_ids=[local_rank] if cuda else None)
        mpd = DistributedDataParallel(mpd, device_ids=[local_rank] if cuda else None)
        msd = DistributedDataParallel(msd, device_ids=[local_rank] if cuda else None)
    opt_g = torch.optim.AdamW(gen.parameters(), h.learning_rate, betas=(h.adam_b1, h.adam_b2))
    opt_d = torch.optim.AdamW(itertools.chain(msd.parameters(), mpd.parameters()), h.learning_rate,
                              betas=(h.adam_b1, h.adam_b2))
    if state_do is not None:
        opt_g.load_state_dict(state_do["optim_g"])
        opt_d.load_state_dict(state_do["optim_d"])
    sch_g = torch.optim.lr_scheduler.ExponentialLR(opt_g, gamma=h.lr_decay, last_epoch=last_epoch)
    sch_d = torch.optim.lr_scheduler.ExponentialLR(opt_d, gamma=h.lr_decay, last_epoch=last_epoch)
    files = sorted(glob.glob(os.path.join(a.input_wavs_dir, "*.wav")))
    ds = MelDataset(files, h, synthetic_n=64 if (a.synthetic or not files) else 0)
    sampler = torch.utils.data.distributed.DistributedSampler(ds) if world > 1 else None
    bs = a.batch_size or max(1, h.batch_size // world)
    loader = torch.utils.data.DataLoader(ds, batch_size=bs, shuffle=sampler is None, sampler=sampler, drop_last=True,
                                         num_workers=0)
    stft = TacotronSTFT(h.n_fft, h.hop_size, h.win_size, h.num_mels, h.sampling_rate, h.fmin, h.fmax).to(dev)
    gen.train(); mpd.train(); msd.train()
    for epoch in range(max(0, last_epoch + 1), a.training_epochs):
        if sampler is not None:
            sampler.set_epoch(epoch)
        t_ep = time.time()
        for mel, y in loader:
            mel, y = mel.to(dev), y.to(dev).unsqueeze(1)
            y_g = gen(mel)
            y_g_mel, _ = stft.mel_spectrogram(y_g.squeeze(1).clamp(-1, 1))
            opt_d.zero_grad()
            r, g_, _, _ = mpd(y, y_g.detach())
            r2, g2, _, _ = msd(y, y_g.detach())
            loss_d = H.discriminator_loss(r, g_)[0] + H.discriminator_loss(r2, g2)[0]
            loss_d.backward()
            opt_d.step()
            opt_g.zero_grad()
            loss_mel = F.l1_loss(mel, y_g_mel[..., : mel.shape[-1]]) * 45
            _, g_, fr, fg = mpd(y, y_g)
            _, g2, fr2, fg2 = msd(y, y_g)
            loss_g = (H.generator_loss(g_)[0] + H.generator_loss(g2)[0] + H.feature_loss(fr, fg) +
                      H.feature_loss(fr2, fg2) + loss_mel)
            loss_g.backward()
            opt_g.step()
            if rank == 0 and steps % 10 == 0:
                print(f"Steps : {steps:d}, Gen Loss Total : {float(loss_g):4.3f}, Mel-Spec. Error : "
                      f"{float(loss_mel) / 45:4.3f}", flush=True)
            if rank == 0 and steps % a.checkpoint_interval == 0 and steps:
                gm = gen.module if hasattr(gen, "module") else gen
                torch.save({"generator": gm.state_dict()}, os.path.join(a.checkpoint_path, f"g_{steps:08d}"))
                torch.save({"mpd": (mpd.module if hasattr(mpd, "module") else mpd).state_dict(),
                            "msd": (msd.module if hasattr(msd, "module") else msd).state_dict(),
                            "optim_g": opt_g.state_dict(), "optim_d": opt_d.state_dict(), "steps": steps,
                            "epoch": epoch}, os.path.join(a.checkpoint_path, f"do_{steps:08d}"))
            steps += 1
            if a.training_steps and steps >= a.training_steps:
                return steps
        sch_g.step()
        sch_d.step()
        if rank == 0:
            print(f"Time taken for epoch {epoch + 1} is {int(time.time() - t_ep)} sec", flush=True)
    return steps


if __name__ == "__main__":
    main()
