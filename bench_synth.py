#!/usr/bin/env python
"""Synthesis benchmark: real-time factor of text -> int16 waveform (FastSpeech2 + HiFi-GAN).

BASELINE.json's second headline metric ("synth RTF"): wall time of text ids ->
int16 wav (FastSpeech2 forward incl. style encoder, HiFi-GAN V1 generator,
int16 conversion on the device) for a batch of utterances, divided by the
seconds of audio produced.  Lower is better.  Random-init weights; because a
random duration predictor emits ~0 frames, durations are injected
(``--frames-per-phone``, default 8: LJSpeech-like ~568 frames per utterance) --
SURVEY §7.7.  Multi-GPU: each rank synthesizes its own shard (launched by
torchrun); the RTF uses the max wall time over ranks and the summed audio.

Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_RTF = 1.33  # batch-1 E2E synthesis on the authors' GPU node (notebooks/control.ipynb:778)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="LJSpeech")
    ap.add_argument("--frames-per-phone", type=int, default=8)
    ap.add_argument("--gpus", type=int, default=1)
    args = ap.parse_args()
    os.environ.setdefault("PYTORCH_HIP_ALLOC_CONF", "expandable_segments:True")

    import torch

    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.parallel import ddp
    from speakingstyle_amd.utils.model import get_vocoder

    rank, world, local_rank = ddp.init_distributed()
    cuda = torch.cuda.is_available()
    dev = torch.device("cuda", local_rank) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(dev)
    pp, mc, tc = load_named(args.config)
    torch.manual_seed(0)
    model = FastSpeech2(pp, mc).to(dev).eval().set_compute_dtype(torch.bfloat16 if cuda else torch.float32)
    model.requires_grad_(False)
    voc = get_vocoder(mc, dev)
    hop = pp["preprocessing"]["stft"]["hop_length"]
    sr = pp["preprocessing"]["audio"]["sampling_rate"]
    gen = SyntheticBatches(args.batch, device=dev, seed=7 + rank)
    batch = gen.make_batch()
    speakers, texts, src_lens = batch[2], batch[3], batch[4]
    d = torch.full_like(texts, args.frames_per_phone).masked_fill(
        torch.arange(texts.shape[1], device=dev)[None] >= src_lens[:, None], 0)

    @torch.no_grad()
    def synth():
        out = model(speakers, texts, src_lens, batch[5], d_targets=d)
        mel, mel_len = out[1], out[9]
        if cuda:  # int16 conversion fused into the vocoder's conv_post kernel
            pcm = voc.infer(mel.to(torch.bfloat16).contiguous(), int16_scale=32768.0)
        else:
            wav = voc(mel.transpose(1, 2)).squeeze(1)
            pcm = (wav.float() * 32768.0).clamp(-32768, 32767).to(torch.int16)
        return pcm, mel_len

    for _ in range(args.warmup):
        synth()
    if cuda:
        torch.cuda.synchronize()
    ddp.barrier()
    t0 = time.perf_counter()
    samples = 0
    for _ in range(args.steps):
        pcm, mel_len = synth()
        samples += int(mel_len.sum().item()) * hop  # valid audio (the D2H of lengths is part of the pipeline)
    if cuda:
        torch.cuda.synchronize()
    ddp.barrier()
    wall = time.perf_counter() - t0
    audio_s = samples / sr
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([wall], device=dev, dtype=torch.float64)
        a = torch.tensor([audio_s], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(a)
        wall, audio_s = float(t.item()), float(a.item())
    rtf = wall / audio_s
    if rank == 0:
        print(json.dumps({
            "metric": "synth RTF (FastSpeech2 + HiFi-GAN, text -> int16 wav)",
            "value": rtf, "unit": "s wall / s audio", "higher_is_better": False, "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "audio_seconds": round(audio_s, 2), "wall_s": round(wall, 4),
            "vs_baseline": round(BASELINE_RTF / rtf, 1), "dtype": "bf16" if cuda else "fp32",
            "data": "synthetic text ids, injected durations, random-init weights",
            "config": {"model": f"FastSpeech2 ({args.config}) + HiFi-GAN V1", "batch_per_gpu": args.batch,
                       "parallelism": f"dp{world} (independent shards)"},
        }), flush=True)


if __name__ == "__main__":
    main()
