"""Benchmark harness behind ``bench.py`` / ``bench_synth.py``.

Two measurements (BASELINE.json: "train mel-frames/sec (node) + synth RTF"):

* ``train_phase`` -- W untimed + K timed full training steps of FastSpeech2
  (forward + loss + backward + bucketed RCCL gradient all-reduce + clip + Adam +
  LR schedule) on synthetic LJSpeech-shaped batches; value = valid mel frames
  summed over ranks / max-over-ranks wall time.
* ``synth_phase`` -- text ids -> int16 waveform with the style encoder in the
  loop (FastSpeech2 + FiLM reference encoder or GST on a reference mel, +
  HiFi-GAN V1 generator, int16 conversion on the device), batch 256 per GPU;
  RTF = max-over-ranks wall time / seconds of audio summed over ranks.  The
  random-init duration predictor would emit ~0 frames, so its
  output layer is re-initialised to predict ~``frames_per_phone`` frames with a
  little spread (bias = log(fpp + 1), weight ~ N(0, 0.005)); everything else --
  duration rounding, the one D2H of the mel lengths, length regulation, decoder,
  PostNet, vocoder -- is the real inference path (reference
  ``synthesize.py:128-150``, ``utils/model.py:97-115``).

Multi-GPU: ``launch()`` starts one rank per GPU with ``torch.distributed.run``
as a *child process* of a parent that never touched the GPU (re-exec'ing a
process that initialised HIP is forbidden on this platform), and every rank
asserts the world size it was promised.
"""
from __future__ import annotations

import json
import math
import os

import numpy as np
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---------------------------------------------------------------------- launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def needs_launch(n_gpus: int) -> bool:
    return n_gpus > 1 and "WORLD_SIZE" not in os.environ


def launch(script: str, n: int, argv) -> int:
    """Run ``script argv`` on ``n`` local ranks (torchrun child process); returns its exit code."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL peer buffers)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", script] + list(argv)
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------------- helpers
def _sync(cuda):
    import torch

    if cuda:
        torch.cuda.synchronize()


def _max_sum(world, device, t_local, x_local):
    """(max over ranks of t, sum over ranks of x)."""
    if world <= 1:
        return t_local, x_local
    import torch
    import torch.distributed as dist

    t = torch.tensor([t_local], dtype=torch.float64, device=device)
    x = torch.tensor([x_local], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(x, op=dist.ReduceOp.SUM)
    return float(t.item()), float(x.item())


def tiny_overrides(mc):
    """Plumbing-size model (CPU tests of the launcher): 1+1 layers, small widths."""
    mc["transformer"].update(encoder_layer=1, decoder_layer=1, conv_filter_size=64, encoder_hidden=32,
                             decoder_hidden=32, encoder_head=2, decoder_head=2)
    mc["variance_predictor"]["filter_size"] = 32
    if mc.get("reference_encoder"):
        mc["reference_encoder"].update(encoder_layer=1, encoder_head=2, encoder_hidden=32, conv_layer=1,
                                       conv_filter_size=32)
    if mc.get("gst"):
        mc["gst"].update(conv_filters=[4, 4, 8, 8, 16, 16], gru_hidden=16, token_size=16, n_style_token=4,
                         attn_head=2)


# ---------------------------------------------------------------------- training
def train_phase(args, rank, world, device):
    import torch

    from .config import load_named
    from .data.synthetic import SyntheticBatches
    from .models.fastspeech2 import FastSpeech2
    from .parallel import ddp
    from .train.trainer import Trainer

    cuda = device.type == "cuda"
    pp, mc, tc = load_named(args.config)
    if args.tiny:
        tiny_overrides(mc)
    batch = args.batch or int(tc["optimizer"]["batch_size"])
    torch.manual_seed(1234)
    model = FastSpeech2(pp, mc).to(device)
    model.set_compute_dtype(torch.bfloat16 if cuda else torch.float32)
    ddp.broadcast_module_state(model)
    trainer = Trainer(model, (pp, mc, tc), seed=1234)
    # the step's main chain on a high-priority stream, weight gradients on the normal-priority side stream
    trainer.use_priority_stream(cuda and not getattr(args, "normal_priority", False))
    trainer.timer.enabled = bool(getattr(args, "phase_times", False)) or trainer.timer.enabled

    if getattr(args, "force_buckets", False) and world == 1 and cuda:
        # the multi-GPU gradient path on one GPU: a 1-rank RCCL group, per-parameter hooks and bucket
        # all-reduces run exactly as under DP (identity reductions) -- measures their host cost
        import torch.distributed as dist

        if not dist.is_initialized():
            dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{_free_port()}")
        trainer.buckets = ddp.GradBuckets(trainer.opt.arena, trainer.buckets_mb, force=True)
    n_spk = n_speakers_of(pp) if mc.get("multi_speaker") else 1
    budget = getattr(args, "frames_per_gpu", None)
    gen = SyntheticBatches(batch, device=device, max_seq_len=mc["max_seq_len"], seed=1000 + rank, n_speakers=n_spk,
                           frames_per_batch=budget,
                           frame_level=pp["preprocessing"]["pitch"]["feature"] == "frame_level")
    pool = []
    for _ in range(args.pool):
        b = gen.make_batch()
        pool.append((b, gen.last_valid_frames))
    utts = [len(e[0][0]) for e in pool]
    # largest padded batch first: the first warm-up step sizes the allocator for all others
    pool.sort(key=lambda e: -(len(e[0][0]) * e[0][8]))

    from . import experimental

    fail_rank = experimental.get("fail_rank")  # fault injection (launcher failure-path test)
    def step(i):
        if fail_rank is not None and int(fail_rank) == rank and i == 1:
            raise RuntimeError(f"injected failure on rank {rank}")
        b, frames = pool[i % len(pool)]
        trainer.train_step(b)
        return frames

    # at least one untimed step under DP: the gradient-bucket calibration pass (ddp.GradBuckets)
    warm = max(args.warmup, 1 if (world > 1 or trainer.buckets.active) else 0)
    for i in range(warm):
        step(i)
    trainer.timer.summary()  # drop the warm-up phases
    _sync(cuda)
    ddp.barrier()
    _sync(cuda)
    if trainer._host_tail is not None:
        trainer._host_tail.clear()  # timed steps only
    t0 = time.perf_counter()
    frames = 0
    host = 0.0  # time inside train_step (enqueue): ~= elapsed when the step is host-bound
    # diagnostics: per step, how far the host's enqueue ran ahead of the GPU finishing the step
    lead = cuda and experimental.get("host_lead")
    if lead:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        evs, hts = [], []
    # diagnostics: device events at the step tail, in stream order -- after the joined backward + gradient
    # finalisation, before / after the clip + Adam launch: GPU time of the tail incl. any idle, free of the
    # host slowdown a kernel tracer adds (its traces show a ~0.8 ms step-end bubble)
    tail_ev = cuda and experimental.get("tail_events")
    if tail_ev:
        tail_recs = []
        fin0, opt0 = trainer.opt.arena.finalize_grads, trainer.opt.step_and_update_lr

        def _ev():
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e

        from .ops import hip as _hip

        join0 = _hip.join_side_streams

        def join(*a, **k):
            tail_recs.append({"bwd": _ev()})  # backward() returned: every main-stream backward kernel enqueued
            r = join0(*a, **k)
            tail_recs[-1]["joined"] = _ev()
            return r

        def fin(*a, **k):
            r = fin0(*a, **k)
            tail_recs[-1]["fin"] = _ev()
            return r

        _hip.join_side_streams = join

        def opt(*a, **k):
            tail_recs[-1]["opt0"] = _ev()
            r = opt0(*a, **k)
            tail_recs[-1]["opt1"] = _ev()
            return r

        trainer.opt.arena.finalize_grads, trainer.opt.step_and_update_lr = fin, opt
    for i in range(args.steps):
        h0 = time.perf_counter()
        frames += step(warm + i)
        host += time.perf_counter() - h0
        if lead:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            evs.append(e)
            hts.append(time.perf_counter() - t0)
    _sync(cuda)
    ddp.barrier()
    _sync(cuda)
    elapsed = time.perf_counter() - t0
    elapsed, frames_all = _max_sum(world, device, elapsed, float(frames))
    phases = trainer.timer.summary()
    info = {
        "phases": phases,
        "elapsed": elapsed, "frames": frames_all, "batch": batch, "warmup": warm,
        "utts_per_step": sum(utts[(warm + i) % len(pool)] for i in range(args.steps)) / max(1, args.steps),
        "frames_per_gpu": budget, "n_speakers": n_spk,
        "buckets": len(trainer.buckets.buckets),
        "overlap": trainer.buckets.calibrated() if (world > 1 or trainer.buckets.active) else None,
        "skipped_steps": int(trainer.opt.skipped_steps),
        "host_ms_per_step": 1000.0 * host / max(1, args.steps),
    }
    if lead:
        # GPU finish time of step i minus the host time its enqueue ended (both from t0; ev0 recorded ~t0)
        info["host_lead_ms"] = [round(ev0.elapsed_time(e) - 1e3 * h, 2) for e, h in zip(evs, hts)]
    if tail_ev:
        trainer.opt.arena.finalize_grads, trainer.opt.step_and_update_lr = fin0, opt0
        _hip.join_side_streams = join0
        rec = [r for r in tail_recs if "opt1" in r]
        mean = lambda xs: round(sum(xs) / max(1, len(xs)), 3)  # noqa: E731
        info["tail_events_ms"] = {
            "bwd_return->joined": mean([r["bwd"].elapsed_time(r["joined"]) for r in rec]),
            "joined->finalized": mean([r["joined"].elapsed_time(r["fin"]) for r in rec]),
            "finalized->opt_launch": mean([r["fin"].elapsed_time(r["opt0"]) for r in rec]),
            "opt_launch->opt_done": mean([r["opt0"].elapsed_time(r["opt1"]) for r in rec]),
            "step (opt_done->opt_done)": mean([a["opt1"].elapsed_time(b["opt1"]) for a, b in zip(rec, rec[1:])]),
        }
    tail = trainer.host_tail_summary()
    if tail is not None:
        info["host_tail_ms"] = tail
    del trainer, model, pool
    if cuda:
        torch.cuda.empty_cache()
    return info


# ---------------------------------------------------------------------- synthesis
def synth_phase(args, rank, world, device):
    import torch

    from .config import load_named
    from .data.synthetic import SyntheticBatches
    from .models.fastspeech2 import FastSpeech2
    from .parallel import ddp
    from .utils.model import get_vocoder

    cuda = device.type == "cuda"
    pp, mc, tc = load_named(args.synth_config)
    if args.tiny:
        tiny_overrides(mc)
    torch.manual_seed(0)
    model = FastSpeech2(pp, mc).to(device)
    with torch.no_grad():  # ~frames_per_phone frames per phoneme (see module docstring)
        lin = model.variance_adaptor.duration_predictor.linear_layer
        lin.weight.normal_(0.0, 0.005)
        lin.bias.fill_(math.log(args.frames_per_phone + 1.0))
    model.eval().set_compute_dtype(torch.bfloat16 if cuda else torch.float32)
    model.requires_grad_(False)
    voc = get_vocoder(mc, device)
    hop = pp["preprocessing"]["stft"]["hop_length"]
    sr = pp["preprocessing"]["audio"]["sampling_rate"]
    mx = float(pp["preprocessing"]["audio"]["max_wav_value"])
    # texts + a reference mel per utterance (the style input of synthesize.py single/batch mode): one distinct
    # synthetic batch per timed step (and per warm-up step), all generated on the device before timing
    gen = SyntheticBatches(args.synth_batch, device=device, seed=7 + rank, max_seq_len=mc["max_seq_len"])
    nb = args.synth_warmup + args.synth_steps
    batches = [gen.make_batch() for _ in range(max(1, nb))]

    # Two-stage pipeline: the vocoder of batch i runs on its own stream while FastSpeech2 of batch i+1
    # runs on the main stream -- FastSpeech2's host syncs (predicted lengths) wait for the main stream
    # only, so the GPU is not drained between batches.  Every batch still does its full FS2 + vocoder
    # work; the RTF is wall time over all audio of the timed batches (--synth-serial: one stream, A/B).
    voc_stream = torch.cuda.Stream(device=device) if (cuda and not getattr(args, "synth_serial", False)) else None
    # FastSpeech2 of batch i+1 on a HIGH-priority stream: its (short, latency-bound) kernels are dispatched as soon
    # as the vocoder of batch i frees CUs, so the host's length sync -- and with it the next vocoder launch -- is not
    # queued behind the whole vocoder (its persistent grids hold every CU)
    # (measured neutral-to-slightly-worse, profiles/r6_ab_synth.txt: off unless --synth-prio)
    fs2_stream = (torch.cuda.Stream(device=device, priority=-1)
                  if (voc_stream is not None and getattr(args, "synth_prio", False)) else None)

    packed = cuda and getattr(args, "packed_fs2", True)

    @torch.no_grad()
    def synth(b, stream=voc_stream, host_wav=False):
        speakers, texts, src_lens, max_src = b[2], b[3], b[4], b[5]
        ref_mels, ref_lens, ref_max = b[6], b[7], b[8]
        if packed and model.packed_inference_ok(texts):
            # decoder / PostNet / vocoder on the valid frames only (FastSpeech2.infer_packed -> Generator.infer_packed)
            if stream is not None and fs2_stream is not None:
                fs2_stream.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(fs2_stream):
                    rows, lens_l, _ = model.infer_packed(speakers, texts, src_lens, max_src, ref_mels, ref_lens,
                                                         ref_max)
                stream.wait_stream(fs2_stream)
                rows.record_stream(stream)
                with torch.cuda.stream(stream):
                    pcm = voc.infer_packed(rows, lens_l, int16_scale=mx)
                if host_wav:
                    pcm = pcm.cpu()
                return pcm, torch.tensor(lens_l)
            rows, lens_l, _ = model.infer_packed(speakers, texts, src_lens, max_src, ref_mels, ref_lens, ref_max)
            if stream is not None:
                stream.wait_stream(torch.cuda.current_stream())
                rows.record_stream(stream)
                with torch.cuda.stream(stream):
                    pcm = voc.infer_packed(rows, lens_l, int16_scale=mx)
            else:
                pcm = voc.infer_packed(rows, lens_l, int16_scale=mx)
            if host_wav:
                pcm = pcm.cpu()
            return pcm, torch.tensor(lens_l)
        out = model(speakers, texts, src_lens, max_src, ref_mels, ref_lens, ref_max)
        mel, mel_len = out[1], out[9]
        lens = mel_len.cpu()  # host lengths: the vocoder runs length-bucketed (exact on valid samples)
        if cuda:  # int16 conversion fused into the vocoder's conv_post kernel; the pack kernel casts fp32 -> bf16
            mel_b = mel.contiguous()
            if stream is not None:
                stream.wait_stream(torch.cuda.current_stream())
                mel_b.record_stream(stream)  # the main stream's allocator must not recycle it early
                with torch.cuda.stream(stream):
                    pcm = voc.infer(mel_b, int16_scale=mx, lengths=lens.tolist(), max_buckets=args.vocoder_buckets)
            else:
                pcm = voc.infer(mel_b, int16_scale=mx, lengths=lens.tolist(), max_buckets=args.vocoder_buckets)
        else:
            wav = voc(mel.transpose(1, 2)).squeeze(1)
            pcm = (wav.float() * mx).clamp(-32768, 32767).to(torch.int16)
        if host_wav:  # the int16 waveform on the host: the end of the text -> wav path (synthesize.py)
            pcm = pcm.cpu()
        return pcm, lens

    # warm-up: the --synth-warmup batches, then every timed batch once -- each distinct (B, T) bucket shape of
    # the FS2 layers and of the vocoder's length groups has then been allocated and launched once, so the timed
    # region measures steady-state synthesis (not first-use allocations); every timed step still computes its
    # whole text -> wav path from scratch
    for i in range(args.synth_warmup):
        synth(batches[i % len(batches)])
    for i in range(args.synth_steps):
        synth(batches[(args.synth_warmup + i) % len(batches)])
    _sync(cuda)
    ddp.barrier()
    _sync(cuda)
    # host-lead probe (``--synth-lead``): per timed batch, the time the host finished enqueueing it and the time the
    # GPU finished its vocoder (an event on the vocoder stream), both from t0.  GPU-bound steady state: every batch
    # completes on the GPU well after the host enqueued it (lead ~ one batch of vocoder work), and the host's own
    # time per batch (enqueue + the one length sync) is a fraction of the GPU's
    lead = cuda and voc_stream is not None and getattr(args, "synth_lead", False)
    if lead:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        evs, hts = [], []
    t0 = time.perf_counter()
    samples = 0
    for i in range(args.synth_steps):
        pcm, mel_len = synth(batches[(args.synth_warmup + i) % len(batches)])
        samples += int(mel_len.sum()) * hop  # valid audio (the D2H of lengths is inside synth())
        if lead:
            e = torch.cuda.Event(enable_timing=True)
            e.record(voc_stream)
            evs.append(e)
            hts.append(time.perf_counter() - t0)
    _sync(cuda)
    ddp.barrier()
    _sync(cuda)
    wall = time.perf_counter() - t0
    wall, audio_s = _max_sum(world, device, wall, samples / sr)
    info = {"wall": wall, "audio_s": audio_s, "rtf": wall / max(audio_s, 1e-12),
            "frames_per_utt": samples / hop / max(1, args.synth_steps * args.synth_batch),
            "distinct_batches": min(args.synth_steps, len(batches))}
    if lead:
        done = [ev0.elapsed_time(e) for e in evs]
        info["lead"] = {"host_enqueued_ms": [round(1e3 * h, 2) for h in hts], "gpu_done_ms": [round(d, 2) for d in done],
                        "gpu_minus_host_ms": [round(d - 1e3 * h, 2) for d, h in zip(done, hts)],
                        "gpu_ms_per_batch": round((done[-1] - done[0]) / max(1, len(done) - 1), 2)}
    del batches

    # Batch-1 latency, like-for-like with the reference's only synthesis number (one utterance of 113 mel
    # frames, text -> wav, notebooks/control.ipynb:778): ~14 phonemes at ~8 predicted frames each, one
    # stream, each run from an idle GPU to the int16 waveform on the host; median over the runs.
    runs = int(getattr(args, "synth_b1_runs", 0) or 0)
    if runs > 0:
        g1 = SyntheticBatches(1, device=device, seed=17 + rank, max_seq_len=mc["max_seq_len"],
                              phone_counts=np.array([int(getattr(args, "synth_b1_phones", 14))]))
        b1 = g1.make_batch()
        # serving path: the packed synthesis replayed from HIP graphs (infer/graphs.py; every replay recomputes
        # text -> wav from the inputs, only the ~350 launches' host cost goes)
        sg = None
        if packed and getattr(args, "synth_graphs", True):
            from .infer.graphs import SynthGraphs

            sg = SynthGraphs(model, voc, int16_scale=mx)
            if not sg.supported(b1[3]):
                sg = None

        def one():
            if sg is None:
                return synth(b1, stream=None, host_wav=True)
            pcm_d, lens_l = sg(b1[2], b1[3], b1[4], b1[5], b1[6], b1[7], b1[8])
            return pcm_d.cpu(), torch.tensor(lens_l)

        for _ in range(max(3, args.synth_warmup)):
            one()
        times, frames = [], 0
        for _ in range(runs):
            _sync(cuda)
            t1 = time.perf_counter()
            pcm, mel_len = one()
            times.append(time.perf_counter() - t1)
            frames = int(mel_len.sum())
        med = float(np.median(times))
        audio1 = frames * hop / sr
        info["b1"] = {"median_s": med, "min_s": float(min(times)), "max_s": float(max(times)), "runs": runs,
                      "mel_frames": frames, "audio_s": audio1, "rtf": med / max(audio1, 1e-12),
                      "samples": int(pcm.numel()), "graphs": None if sg is None else dict(sg.stats)}
    del model, voc
    if cuda:
        torch.cuda.empty_cache()
    return info


def n_speakers_of(pp) -> int:
    """Speaker count of the config's ``speakers.json`` (LibriTTS: 904), 1 when absent."""
    p = os.path.join(ROOT, pp["path"]["preprocessed_path"]) if not os.path.isabs(
        pp["path"]["preprocessed_path"]) else pp["path"]["preprocessed_path"]
    f = os.path.join(p, "speakers.json")
    if os.path.exists(f):
        with open(f) as fh:
            return max(1, len(json.load(fh)))
    return 1


def report(rec: dict):
    print(json.dumps(rec), flush=True)
