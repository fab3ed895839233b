#!/usr/bin/env python
"""Headline benchmark: FastSpeech2 training throughput (mel-frames/s, node) + synthesis RTF.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``.  For N>1 the
driver launches it under torch.distributed.run (one rank per GPU, RCCL over
xGMI); run directly with ``--gpus N`` and no torchrun environment, this script
starts the N ranks itself (``speakingstyle_amd.benchmark.launch``: a torchrun
child process of a parent that never initialises the GPU) and exits with the
child's status.  Every rank asserts WORLD_SIZE == N.

Training (headline ``value``): W untimed warm-up steps (>= 1 under DP: the
gradient-bucket calibration pass), then exactly K full training steps (forward
+ loss + backward + bucketed gradient all-reduce + clip + Adam + LR schedule)
bracketed by barrier + device synchronise on both sides; time = MAX over ranks;
value = valid mel frames of the K steps summed over ranks / that time.
Config = BASELINE.json's headline: LJSpeech FastSpeech2 (model.yaml shape: 4+6
FFT blocks, d=256, no style encoder), bf16 compute with fp32 master weights /
Adam state, synthetic LJSpeech-shaped data (phoneme counts drawn from the real
LJSpeech metadata, ~8.1 frames per phoneme, groups of 4 batches sorted by text
length exactly like the reference loader), random-init weights.  Scaling is
weak: every rank runs ``--batch`` utterances (default: the config's
``optimizer.batch_size`` = 200), global batch N*200; ``--frames-per-gpu F`` sizes
each rank's batch by a padded-frame budget instead (``mi355x.frames_per_gpu``, the
same per-GPU batch semantics ``train.py`` uses when that key is set; without it
``train.py`` splits ``batch_size`` across ranks -- the reference's global batch).

Synthesis (``synth_rtf`` field, BASELINE's second metric): text ids -> int16 wav
through FastSpeech2 + style encoder (``--synth-config``, default BC2013_GST = the
GST reference encoder + style-token attention on a reference mel, BASELINE #5) +
HiFi-GAN V1, batch 256 per GPU over ``--synth-steps`` distinct batches, independent
shards per rank; RTF = max-over-ranks wall / total audio seconds.  ``synth.rtf_also``
repeats it with ``--synth-also`` (default BC2013: the reference's FiLM reference
encoder).  ``synth_rtf_b1``: the like-for-like point of the reference's only
synthesis number (batch 1, one 113-frame utterance, RTF 1.33 in
``notebooks/control.ipynb:778``): median wall time of ``--synth-b1-runs`` runs of one
~113-frame utterance (text ids -> int16 waveform on the host) / its audio seconds;
``synth_vs_baseline`` compares THAT with 1.33.
See ``speakingstyle_amd/benchmark.py`` for the duration-injection detail.
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_FRAMES_PER_S = 2.5e4  # derived GTX-1080Ti lower bound (train mel-frames/s)
BASELINE_RTF = 1.33  # batch-1 E2E synthesis on the authors' GPU node (notebooks/control.ipynb:778)


def _num(x):
    return int(x) if float(x).is_integer() else round(float(x), 1)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="LJSpeech")
    ap.add_argument("--batch", type=int, default=None, help="utterances per GPU (default: config batch_size)")
    ap.add_argument("--pool", type=int, default=8, help="distinct synthetic batches cycled through")
    ap.add_argument("--backend", default=None, choices=[None, "hip", "reference"])
    ap.add_argument("--synth-config", default="BC2013_GST",
                    help="FS2 + style encoder of the synth_rtf line (BASELINE #5: FS2 + GST)")
    ap.add_argument("--synth-also", default="BC2013",
                    help="second synthesis config reported as synth.rtf_also ('' disables): the FiLM encoder")
    ap.add_argument("--synth-batch", type=int, default=256)
    ap.add_argument("--synth-steps", type=int, default=10,
                    help="timed batch-256 synthesis steps, each on a distinct batch (0 disables the synthesis phase)")
    ap.add_argument("--synth-b1-runs", type=int, default=30,
                    help="batch-1 latency runs (one ~113-frame utterance, text -> int16 wav on the host; 0 disables)")
    ap.add_argument("--synth-b1-phones", type=int, default=14, help="phonemes of the batch-1 utterance")
    ap.add_argument("--no-synth-graphs", action="store_false", dest="synth_graphs",
                    help="batch-1 synthesis launched eagerly instead of replayed from HIP graphs (A/B)")
    ap.add_argument("--synth-warmup", type=int, default=1)
    ap.add_argument("--frames-per-phone", type=float, default=8.1)
    ap.add_argument("--vocoder-buckets", type=int, default=8,
                    help="max length buckets of the vocoder (1: vocode the padded batch)")
    ap.add_argument("--tiny", action="store_true", help="plumbing-size model (CPU launcher tests only)")
    ap.add_argument("--phase-times", action="store_true", help="per-phase host/device ms of the timed steps")
    ap.add_argument("--frames-per-gpu", type=int, default=None,
                    help="per-GPU padded mel-frame budget per step (mi355x.frames_per_gpu) instead of --batch")
    ap.add_argument("--no-side-wgrad", action="store_true",
                    help="weight gradients on the main stream (A/B of the side-stream overlap)")
    ap.add_argument("--synth-serial", action="store_true",
                    help="synthesis on one stream (A/B of the FS2 / vocoder two-stream pipeline)")
    ap.add_argument("--ln-reduce-main", action="store_true",
                    help="LayerNorm weight-gradient reductions on the main stream (A/B of the side-stream move)")
    ap.add_argument("--normal-priority", action="store_true",
                    help="main chain on a normal-priority stream (A/B of Trainer.use_priority_stream)")
    ap.add_argument("--ctypes-bindings", action="store_true",
                    help="launch kernels through ctypes instead of the generated native bindings (A/B)")
    ap.add_argument("--force-buckets", action="store_true",
                    help="1 GPU: run the DP gradient path (1-rank RCCL group, hooks, bucket all-reduces)")
    ap.add_argument("--dist-backend", default=None, choices=[None, "nccl", "gloo"],
                    help="default: nccl (RCCL) on GPUs; gloo rehearses the multi-rank path on fewer GPUs")
    return ap.parse_args(argv)


def main():
    args = parse()
    from speakingstyle_amd import benchmark as B

    if B.needs_launch(args.gpus):
        sys.exit(B.launch(os.path.abspath(__file__), args.gpus, sys.argv[1:]))

    from speakingstyle_amd.parallel import ddp

    ddp.fail_fast(run, args)


def run(args):
    import torch

    from speakingstyle_amd import benchmark as B
    from speakingstyle_amd import ops
    from speakingstyle_amd.parallel import ddp

    if args.backend:
        ops.set_backend(args.backend)
    if args.ctypes_bindings:
        from speakingstyle_amd.ops import hip

        hip._USE_FAST[0] = False
    if args.no_side_wgrad and torch.cuda.is_available():
        from speakingstyle_amd import experimental

        experimental.set_value("side_wgrad", "0", "bench --no-side-wgrad")
    if args.ln_reduce_main and torch.cuda.is_available():
        from speakingstyle_amd.ops import hip

        hip._SIDE_LN[0] = False
    rank, world, local_rank = ddp.init_distributed(backend=args.dist_backend, expect_world=args.gpus)
    cuda = torch.cuda.is_available()
    device = torch.device("cuda", local_rank) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(device)
    seen = torch.distributed.get_world_size() if world > 1 else 1
    comm = torch.distributed.get_backend() if world > 1 else None

    tr = B.train_phase(args, rank, world, device)
    sy = B.synth_phase(args, rank, world, device) if args.synth_steps > 0 else None
    sy2 = None
    if sy is not None and args.synth_also and args.synth_also != args.synth_config:
        import copy

        a2 = copy.copy(args)
        a2.synth_config = args.synth_also
        a2.synth_b1_runs = 0
        sy2 = B.synth_phase(a2, rank, world, device)

    value = tr["frames"] / tr["elapsed"]
    rec = {
        "metric": "train mel-frames/sec (node)",
        "value": round(value, 1),
        "unit": "mel-frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": tr["warmup"],
        "ms_per_step": round(1000.0 * tr["elapsed"] / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / BASELINE_FRAMES_PER_S, 3),
        "dtype": "bf16" if cuda else "fp32",
        "data": "synthetic (LJSpeech-shaped lengths, random-init weights)",
        "config": {
            "model": f"FastSpeech2 ({args.config} model.yaml)" + (" tiny" if args.tiny else ""),
            "global_batch": _num(tr["utts_per_step"] * world),
            "seq_len": "T~LJSpeech phonemes, M<=1000 mel frames",
            "parallelism": f"dp{world}",
        },
        "batch_per_gpu": tr["batch"] if not tr["frames_per_gpu"] else None,
        "frames_per_gpu": tr["frames_per_gpu"],
        "utterances_per_gpu_step": round(tr["utts_per_step"], 1),
        "n_speakers": tr["n_speakers"],
        "world_size_seen": seen,
        "comm_backend": comm,
        "grad_buckets": tr["buckets"],
        "bucket_overlap": tr["overlap"],
        "skipped_steps": tr["skipped_steps"],
        "host_enqueue_ms_per_step": round(tr["host_ms_per_step"], 3),
    }
    if tr.get("host_lead_ms"):
        rec["host_lead_ms"] = tr["host_lead_ms"]
    if tr.get("host_tail_ms"):
        rec["host_tail_ms"] = tr["host_tail_ms"]
    if tr.get("tail_events_ms"):
        rec["tail_events_ms"] = tr["tail_events_ms"]
    if tr.get("phases"):
        rec["phase_ms"] = {k: {"host": round(v["host_ms"], 3), "device": round(v["device_ms"], 3)}
                           for k, v in tr["phases"].items()}
    if sy is not None:
        b1 = sy.get("b1")
        rec.update({
            "synth_rtf": sy["rtf"],
            "synth_rtf_b1": None if b1 is None else b1["rtf"],
            "synth_vs_baseline": None if b1 is None else round(BASELINE_RTF / b1["rtf"], 1),
            "synth": {
                "metric": "synth RTF (text ids -> int16 wav; lower is better)",
                "model": f"FastSpeech2 ({args.synth_config}, style encoder on a reference mel) + HiFi-GAN V1"
                         + (" tiny" if args.tiny else ""),
                "batch_per_gpu": args.synth_batch, "steps": args.synth_steps, "warmup": args.synth_warmup,
                "distinct_batches": sy["distinct_batches"],
                "audio_seconds": round(sy["audio_s"], 2), "wall_s": round(sy["wall"], 4),
                "mel_frames_per_utt": round(sy["frames_per_utt"], 1),
                "vocoder_length_buckets": args.vocoder_buckets,
                "parallelism": f"dp{world} (independent shards)",
            },
        })
        if b1 is not None:
            rec["synth"]["b1"] = {"metric": "batch-1 latency: one utterance, text ids -> int16 wav on the host",
                                  "median_ms": round(1e3 * b1["median_s"], 3), "min_ms": round(1e3 * b1["min_s"], 3),
                                  "max_ms": round(1e3 * b1["max_s"], 3), "runs": b1["runs"],
                                  "mel_frames": b1["mel_frames"], "audio_seconds": round(b1["audio_s"], 4),
                                  "hip_graphs": b1.get("graphs"),
                                  "baseline": "RTF 1.33: 113 frames, batch 1 (notebooks/control.ipynb:778)"}
        if sy2 is not None:
            rec["synth"]["rtf_also"] = {"model": f"FastSpeech2 ({args.synth_also}) + HiFi-GAN V1", "rtf": sy2["rtf"],
                                        "audio_seconds": round(sy2["audio_s"], 2)}
    if rank == 0:
        B.report(rec)
    if world > 1:
        ddp.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
