#!/usr/bin/env python
"""Synthesis benchmark alone: real-time factor of text ids -> int16 waveform.

Same measurement as the ``synth_rtf`` field of ``bench.py`` (FastSpeech2 + style
encoder on a reference mel + HiFi-GAN V1, int16 on the device, batch 256 per
GPU; see ``speakingstyle_amd/benchmark.py``), without the training phase -- for
profiling the inference path (``tools/gpu.sh synthprof``).  ``--gpus N`` starts
N independent-shard ranks like bench.py.  Prints one JSON line; lower is better.
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_RTF = 1.33  # batch-1 E2E synthesis on the authors' GPU node (notebooks/control.ipynb:778)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--batch", type=int, default=256, dest="synth_batch")
    ap.add_argument("--steps", type=int, default=3, dest="synth_steps")
    ap.add_argument("--warmup", type=int, default=1, dest="synth_warmup")
    ap.add_argument("--config", default="BC2013_GST", dest="synth_config")
    ap.add_argument("--vocoder-buckets", type=int, default=8, help="1: vocode the padded batch")
    ap.add_argument("--frames-per-phone", type=float, default=8.1)
    ap.add_argument("--tiny", action="store_true")
    ap.add_argument("--synth-serial", action="store_true", help="one stream (A/B of the two-stream pipeline)")
    ap.add_argument("--b1-runs", type=int, default=0, dest="synth_b1_runs", help="batch-1 latency runs (0: off)")
    ap.add_argument("--b1-phones", type=int, default=14, dest="synth_b1_phones")
    ap.add_argument("--no-graphs", action="store_false", dest="synth_graphs", help="eager batch-1 synthesis (A/B)")
    ap.add_argument("--synth-lead", action="store_true", help="host-lead probe of the timed batches (diagnostic)")
    ap.add_argument("--synth-prio", action="store_true",
                    help="FastSpeech2 on a high-priority stream instead of the default one (A/B)")
    ap.add_argument("--whole-skip", default="",
                    help="C:K,C:K whole-ResBlock geometries to run on the per-layer kernel instead (A/B)")
    ap.add_argument("--no-rb256", action="store_true",
                    help="C = 256 MRF on the GEMM path instead of the tall per-layer ResBlock kernel (A/B)")
    ap.add_argument("--rb256-min-rows", type=int, default=None,
                    help="row count from which the C = 256 MRF uses the tall per-layer kernel (A/B; default 65536)")
    ap.add_argument("--splitk", type=int, default=None, help="GEMM split-K: -1 auto, 0 off, S forced (A/B)")
    ap.add_argument("--no-skinny", action="store_true", help="small-M GEMMs (<= 1024 rows) on the tile kernels instead of the skinny kernel (A/B)")
    ap.add_argument("--gemm-addln-rows", type=int, default=None,
                    help="inference FFT blocks: GEMM + residual + LayerNorm as one kernel up to this many rows (A/B)")
    ap.add_argument("--skinny-maxm", type=int, default=None, help="row limit of the skinny GEMM kernel (A/B)")
    ap.add_argument("--skinny-w8", type=int, default=None, help="8-wave skinny blocks from this many k-steps (A/B)")
    ap.add_argument("--skinny-cin32", action="store_true", help="skinny GEMMs only for Cin % 32 == 0 (A/B)")
    ap.add_argument("--rf-short-tiles", type=int, default=None,
                    help="whole-ResBlock short tile below this many regular tiles (A/B; 0: never)")
    ap.add_argument("--rb-small-tiles", type=int, default=None,
                    help="per-layer ResBlock 64-row tile below this many 128-row tiles (A/B; 0: never)")
    ap.add_argument("--addln-small-rows", type=int, default=None,
                    help="rows at or below which add_layernorm runs one row iteration per wave (A/B; 0: off)")
    ap.add_argument("--splitk-tiny", type=int, default=None,
                    help="min k-steps per split-K slice for <= 8 GEMM tiles (0: general rule only) (A/B)")
    ap.add_argument("--rb-whole-extra", action="store_true",
                    help="whole-ResBlock kernels also for C = 64 / K = 11 and C = 128 / K = 7 (A/B)")
    ap.add_argument("--rb-half", action="store_true",
                    help="per-layer ResBlock kernel on the half tall block (4 waves, two blocks per CU) (A/B)")
    ap.add_argument("--rb-regular", action="store_true",
                    help="per-layer ResBlock kernel on the 128-row tile instead of the tall 64x64-per-wave tile (A/B)")
    ap.add_argument("--bucketed", action="store_true",
                    help="padded FS2 + length-bucketed vocoding instead of the packed length-exact path (A/B)")
    ap.add_argument("--padded-fs2", action="store_false", dest="packed_fs2",
                    help="padded FS2 decoder / PostNet, packed vocoder (A/B)")
    return ap.parse_args()


def run(args):
    import torch

    from speakingstyle_amd import benchmark as B
    from speakingstyle_amd.parallel import ddp

    rank, world, local_rank = ddp.init_distributed(expect_world=args.gpus)
    cuda = torch.cuda.is_available()
    dev = torch.device("cuda", local_rank) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(dev)
    if args.rb_half and cuda:
        from speakingstyle_amd.ops import hip

        hip.lib().ssamd_resblock_set_tall(2)
    if args.rb_regular and cuda:
        from speakingstyle_amd.ops import hip

        hip.lib().ssamd_resblock_set_tall(0)
    if args.whole_skip:
        from speakingstyle_amd.models import hifigan as _H

        _H._WHOLE_SKIP.update(tuple(int(v) for v in g.split(":")) for g in args.whole_skip.split(","))
    if args.no_rb256:
        from speakingstyle_amd.models import hifigan as _H

        _H._RB256[0] = False
    if args.rb256_min_rows is not None:
        from speakingstyle_amd.models import hifigan as _H

        _H._RB256_MIN_ROWS[0] = args.rb256_min_rows
    if args.splitk is not None and cuda:
        from speakingstyle_amd.ops import hip

        hip.lib().ssamd_gemm_set_splitk(args.splitk)
    if args.no_skinny and cuda:
        from speakingstyle_amd.ops import hip

        hip.lib().ssamd_gemm_set_skinny(0)
    if args.gemm_addln_rows is not None and cuda:
        from speakingstyle_amd.ops import hip

        hip.GEMM_ADDLN_MAX_ROWS = args.gemm_addln_rows
    if args.skinny_w8 is not None and cuda:
        from speakingstyle_amd.ops import hip

        hip.lib().ssamd_gemm_set_skinny_w8(args.skinny_w8)
    if args.rf_short_tiles is not None and cuda:
        from speakingstyle_amd.ops import hip

        hip._RF_SHORT_MAX_TILES[0] = args.rf_short_tiles
    if args.rb_small_tiles is not None and cuda:
        from speakingstyle_amd.ops import hip

        hip._SMALL_MAX_TILES[0] = args.rb_small_tiles
    if args.skinny_cin32 and cuda:
        from speakingstyle_amd.ops import hip

        hip.lib().ssamd_gemm_set_skinny_any_cin(0)
    if args.addln_small_rows is not None and cuda:
        from speakingstyle_amd.ops import hip

        hip.lib().ssamd_addln_set_small_rows(args.addln_small_rows)
    if args.skinny_maxm is not None and cuda:
        from speakingstyle_amd.ops import hip

        hip.lib().ssamd_gemm_set_skinny_maxm(args.skinny_maxm)
    if args.splitk_tiny is not None and cuda:
        from speakingstyle_amd.ops import hip

        hip.lib().ssamd_gemm_set_splitk_tiny(args.splitk_tiny)
    if args.rb_whole_extra and cuda:
        from speakingstyle_amd.ops import hip

        hip.lib().ssamd_resblock_set_whole_extra(1)
    if args.bucketed:
        from speakingstyle_amd.models import hifigan

        hifigan._PACKED[0] = False
        args.packed_fs2 = False
    sy = B.synth_phase(args, rank, world, dev)
    if rank == 0:
        b1 = sy.get("b1")
        B.report({
            "b1_ms": None if b1 is None else round(1e3 * b1["median_s"], 3),
            "b1_rtf": None if b1 is None else b1["rtf"], "vocoder": "bucketed" if args.bucketed else "packed",
            "lead": sy.get("lead"),
            "fs2": "packed" if getattr(args, "packed_fs2", True) else "padded",
            "metric": "synth RTF (FastSpeech2 + style + HiFi-GAN, text ids -> int16 wav)",
            "value": sy["rtf"], "unit": "s wall / s audio", "higher_is_better": False, "n_gpus": world,
            "steps": args.synth_steps, "warmup": args.synth_warmup, "audio_seconds": round(sy["audio_s"], 2),
            "wall_s": round(sy["wall"], 4), "mel_frames_per_utt": round(sy["frames_per_utt"], 1),
            "vs_baseline": round(BASELINE_RTF / sy["rtf"], 1), "dtype": "bf16" if cuda else "fp32",
            "data": "synthetic text ids + reference mels, predicted durations (biased head), random-init weights",
            "config": {"model": f"FastSpeech2 ({args.synth_config}) + HiFi-GAN V1", "batch_per_gpu": args.synth_batch,
                       "parallelism": f"dp{world} (independent shards)"},
        })
    if world > 1:
        torch.distributed.destroy_process_group()


def main():
    args = parse()
    from speakingstyle_amd import benchmark as B

    if B.needs_launch(args.gpus):
        sys.exit(B.launch(os.path.abspath(__file__), args.gpus, sys.argv[1:]))
    from speakingstyle_amd.parallel import ddp

    ddp.fail_fast(run, args)


if __name__ == "__main__":
    main()
