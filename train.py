#!/usr/bin/env python
"""FastSpeech2 (+ speaking style) training CLI -- same flags as the reference's
``train.py`` (``--restore_step``, ``-p``, ``-m``, ``-t``).  Multi-GPU: launch one
process per GPU, e.g. ``torchrun --standalone --nproc-per-node 8 train.py -p ... -m ... -t ...``.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from speakingstyle_amd.config import load_configs  # noqa: E402
from speakingstyle_amd.train.loop import train  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--restore_step", type=int, default=0)
    ap.add_argument("-p", "--preprocess_config", type=str, required=True, help="path to preprocess.yaml")
    ap.add_argument("-m", "--model_config", type=str, required=True, help="path to model.yaml")
    ap.add_argument("-t", "--train_config", type=str, required=True, help="path to train.yaml")
    ap.add_argument("--auto_resume", action="store_true", help="resume from the latest checkpoint in ckpt_path")
    ap.add_argument("--synthetic", action="store_true", help="train on synthetic LJSpeech-shaped batches")
    ap.add_argument("--max_steps", type=int, default=None, help="override step.total_step")
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--no_vocoder", action="store_true")
    ap.add_argument("--fail_at_step", type=int, default=0, help="fault injection (resume tests)")
    args = ap.parse_args(argv)
    configs = load_configs(args.preprocess_config, args.model_config, args.train_config)
    return train(args, configs)


if __name__ == "__main__":
    main()
