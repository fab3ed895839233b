#!/usr/bin/env python
"""HiFi-GAN vocoder training CLI (reference ``hifigan/train.py`` flags).

  torchrun --standalone --nproc-per-node 8 hifigan_train.py --input_wavs_dir LJSpeech-1.1/wavs \\
      --input_training_file LJSpeech-1.1/training.txt --input_validation_file LJSpeech-1.1/validation.txt \\
      --checkpoint_path cp_hifigan --config config/hifigan/config.json
  fine-tuning on ground-truth-aligned mels:  ... --fine_tuning True --input_mels_dir ft_dataset
  plumbing (no corpus, CPU or GPU):          python hifigan_train.py --synthetic --training_steps 2

Implementation: ``speakingstyle_amd/vocoder/train.py``.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _bool(s):
    return str(s).lower() in ("1", "true", "yes", "y")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--group_name", default=None)
    ap.add_argument("--input_wavs_dir", default="LJSpeech-1.1/wavs")
    ap.add_argument("--input_mels_dir", default="ft_dataset")
    ap.add_argument("--input_training_file", default="LJSpeech-1.1/training.txt")
    ap.add_argument("--input_validation_file", default="LJSpeech-1.1/validation.txt")
    ap.add_argument("--checkpoint_path", default="cp_hifigan")
    ap.add_argument("--config", default=None)
    ap.add_argument("--training_epochs", default=3100, type=int)
    ap.add_argument("--stdout_interval", default=5, type=int)
    ap.add_argument("--checkpoint_interval", default=5000, type=int)
    ap.add_argument("--summary_interval", default=100, type=int)
    ap.add_argument("--validation_interval", default=1000, type=int)
    ap.add_argument("--fine_tuning", default=False, type=_bool)
    # additions
    ap.add_argument("--training_steps", type=int, default=0, help="stop after N steps (0 = run the epochs)")
    ap.add_argument("--batch_size", type=int, default=None, help="global batch (default: config batch_size)")
    ap.add_argument("--num_workers", type=int, default=4)
    ap.add_argument("--synthetic", action="store_true", help="generated tones instead of a corpus")
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args(argv)
    from speakingstyle_amd.parallel import ddp
    from speakingstyle_amd.vocoder.train import train

    return ddp.fail_fast(train, a)


if __name__ == "__main__":
    main()
