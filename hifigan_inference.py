#!/usr/bin/env python
"""HiFi-GAN copy-synthesis CLI (reference ``hifigan/inference.py``): every wav in
--input_wavs_dir -> mel -> waveform ``{name}_generated.wav`` in --output_dir.

  python hifigan_inference.py --checkpoint_file cp_hifigan/g_02500000 [--input_wavs_dir test_files]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--input_wavs_dir", default="test_files")
    ap.add_argument("--output_dir", default="generated_files")
    ap.add_argument("--checkpoint_file", required=True)
    ap.add_argument("--config", default=None, help="default: config.json next to the checkpoint")
    ap.add_argument("--batch_size", type=int, default=16)
    a = ap.parse_args(argv)
    from speakingstyle_amd.vocoder.infer import from_wavs

    for p in from_wavs(a.input_wavs_dir, a.output_dir, a.checkpoint_file, config=a.config, batch_size=a.batch_size):
        print(p)


if __name__ == "__main__":
    main()
