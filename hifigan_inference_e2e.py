#!/usr/bin/env python
"""HiFi-GAN end-to-end CLI (reference ``hifigan/inference_e2e.py``): every ``.npy`` mel in
--input_mels_dir (e.g. FastSpeech2 output, [n_mels, T]) -> ``{name}_generated_e2e.wav``.

  python hifigan_inference_e2e.py --checkpoint_file cp_hifigan/g_02500000 [--input_mels_dir test_mel_files]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--input_mels_dir", default="test_mel_files")
    ap.add_argument("--output_dir", default="generated_files_from_mel")
    ap.add_argument("--checkpoint_file", required=True)
    ap.add_argument("--config", default=None, help="default: config.json next to the checkpoint")
    ap.add_argument("--batch_size", type=int, default=16)
    a = ap.parse_args(argv)
    from speakingstyle_amd.vocoder.infer import from_mels

    for p in from_mels(a.input_mels_dir, a.output_dir, a.checkpoint_file, config=a.config, batch_size=a.batch_size):
        print(p)


if __name__ == "__main__":
    main()
