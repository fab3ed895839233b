#!/usr/bin/env python
"""Prepare corpora for Montreal Forced Aligner (reference ``prepare_align.py``):
resampled, peak-normalised int16 wavs + ``.lab`` transcripts under ``raw_path``."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from speakingstyle_amd.config import load_yaml, normalize_preprocess_config  # noqa: E402
from speakingstyle_amd.data.preprocess import prepare_align  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("config", type=str, help="path to preprocess.yaml")
    a = ap.parse_args(argv)
    n = prepare_align(normalize_preprocess_config(load_yaml(a.config)))
    print(f"prepared {n} utterances")
    return n


if __name__ == "__main__":
    main()
