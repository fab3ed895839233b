#!/usr/bin/env python
"""Feature extraction CLI (reference ``preprocess.py``).  Accepts both the
positional form shown in the reference README and the ``-preprocess_config``
flag form (reference D4: its CLI passes two args to a one-arg constructor)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from speakingstyle_amd.config import load_yaml, normalize_preprocess_config  # noqa: E402
from speakingstyle_amd.data.preprocess import Preprocessor  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", help="path to preprocess.yaml")
    ap.add_argument("-preprocess_config", "--preprocess_config", "-p", dest="pconf", default=None)
    ap.add_argument("-model_config", "--model_config", "-m", dest="mconf", default=None)
    ap.add_argument("--workers", type=int, default=max(1, (os.cpu_count() or 2) // 2))
    a = ap.parse_args(argv)
    path = a.pconf or a.config
    if not path:
        ap.error("a preprocess.yaml is required")
    cfg = normalize_preprocess_config(load_yaml(path))
    return Preprocessor(cfg).build_from_path(workers=a.workers)


if __name__ == "__main__":
    main()
