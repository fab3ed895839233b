#!/usr/bin/env python
"""Standalone validation CLI (reference ``evaluate.py:91-122``; works without
``named_param``)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from speakingstyle_amd.config import load_configs  # noqa: E402
from speakingstyle_amd.train.evaluate import evaluate  # noqa: E402
from speakingstyle_amd.utils.model import get_model, get_vocoder  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--restore_step", type=int, default=30000)
    ap.add_argument("-p", "--preprocess_config", type=str, required=True)
    ap.add_argument("-m", "--model_config", type=str, required=True)
    ap.add_argument("-t", "--train_config", type=str, required=True)
    args = ap.parse_args(argv)
    configs = load_configs(args.preprocess_config, args.model_config, args.train_config)
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    model = get_model(args.restore_step, configs, device, train=False)
    message = evaluate(model, args.restore_step, configs, None, None)
    print(message)
    return message


if __name__ == "__main__":
    main()
