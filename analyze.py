#!/usr/bin/env python
"""Research tooling CLI (the reference's notebooks as commands).

  variance distributions, ground truth vs predictions (notebooks/variance_control_distbn.ipynb):
    python analyze.py variance --restore_step 900000 -p P -m M -t T [--source val.txt] [--out_dir analysis]
        [--pitch_control 1.2 --energy_control 1 --duration_control 1] [--outlier_k 3]
  one-batch forward / style-encoder inspection (notebooks/ref_encoder.ipynb):
    python analyze.py inspect --restore_step 0 -p P -m M -t T [--synthetic]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("command", choices=["variance", "inspect"])
    ap.add_argument("--restore_step", type=int, default=0)
    ap.add_argument("--seed", type=int, default=1234, help="parameter init seed (restore_step 0: reproducible runs)")
    ap.add_argument("-p", "--preprocess_config", required=True)
    ap.add_argument("-m", "--model_config", required=True)
    ap.add_argument("-t", "--train_config", required=True)
    ap.add_argument("--source", default=None, help="metadata list (default: <preprocessed_path>/val.txt)")
    ap.add_argument("--out_dir", default=None)
    ap.add_argument("--pitch_control", type=float, default=1.0)
    ap.add_argument("--energy_control", type=float, default=1.0)
    ap.add_argument("--duration_control", type=float, default=1.0)
    ap.add_argument("--outlier_k", type=float, default=3.0)
    ap.add_argument("--batch_size", type=int, default=8)
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args(argv)

    import torch

    from speakingstyle_amd.config import load_configs
    from speakingstyle_amd.utils.model import get_model

    configs = load_configs(a.preprocess_config, a.model_config, a.train_config)
    dev = torch.device("cuda" if torch.cuda.is_available() and not a.cpu else "cpu")
    torch.manual_seed(a.seed)
    model = get_model(a.restore_step, configs, dev, train=False, ignore_layers=configs[2].get("ignore_layers", []))
    if a.command == "variance":
        from speakingstyle_amd.analysis.variance import analyze

        src = a.source or os.path.join(configs[0]["path"]["preprocessed_path"], "val.txt")
        rep = analyze(model, configs, src, dev, (a.pitch_control, a.energy_control, a.duration_control), a.out_dir,
                      a.batch_size, a.outlier_k)
    else:
        from speakingstyle_amd.analysis.inspect import inspect_batch

        rep = inspect_batch(model, configs, dev, synthetic=a.synthetic)
    print(json.dumps(rep, indent=2))
    return rep


if __name__ == "__main__":
    main()
