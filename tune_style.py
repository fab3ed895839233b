#!/usr/bin/env python
"""Tune the GST style-token bank from human-annotated utterances (the reference's research goal,
README.md:3-7; see speakingstyle_amd/train/style_tuning.py for the procedure).

  python tune_style.py -p config/BC2013_GST/preprocess.yaml -m config/BC2013_GST/model.yaml \
      -t config/BC2013_GST/train.yaml --restore_step 100000 --annotations styles.txt \
      [--steps 300 --lr 1e-2 --mse_weight 1.0 --tune_projections --out_step 100001]

``styles.txt`` lines: ``basename|speaker|token_index`` or ``basename|speaker|w0,w1,...``.
Writes ``{ckpt_path}/{out_step}.pth.tar`` (reference checkpoint layout) with the tuned bank;
synthesize with ``synthesize.py --restore_step {out_step} --style_weights ...``.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from speakingstyle_amd.config import load_configs  # noqa: E402
from speakingstyle_amd.train.style_tuning import StyleTokenTuner, parse_annotations  # noqa: E402
from speakingstyle_amd.utils.model import ckpt_file, get_model, save_checkpoint  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-p", "--preprocess_config", required=True)
    ap.add_argument("-m", "--model_config", required=True)
    ap.add_argument("-t", "--train_config", required=True)
    ap.add_argument("--restore_step", type=int, required=True)
    ap.add_argument("--annotations", required=True)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--lr", type=float, default=1e-2)
    ap.add_argument("--mse_weight", type=float, default=1.0)
    ap.add_argument("--tune_projections", action="store_true", help="also tune the token key/value projections")
    ap.add_argument("--out_step", type=int, default=None, help="checkpoint step to write (default restore_step + 1)")
    args = ap.parse_args(argv)

    configs = load_configs(args.preprocess_config, args.model_config, args.train_config)
    pp, mc, tc = configs
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    model = get_model(args.restore_step, configs, device, train=False)
    if getattr(model, "gst", None) is None:
        sys.exit("the model config has no GST block (gst: use_gst: true)")
    n_tok = model.gst.embed.shape[0]
    names, mels, targets = parse_annotations(args.annotations, pp["path"]["preprocessed_path"], n_tok)
    tuner = StyleTokenTuner(model, lr=args.lr, steps=args.steps, mse_weight=args.mse_weight,
                            tune_projections=args.tune_projections)
    res = tuner.fit(mels, targets, log_every=max(1, args.steps // 10))
    print(f"{len(names)} annotated utterances, argmax-token agreement {res['accuracy']:.3f}")
    out = ckpt_file(tc, args.out_step if args.out_step is not None else args.restore_step + 1)
    save_checkpoint(out, model, step=args.out_step)
    print("wrote", out)


if __name__ == "__main__":
    main()
