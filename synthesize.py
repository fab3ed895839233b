#!/usr/bin/env python
"""Synthesis CLI -- reference flags (``synthesize.py:153-225``) plus word-level
prosody control and GST style weights.

  single:  python synthesize.py --mode single --text "..." [--ref_audio x.wav] --restore_step N -p -m -t
  batch:   python synthesize.py --mode batch --source val.txt --restore_step N -p -m -t
  word-level control: --word_pitch 1,1.3,0.8 --word_energy ... --word_duration ... (one factor per word)
  GST:     --style_weights 0.5,0,0,...   (one weight per style token)
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch.utils.data import DataLoader  # noqa: E402

from speakingstyle_amd.config import load_configs  # noqa: E402
from speakingstyle_amd.data.dataset import TextDataset  # noqa: E402
from speakingstyle_amd.infer.synthesis import single_batch, synthesize, word_level_controls  # noqa: E402
from speakingstyle_amd.text import g2p  # noqa: E402
from speakingstyle_amd.utils.model import get_model, get_vocoder  # noqa: E402


def _floats(s):
    return None if s is None else [float(x) for x in s.split(",") if x.strip()]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--restore_step", type=int, required=True)
    ap.add_argument("--mode", type=str, choices=["batch", "single"], required=True)
    ap.add_argument("--source", type=str, default=None)
    ap.add_argument("--text", type=str, default=None)
    ap.add_argument("--ref_audio", type=str, default=None)
    ap.add_argument("--speaker_id", type=int, default=0, help="speaker id (multi-speaker models)")
    ap.add_argument("-p", "--preprocess_config", type=str, required=True)
    ap.add_argument("-m", "--model_config", type=str, required=True)
    ap.add_argument("-t", "--train_config", type=str, required=True)
    ap.add_argument("--pitch_control", type=float, default=1.0)
    ap.add_argument("--energy_control", type=float, default=1.0)
    ap.add_argument("--duration_control", type=float, default=1.0)
    ap.add_argument("--word_pitch", type=str, default=None)
    ap.add_argument("--word_energy", type=str, default=None)
    ap.add_argument("--word_duration", type=str, default=None)
    ap.add_argument("--style_weights", type=str, default=None)
    ap.add_argument("--batch_size", type=int, default=8)
    ap.add_argument("--plot", action="store_true", help="also write mel/pitch/energy PNGs")
    ap.add_argument("--result_path", type=str, default=None)
    args = ap.parse_args(argv)
    if args.mode == "batch":
        assert args.source is not None and args.text is None
    else:
        assert args.source is None and args.text is not None

    configs = load_configs(args.preprocess_config, args.model_config, args.train_config)
    pp, mc, tc = configs
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    model = get_model(args.restore_step, configs, device, train=False, ignore_layers=tc.get("ignore_layers", []))
    vocoder = get_vocoder(mc, device)
    result_path = args.result_path or tc["path"]["result_path"]
    os.makedirs(result_path, exist_ok=True)
    controls = [args.pitch_control, args.energy_control, args.duration_control]
    use_ref = True
    if args.mode == "batch":
        ds = TextDataset(args.source, pp, tc)
        batchs = list(DataLoader(ds, batch_size=args.batch_size, collate_fn=ds.collate_fn))
    else:
        lexicon = g2p.load_lexicon(pp["path"]["lexicon_path"], pp["preprocessing"]["text"].get("language", "en"))
        batch, phones, use_ref = single_batch(args.text, pp, args.speaker_id, args.ref_audio, lexicon)
        batchs = [batch]
        if any(v is not None for v in (args.word_pitch, args.word_energy, args.word_duration)):
            groups = g2p.word_groups(args.text, lexicon)
            for i, wv in enumerate((args.word_pitch, args.word_energy, args.word_duration)):
                if wv is not None:
                    controls[i] = word_level_controls(groups, _floats(wv), controls[i])
    sw = _floats(args.style_weights)
    synthesize(model, configs, vocoder, batchs, controls, result_path, plot=args.plot, use_ref=use_ref,
               style_weights=sw)
    print("wrote results to", result_path)


if __name__ == "__main__":
    main()
