"""Batch-1 synthesis latency breakdown (diagnostic): host time of each stage of the bench's b1 path
(FS2 forward enqueue, the mel-length D2H sync, vocoder enqueue, the int16 D2H), device-synchronised between
stages, median of N runs.  python tools/b1_probe.py [--config BC2013_GST] [--runs 30]"""
import argparse
import math
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="BC2013_GST")
ap.add_argument("--runs", type=int, default=30)
ap.add_argument("--phones", type=int, default=14)
args = ap.parse_args()

from speakingstyle_amd.config import load_named  # noqa: E402
from speakingstyle_amd.data.synthetic import SyntheticBatches  # noqa: E402
from speakingstyle_amd.models.fastspeech2 import FastSpeech2  # noqa: E402
from speakingstyle_amd.utils.model import get_vocoder  # noqa: E402

dev = torch.device("cuda", 0)
pp, mc, tc = load_named(args.config)
torch.manual_seed(0)
model = FastSpeech2(pp, mc).to(dev)
with torch.no_grad():
    lin = model.variance_adaptor.duration_predictor.linear_layer
    lin.weight.normal_(0.0, 0.005)
    lin.bias.fill_(math.log(8.1 + 1.0))
model.eval().set_compute_dtype(torch.bfloat16)
model.requires_grad_(False)
voc = get_vocoder(mc, dev)
mx = float(pp["preprocessing"]["audio"]["max_wav_value"])
b = SyntheticBatches(1, device=dev, seed=17, max_seq_len=mc["max_seq_len"],
                     phone_counts=np.array([args.phones])).make_batch()
S = torch.cuda.synchronize
rec = {k: [] for k in ("fs2_enqueue", "fs2_device", "len_d2h", "voc_enqueue", "voc_device", "wav_d2h", "total")}
with torch.no_grad():
    for i in range(args.runs + 5):
        S()
        t0 = time.perf_counter()
        out = model(b[2], b[3], b[4], b[5], b[6], b[7], b[8])
        t1 = time.perf_counter()
        S()
        t2 = time.perf_counter()
        lens = out[9].cpu()
        t3 = time.perf_counter()
        pcm = voc.infer(out[1].contiguous(), int16_scale=mx, lengths=lens.tolist())
        t4 = time.perf_counter()
        S()
        t5 = time.perf_counter()
        pcm.cpu()
        t6 = time.perf_counter()
        if i >= 5:
            for k, v in zip(rec, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5, t6 - t0)):
                rec[k].append(1e3 * v)
print({k: round(float(np.median(v)), 3) for k, v in rec.items()}, "mel frames", int(lens.sum()))
