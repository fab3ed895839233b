#!/usr/bin/env python
"""Per-tensor gradient error of one full FastSpeech2 forward+backward, HIP bf16 vs torch fp32
(the measurement behind the tolerance of ``tests/test_kernels_gpu.py::test_model_step_hip_vs_reference``).

Prints, per config, the relative L2 error of every parameter gradient grouped by module, sorted.
Usage (GPU): python tools/grad_err_budget.py [LJSpeech LibriTTS BC2013 BC2013_GST]"""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp(min=1e-12)).item()


def run(cfg_name, seed=9):
    from speakingstyle_amd import ops
    from speakingstyle_amd.benchmark import n_speakers_of
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.models.loss import FastSpeech2Loss
    from speakingstyle_amd.train.optim import FlatArena

    pp, mc, tc = load_named(cfg_name)
    torch.manual_seed(seed)
    m = FastSpeech2(pp, mc).to("cuda").eval()
    mr = copy.deepcopy(m)
    m.set_compute_dtype(torch.bfloat16)
    FlatArena(list(reversed(list(m.parameters()))), groups=m.fused_param_groups())
    nspk = n_speakers_of(pp) if mc.get("multi_speaker") else 1
    b = SyntheticBatches(4, device="cuda", seed=11, phone_counts=[40, 55, 61, 20], n_speakers=nspk).make_batch()
    lossf = FastSpeech2Loss(pp, tc)
    out = m(*b[2:])
    lossf(b, out, m.film_scalars())[0].backward()
    ops.set_backend("reference")
    try:
        outr = mr(*b[2:])
        lossf(b, outr, mr.film_scalars())[0].backward()
    finally:
        ops.set_backend(None)
    gr = dict(mr.named_parameters())
    rows = []
    for n, p in m.named_parameters():
        g = p.grad
        if g is None or gr[n].grad is None or gr[n].grad.norm() <= 1e-6 or p.numel() == 1:
            continue
        rows.append((rel(g, gr[n].grad), n))
    rows.sort(reverse=True)
    print(f"== {cfg_name}: mel rel {rel(out[1], outr[1]):.4f}, {len(rows)} tensors; "
          f"max {rows[0][0]:.4f}, p90 {rows[len(rows) // 10][0]:.4f}, median {rows[len(rows) // 2][0]:.4f}")
    for r, n in rows[:15]:
        print(f"   {r:.4f}  {n}")


if __name__ == "__main__":
    for c in (sys.argv[1:] or ["LJSpeech", "LibriTTS", "BC2013", "BC2013_GST"]):
        run(c)
