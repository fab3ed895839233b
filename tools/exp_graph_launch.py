#!/usr/bin/env python
"""Host cost of a HIP-graph replay on this ROCm: (1) graphs of N trivial kernels, replay call time and
device time per replay; (2) the LibriTTS training step under train/graphs.py, host time of each part."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def trivial(n):
    x = torch.zeros(1024, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            x.add_(1)
    g.replay()
    torch.cuda.synchronize()
    hs = []
    t0 = time.perf_counter()
    for _ in range(20):
        h0 = time.perf_counter()
        g.replay()
        hs.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 20
    return {"nodes": n, "replay_call_ms": round(1e3 * sorted(hs)[10], 3), "wall_ms_per_replay": round(1e3 * wall, 3)}


def step_parts():
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.ops import hip
    from speakingstyle_amd.train.graphs import GraphedSteps
    from speakingstyle_amd.train.trainer import Trainer

    pp, mc, tc = load_named("LibriTTS")
    m = FastSpeech2(pp, mc).to("cuda").set_compute_dtype(torch.bfloat16)
    tr = Trainer(m, (pp, mc, tc), seed=1)
    tr.use_priority_stream()
    gs = GraphedSteps(tr, warm=1)
    b = SyntheticBatches(16, device="cuda", seed=5).make_batch()
    for _ in range(4):
        gs.step(b)
    torch.cuda.synchronize()
    parts = {}

    def tick(k, t):
        parts[k] = parts.get(k, 0.0) + (time.perf_counter() - t) * 1e3

    n = 10
    for _ in range(n):
        t = time.perf_counter()
        pb, key = gs.pad_batch(b)
        tick("pad", t)
        ent = gs.buckets[key]
        t = time.perf_counter()
        tr._step_seed()
        tick("seed", t)
        t = time.perf_counter()
        hip.refresh_stale_images(tr.opt.arena.data.device)
        tick("images", t)
        t = time.perf_counter()
        for dst, src in zip(ent["static"], pb):
            if isinstance(dst, torch.Tensor):
                dst.copy_(src, non_blocking=True)
        tick("copy", t)
        t = time.perf_counter()
        ent["graph"].replay()
        tick("replay", t)
        t = time.perf_counter()
        tr.step_tail(b, True, graphed=True)
        tick("tail", t)
    torch.cuda.synchronize()
    return {k: round(v / n, 3) for k, v in parts.items()}


if __name__ == "__main__":
    out = [trivial(n) for n in (10, 100, 700)]
    out.append({"libritts_step_host_ms": step_parts()})
    for o in out:
        print(json.dumps(o))
