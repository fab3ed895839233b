#!/usr/bin/env python
"""Sustained-load behaviour of the k9 decoder conv GEMM (GPU box): per-iteration time over a
long run (clock / power throttling) and with real-looking (ReLU-sparse) vs Gaussian inputs."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from speakingstyle_amd.ops import hip  # noqa: E402
from speakingstyle_amd.ops.packing import PackInfo  # noqa: E402


def main():
    dev = "cuda"
    M, Cin, ks, N = 64607, 256, 9, 1024
    lens = torch.full((M // 800,), 800, device=dev, dtype=torch.int64)
    lens[-1] += M - lens.sum()
    ri = PackInfo.build(lens, int(lens.max()), M).rinfo
    w = (torch.randn(N, ks, Cin, device=dev) / (ks * Cin) ** 0.5).to(torch.bfloat16)
    for kind in ("randn", "relu"):
        x = torch.randn(1, M, Cin, device=dev)
        if kind == "relu":
            x = torch.relu(x)
        x = x.to(torch.bfloat16)
        fn = lambda: hip.conv_gemm_raw(x, w, None, 1, M, Cin, ks, 1, 4, N, 0, rinfo=ri)  # noqa: E731
        evs = []
        t0 = time.time()
        for i in range(3000):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            evs.append((s, e))
        torch.cuda.synchronize()
        ts = [s.elapsed_time(e) * 1000 for s, e in evs]
        wall = time.time() - t0
        chunks = [round(sum(ts[i:i + 300]) / 300, 1) for i in range(0, 3000, 300)]
        print(json.dumps({"input": kind, "us_per_call_by_300": chunks, "wall_s": round(wall, 2)}), flush=True)


if __name__ == "__main__":
    main()
