"""Timing breakdown of the fused ResBlock layer kernel via its debug switch (skip phases)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.ops import hip  # noqa: E402

dev = "cuda"
hip.lib().ssamd_resblock_debug.argtypes = [hip.I]
for C, K, d, T, B in ((128, 11, 5, 36352, 16), (128, 3, 1, 36352, 16), (64, 11, 5, 72704, 16), (64, 3, 1, 72704, 16), (32, 11, 5, 145408, 16)):
    c1 = torch.nn.Conv1d(C, C, K, dilation=d, padding=d * (K - 1) // 2).to(dev)
    c2 = torch.nn.Conv1d(C, C, K, padding=(K - 1) // 2).to(dev)
    x = torch.randn(B, T, C, device=dev).to(torch.bfloat16)
    for dbg in ((0, 3) if C < 128 else (0, 1, 3, 7)):
        hip.lib().ssamd_resblock_debug(dbg)
        with torch.no_grad():
            for _ in range(2):
                hip.resblock_layer(x, c1, c2, d, 0.1)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(10):
                hip.resblock_layer(x, c1, c2, d, 0.1)
            torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / 10 * 1e3
        fl = 2 * 2 * B * T * C * C * K
        print(f"C={C} K={K} d={d} dbg={dbg}: {ms:.3f} ms  ({fl / ms / 1e9:.0f} TF/s if full)", flush=True)
hip.lib().ssamd_resblock_debug(0)
