#!/usr/bin/env python
"""GEMM variant sweep at encoder-sized M (B*T ~ 14k phoneme rows): which tile shape fills
256 CUs best when the 256x256 tiling yields only ~56 tiles.  GPU box only."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from speakingstyle_amd.ops import hip  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    dev = "cuda"
    B, L = 200, int(os.environ.get("L", 70))
    shapes = [("fc", 256, 256, 1), ("w2", 1024, 256, 1), ("qkv_dgrad", 768, 256, 1), ("w1_dgrad_k9", 1024, 256, 9),
              ("vp_k3", 256, 256, 3), ("qkv", 256, 768, 1), ("w1_k9", 256, 1024, 9), ("w2_dgrad", 256, 1024, 1)]
    for name, Cin, N, ks in shapes:
        x = torch.randn(B, L, Cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, ks, Cin, device=dev) / (Cin * ks) ** 0.5).to(torch.bfloat16)
        b = torch.zeros(N, device=dev)
        flops = 2.0 * B * L * N * ks * Cin
        rec = {"op": name, "M": B * L}
        for v in (-1, 0, 1, 2, 4, 5):
            hip.lib().ssamd_gemm_set_variant(v)
            try:
                t = timeit(lambda: hip.conv_gemm_raw(x, w, b, B, L, Cin, ks, 1, (ks - 1) // 2, N, 0))
                rec[f"v{v}_us"] = round(t, 1)
                rec[f"v{v}_TF"] = round(flops / t / 1e6, 1)
            except Exception as e:  # noqa: BLE001
                rec[f"v{v}"] = str(e)[:40]
        hip.lib().ssamd_gemm_set_variant(-1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
