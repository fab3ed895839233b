#!/usr/bin/env python
"""A/B of the ping-pong wgrad main loop (ssamd_wgrad_set_pp) against the double-buffered one on the
training step's weight-gradient shapes: dW / db must be bitwise equal (same per-accumulator row
order), then time both (kernel + slab reduce, same process, alternating, warm).  JSON per shape.
Usage (GPU): python tools/exp_wgrad_pp.py [--iters 20]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from speakingstyle_amd import ops  # noqa: E402
from speakingstyle_amd.ops import hip  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    B = 200
    lens = torch.clamp(torch.normal(565.0, 150.0, (B,)), 100, 1000).to(torch.int64).to(dev)
    M = int(lens.max())
    R = int(lens.sum())
    pk = ops.PackInfo.build(lens, M, R)
    shapes = [  # name, Cin, N, ks, packed, rows
        ("dec ffn.w1 k9 256->1024 packed", 256, 1024, 9, True, R),
        ("dec ffn.w2 k1 1024->256", 1024, 256, 1, False, R),
        ("dec qkv 256->768", 256, 768, 1, False, R),
        ("dec fc 256->256", 256, 256, 1, False, R),
        ("postnet k5 512->512", 512, 512, 5, False, 140000),
        ("postnet k5 80->512", 80, 512, 5, False, 140000),
        ("enc ffn.w1 k9 256->1024", 256, 1024, 9, False, 14000),
    ]
    for name, Cin, N, ks, packed, rows in shapes:
        if packed:
            Bq, L, rinfo, cu = 1, rows, pk.rinfo, pk.cu
        else:
            Bq, L, rinfo, cu = 200, rows // 200, None, None
        x = torch.randn(Bq, L, Cin, device=dev).to(torch.bfloat16)
        dy = torch.randn(Bq, L, N, device=dev).to(torch.bfloat16)
        pad = (ks - 1) // 2

        def run():
            return hip.conv_wgrad_raw(x, dy, Bq, L, Cin, ks, 1, pad, N, with_bias=True, rinfo=rinfo, cu=cu)

        hip.lib().ssamd_wgrad_set_pp(0)
        w0, b0 = run()
        w0, b0 = w0.clone(), b0.clone()
        hip.lib().ssamd_wgrad_set_pp(1)
        w1, b1 = run()
        same = bool(torch.equal(w0, w1) and torch.equal(b0, b1))
        t = {0: [], 1: []}
        for rep in range(3):
            for v in (0, 1):
                hip.lib().ssamd_wgrad_set_pp(v)
                t[v].append(timeit(run, a.iters))
        hip.lib().ssamd_wgrad_set_pp(0)
        flops = 2.0 * Bq * L * N * ks * Cin
        t0, t1 = min(t[0]), min(t[1])
        print(json.dumps({"shape": name, "rows": Bq * L, "bitwise_equal": same, "base_us": round(t0, 1),
                          "pp_us": round(t1, 1), "base_TF": round(flops / t0 / 1e6, 1),
                          "pp_TF": round(flops / t1 / 1e6, 1), "speedup": round(t0 / t1, 3)}), flush=True)


if __name__ == "__main__":
    main()
