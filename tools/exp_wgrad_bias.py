#!/usr/bin/env python
"""Cost of the fused bias gradient in the 256x256 weight-gradient kernel: times conv_wgrad_raw with and
without ``with_bias`` on the training step's largest weight-gradient shapes, and checks db against an fp32
column sum.  Usage (GPU): python tools/exp_wgrad_bias.py [--iters 20]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from speakingstyle_amd import ops  # noqa: E402
from speakingstyle_amd.ops import hip  # noqa: E402
from exp_wgrad_pp import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    B = 200
    lens = torch.clamp(torch.normal(565.0, 150.0, (B,)), 100, 1000).to(torch.int64).to(dev)
    M, R = int(lens.max()), int(lens.sum())
    pk = ops.PackInfo.build(lens, M, R)
    for name, Cin, N, ks, packed, rows in (("dec ffn.w1 k9 256->1024 packed", 256, 1024, 9, True, R),
                                           ("dec ffn.w2 k1 1024->256", 1024, 256, 1, False, R),
                                           ("postnet k5 512->512", 512, 512, 5, False, 140000)):
        if packed:
            Bq, L, rinfo, cu = 1, rows, pk.rinfo, pk.cu
        else:
            Bq, L, rinfo, cu = 200, rows // 200, None, None
        x = torch.randn(Bq, L, Cin, device=dev).to(torch.bfloat16)
        dy = torch.randn(Bq, L, N, device=dev).to(torch.bfloat16)
        pad = (ks - 1) // 2
        flops = 2.0 * Bq * L * N * ks * Cin
        res = {"shape": name, "rows": Bq * L}
        _, db = hip.conv_wgrad_raw(x, dy, Bq, L, Cin, ks, 1, pad, N, with_bias=True, rinfo=rinfo, cu=cu)
        ref = dy.float().reshape(-1, N).sum(0)
        res["db_rel"] = float((db - ref).norm() / ref.norm())
        for wb in (True, False, True, False):
            us = timeit(lambda: hip.conv_wgrad_raw(x, dy, Bq, L, Cin, ks, 1, pad, N, with_bias=wb, rinfo=rinfo, cu=cu),
                        a.iters)
            res.setdefault("bias_us" if wb else "nobias_us", []).append(round(us, 1))
        res["TF_bias"] = round(flops / min(res["bias_us"]) / 1e6, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
