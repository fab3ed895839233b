#!/usr/bin/env python
"""Weight-gradient split-count sweep at the training step's shapes (GPU box): time of
conv_wgrad_raw (split-M GEMM + slab reduction) vs the target block count (ssamd_wgrad_set_blocks),
to size the splits per shape instead of one global target."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from speakingstyle_amd.ops import hip  # noqa: E402
from tools.gemm_census import timeit  # noqa: E402


def main():
    dev = "cuda"
    shapes = [(64607, 256, 1, 256), (64607, 256, 1, 768), (64607, 1024, 1, 256), (64607, 256, 1, 1024),
              (64607, 256, 9, 1024), (10800, 256, 1, 256), (10800, 256, 3, 256), (10800, 256, 9, 1024),
              (10800, 1024, 1, 256), (106600, 512, 5, 512), (106600, 512, 5, 80), (64607, 256, 1, 80)]
    from speakingstyle_amd.ops.packing import PackInfo

    for M, Cin, ks, N, packed in [(64607, 256, 9, 1024, True), (64607, 1024, 1, 256, True)] + [s + (False,)
                                                                                              for s in shapes]:
        ri = cu = None
        if packed:
            lens = torch.full((M // 800,), 800, device=dev, dtype=torch.int64)
            lens[-1] += M - lens.sum()
            pk = PackInfo.build(lens, int(lens.max()), M)
            ri, cu = pk.rinfo, pk.cu
        x = torch.randn(1, M, Cin, device=dev).to(torch.bfloat16)
        dy = torch.randn(1, M, N, device=dev).to(torch.bfloat16)
        flops = 2.0 * M * N * ks * Cin
        rec = {"M": M, "Cin": Cin, "ks": ks, "N": N, "packed": packed}
        for blocks in (256, 512):
            hip.lib().ssamd_wgrad_set_blocks(blocks)
            t = timeit(lambda: hip.conv_wgrad_raw(x, dy, 1, M, Cin, ks, 1, (ks - 1) // 2, N, with_bias=True, rinfo=ri, cu=cu), 10)
            rec[f"b{blocks}_us"] = round(t, 1)
        hip.lib().ssamd_wgrad_set_blocks(0)
        t = timeit(lambda: hip.conv_wgrad_raw(x, dy, 1, M, Cin, ks, 1, (ks - 1) // 2, N, with_bias=True, rinfo=ri, cu=cu), 10)
        rec["auto_us"] = round(t, 1)
        hip.lib().ssamd_wgrad_set_reduce(1)
        rec["old_reduce_us"] = round(timeit(lambda: hip.conv_wgrad_raw(x, dy, 1, M, Cin, ks, 1, (ks - 1) // 2, N,
                                                                       with_bias=True, rinfo=ri, cu=cu), 10), 1)
        hip.lib().ssamd_wgrad_set_reduce(0)
        rec["auto_TF"] = round(flops / t / 1e6, 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
