#!/usr/bin/env python
"""Split-K slice-count sweep for tile-poor, long-K implicit GEMMs (encoder-sized M): time per S
(ssamd_gemm_set_splitk) and the max-abs difference to the unsplit result (GPU box)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from speakingstyle_amd.ops import hip  # noqa: E402
from tools.gemm_census import timeit  # noqa: E402


def main():
    dev = "cuda"
    for M, Cin, ks, N in ((10800, 1024, 9, 256), (10800, 256, 9, 1024), (5000, 1024, 9, 256), (20000, 1024, 9, 256),
                          (10800, 512, 5, 512)):
        x = torch.randn(1, M, Cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, ks, Cin, device=dev) / (ks * Cin) ** 0.5).to(torch.bfloat16)
        r = torch.randn(1, M, N, device=dev).to(torch.bfloat16)
        pad = (ks - 1) // 2
        fl = 2.0 * M * N * ks * Cin
        rec = {"M": M, "Cin": Cin, "ks": ks, "N": N}
        hip.lib().ssamd_gemm_set_splitk(0)
        ref = hip.conv_gemm_raw(x, w, None, 1, M, Cin, ks, 1, pad, N, 0, resid=r)
        for S in (0, 2, 3, 4, 6, 8, -1):
            hip.lib().ssamd_gemm_set_splitk(S)
            fn = lambda: hip.conv_gemm_raw(x, w, None, 1, M, Cin, ks, 1, pad, N, 0, resid=r)  # noqa: E731
            t = timeit(fn, 10)
            d = (fn().float() - ref.float()).abs().max().item()
            rec[f"S{S}_us"] = round(t, 1)
            rec[f"S{S}_maxdiff"] = round(d, 4)
        hip.lib().ssamd_gemm_set_splitk(-1)
        rec["auto_TF"] = round(fl / rec["S-1_us"] / 1e6, 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
