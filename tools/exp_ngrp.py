#!/usr/bin/env python
"""256x256 GEMM tile order (csrc/k_gemm.hip tile_of): N tiles split into G groups so that each
XCD keeps a 1/G slice of the weight image L2-resident.  Times G = 1 / 2 / 4, interleaved, warm
(back-to-back) and cold (L2 + MALL flushed), on the step's multi-N-tile shapes (GPU box)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from speakingstyle_amd.ops import hip  # noqa: E402
from speakingstyle_amd.ops.packing import PackInfo  # noqa: E402
from tools.gemm_census import timeit, timeit_cold  # noqa: E402


def main():
    dev = "cuda"
    M = int(os.environ.get("M", 108000))
    lens = torch.full((M // 800,), 800, device=dev, dtype=torch.int64)
    lens[-1] += M - lens.sum()
    pk = PackInfo.build(lens, int(lens.max()), M)
    setg = hip.lib().ssamd_gemm_set_ngrp
    for Cin, ks, N, packed in ((256, 9, 1024, True), (256, 1, 1024, False), (256, 1, 768, False),
                               (512, 5, 512, False), (80, 5, 512, False)):
        Mx = M if Cin != 512 and Cin != 80 else int(M * 1.6)
        x = torch.randn(1, Mx, Cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, ks, Cin, device=dev) / (ks * Cin) ** 0.5).to(torch.bfloat16)
        ri = pk.rinfo if packed else None
        pad = (ks - 1) // 2
        f = lambda: hip.conv_gemm_raw(x, w, None, 1, Mx, Cin, ks, 1, pad, N, 0, rinfo=ri)  # noqa: E731
        setg(1)
        ref = f().clone()
        res = {}
        for G in (1, 2, 4):
            if (N // 256) % G:
                continue
            setg(G)
            assert torch.equal(f(), ref), f"G={G}: output differs"
        warm = {G: [] for G in (1, 2, 4)}
        cold = {G: [] for G in (1, 2, 4)}
        for _ in range(3):
            for G in (1, 2, 4):
                if (N // 256) % G:
                    continue
                setg(G)
                warm[G].append(timeit(f, 10))
                cold[G].append(timeit_cold(f, 5))
        setg(1)
        for G in (1, 2, 4):
            if warm[G]:
                res[f"G{G}_us"] = round(min(warm[G]), 1)
                res[f"G{G}_cold_us"] = round(min(cold[G]), 1)
        print(json.dumps({"M": Mx, "Cin": Cin, "ks": ks, "N": N, "packed": packed, **res}), flush=True)


if __name__ == "__main__":
    main()
