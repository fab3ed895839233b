#!/usr/bin/env python
"""s_setprio 1 for the second half of the 8-wave big64 GEMM / wgrad blocks (MI355X_MICROARCH
"static priority for the younger half"): time with and without, interleaved, on the step's
largest shapes (GPU box)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from speakingstyle_amd.ops import hip  # noqa: E402
from speakingstyle_amd.ops.packing import PackInfo  # noqa: E402
from tools.gemm_census import timeit  # noqa: E402


def main():
    dev = "cuda"
    M = 64607
    lens = torch.full((M // 800,), 800, device=dev, dtype=torch.int64)
    lens[-1] += M - lens.sum()
    pk = PackInfo.build(lens, int(lens.max()), M)
    for Cin, ks, N, packed in ((256, 9, 1024, True), (1024, 9, 256, True), (512, 5, 512, False), (256, 1, 768, False),
                               (1024, 1, 256, False)):
        x = torch.randn(1, M, Cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, ks, Cin, device=dev) / (ks * Cin) ** 0.5).to(torch.bfloat16)
        dy = torch.randn(1, M, N, device=dev).to(torch.bfloat16)
        ri, cu = (pk.rinfo, pk.cu) if packed else (None, None)
        pad = (ks - 1) // 2
        f = lambda: hip.conv_gemm_raw(x, w, None, 1, M, Cin, ks, 1, pad, N, 0, rinfo=ri)  # noqa: E731
        wg = lambda: hip.conv_wgrad_raw(x, dy, 1, M, Cin, ks, 1, pad, N, with_bias=True, rinfo=ri, cu=cu)  # noqa
        res = {}
        for name, fn in (("fwd", f), ("wgrad", wg)):
            t = {0: [], 1: []}
            setp = hip.lib().ssamd_gemm_set_prio if name == "fwd" else hip.lib().ssamd_wgrad_set_prio
            for p in (0, 1, 0, 1):
                setp(p)
                t[p].append(timeit(fn, 10))
            setp(-1 if name == "fwd" else 1)
            res[f"{name}_us"] = round(min(t[0]), 1)
            res[f"{name}_prio_us"] = round(min(t[1]), 1)
        print(json.dumps({"Cin": Cin, "ks": ks, "N": N, "packed": packed, **res}), flush=True)


if __name__ == "__main__":
    main()
