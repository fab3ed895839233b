#!/usr/bin/env python
"""Weight gradient of the decoder FFN conv (k9, 256->1024) on plain vs packed rows (1..200
sequences), and the postnet k5 conv: the two big64 wgrad read schedules (single wait per k-half /
immediate-offset reads) side by side on the same box, interleaved twice against clock drift."""
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
    for M, Cin, ks, N, seqs in ((64607, 256, 9, 1024, (0, 1, 80)), (106600, 512, 5, 512, (0,))):
        x = torch.randn(1, M, Cin, device=dev).to(torch.bfloat16)
        dy = torch.randn(1, M, N, device=dev).to(torch.bfloat16)
        pad = (ks - 1) // 2
        for nseq in seqs:
            ri = cu = None
            if nseq:
                lens = torch.full((nseq,), M // nseq, device=dev, dtype=torch.int64)
                lens[-1] += M - lens.sum()
                pk = PackInfo.build(lens, int(lens.max()), M)
                ri, cu = pk.rinfo, pk.cu
            fn = lambda: hip.conv_wgrad_raw(x, dy, 1, M, Cin, ks, 1, pad, N, with_bias=True, rinfo=ri, cu=cu)  # noqa
            res = {0: [], 1: []}
            for imm in (0, 1, 0, 1):
                hip.lib().ssamd_wgrad_set_imm(imm)
                res[imm].append(timeit(fn, 10))
            hip.lib().ssamd_wgrad_set_imm(-1)
            print(json.dumps({"M": M, "Cin": Cin, "ks": ks, "N": N, "nseq": nseq,
                              "single_wait_us": round(min(res[0]), 1), "imm_us": round(min(res[1]), 1),
                              "auto_us": round(timeit(fn, 10), 1)}), flush=True)


if __name__ == "__main__":
    main()
