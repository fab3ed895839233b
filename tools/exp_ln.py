#!/usr/bin/env python
"""Micro-benchmark: d=256 GEMM + residual/LayerNorm tail, fused in the GEMM epilogue vs the
separate addln kernel (fc: K=256, w2: K=1024), with and without dropout.  GPU box only."""
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
    return s.elapsed_time(e) / iters * 1000.0  # us


def main():
    dev = "cuda"
    R = int(os.environ.get("ROWS", 100000))
    res = torch.randn(1, R, 256, device=dev).to(torch.bfloat16)
    lw = torch.ones(256, device=dev)
    lb = torch.zeros(256, device=dev)
    for K in (256, 1024):
        x = torch.randn(1, R, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(256, K, 1, device=dev) / K ** 0.5)
        wi = hip.weight_fwd(w)
        b = torch.zeros(256, device=dev)
        out = {"K": K, "rows": R}
        out["gemm_us"] = timeit(lambda: hip.conv_gemm_raw(x, wi, b, 1, R, K, 1, 1, 0, 256))
        for p in (0.0, 0.1):
            def fused():
                sp = hip.ln_spec(res, lw, lb, pre_drop=p, training=True)
                return hip.conv_gemm_ln_raw(x, wi, b, 1, R, K, 1, 1, 0, sp)

            def sep():
                a = hip.conv_gemm_raw(x, wi, b, 1, R, K, 1, 1, 0, 256)
                return hip.add_layernorm(a, res, lw, lb, pre_drop=p, training=True)

            out[f"fused_p{p}_us"] = timeit(fused)
            out[f"separate_p{p}_us"] = timeit(sep)
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
