#!/usr/bin/env python
"""LDS-DMA through buffer descriptors (csrc/k_gemm.hip: big64 wgrad and forward/dgrad GEMM, BUF) vs
the flat global_load_lds path: bitwise-equal outputs and the time of each, interleaved (GPU box)."""
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
    M = int(os.environ.get("M", 108000))
    lens = torch.randint(300, 1000, (M // 600 + 1,), device=dev, dtype=torch.int64)
    lens = lens[torch.cumsum(lens, 0) <= M]
    lens[-1] += M - int(lens.sum())
    pk = PackInfo.build(lens, int(lens.max()), M)
    setb = hip.lib().ssamd_wgrad_set_buf
    shapes = ((256, 9, 1024, True, 1, M), (1024, 1, 256, False, 1, M), (256, 1, 768, False, 1, M),
              (256, 1, 256, False, 1, M), (512, 5, 512, False, 200, 860), (256, 9, 1024, False, 200, 90),
              (256, 3, 256, False, 200, 90), (80, 5, 512, False, 200, 860))
    for Cin, ks, N, packed, B, L in shapes:
        Mx = B * L
        x = torch.randn(1, Mx, Cin, device=dev).to(torch.bfloat16)
        dy = torch.randn(1, Mx, N, device=dev).to(torch.bfloat16)
        ri, cu = (pk.rinfo, pk.cu) if packed else (None, None)
        pad = (ks - 1) // 2
        Bv, Lv = (1, Mx) if packed else (B, L)
        f = lambda: hip.conv_wgrad_raw(x, dy, Bv, Lv, Cin, ks, 1, pad, N, with_bias=True, rinfo=ri, cu=cu)  # noqa
        setb(0)
        ref = [t.clone() for t in f()]
        setb(1)
        out = f()
        same = all(torch.equal(a, b) for a, b in zip(ref, out))
        t = {0: [], 1: []}
        for b in (0, 1, 0, 1, 0, 1):
            setb(b)
            t[b].append(timeit(f, 10))
        setb(1)
        print(json.dumps({"M": Mx, "Cin": Cin, "ks": ks, "N": N, "packed": packed, "bitwise_equal": same,
                          "flat_us": round(min(t[0]), 1), "buf_us": round(min(t[1]), 1)}), flush=True)


def main_fwd():
    dev = "cuda"
    M = int(os.environ.get("M", 108000))
    lens = torch.randint(300, 1000, (M // 600 + 1,), device=dev, dtype=torch.int64)
    lens = lens[torch.cumsum(lens, 0) <= M]
    lens[-1] += M - int(lens.sum())
    pk = PackInfo.build(lens, int(lens.max()), M)
    setb = hip.lib().ssamd_gemm_set_buf
    shapes = ((256, 9, 1024, True, 1, M), (1024, 9, 256, True, 1, M), (256, 1, 768, False, 1, M),
              (1024, 1, 256, False, 1, M), (256, 1, 1024, False, 1, M), (512, 5, 512, False, 200, 860),
              (256, 3, 256, False, 200, 90), (1024, 9, 256, False, 200, 90), (256, 9, 1024, False, 200, 90))
    for Cin, ks, N, packed, B, L in shapes:
        Mx = B * L
        x = torch.randn(1, Mx, Cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, ks, Cin, device=dev) / (ks * Cin) ** 0.5).to(torch.bfloat16)
        bias = torch.randn(N, device=dev)
        ri = pk.rinfo if packed else None
        pad = (ks - 1) // 2
        Bv, Lv = (1, Mx) if packed else (B, L)
        f = lambda: hip.conv_gemm_raw(x, w, bias, Bv, Lv, Cin, ks, 1, pad, N, 1, rinfo=ri)  # noqa: E731
        setb(0)
        ref = f().clone()
        setb(1)
        same = torch.equal(f(), ref)
        t = {0: [], 1: []}
        for b in (0, 1, 0, 1, 0, 1):
            setb(b)
            t[b].append(timeit(f, 10))
        setb(1)
        print(json.dumps({"kind": "fwd", "M": Mx, "Cin": Cin, "ks": ks, "N": N, "packed": packed,
                          "bitwise_equal": same, "flat_us": round(min(t[0]), 1), "buf_us": round(min(t[1]), 1)}),
              flush=True)


def main_ring():
    """256x128 ring kernel (forced variant 2) on the encoder / predictor / mel-head shapes."""
    dev = "cuda"
    setb = hip.lib().ssamd_gemm_set_buf
    hip.lib().ssamd_gemm_set_variant(2)
    for Cin, ks, N, B, L in ((256, 3, 256, 200, 90), (256, 1, 80, 1, 108000), (1024, 1, 256, 200, 90),
                             (256, 1, 256, 200, 90), (256, 9, 1024, 200, 90)):
        Mx = B * L
        x = torch.randn(1, Mx, Cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, ks, Cin, device=dev) / (ks * Cin) ** 0.5).to(torch.bfloat16)
        bias = torch.randn(N, device=dev)
        pad = (ks - 1) // 2
        f = lambda: hip.conv_gemm_raw(x, w, bias, B, L, Cin, ks, 1, pad, N, 1)  # noqa: E731
        setb(0)
        ref = f().clone()
        setb(1)
        same = torch.equal(f(), ref)
        t = {0: [], 1: []}
        for b in (0, 1, 0, 1, 0, 1):
            setb(b)
            t[b].append(timeit(f, 10))
        setb(1)
        print(json.dumps({"kind": "ring", "M": Mx, "Cin": Cin, "ks": ks, "N": N, "bitwise_equal": same,
                          "flat_us": round(min(t[0]), 1), "buf_us": round(min(t[1]), 1)}), flush=True)
    hip.lib().ssamd_gemm_set_variant(-1)


if __name__ == "__main__":
    if os.environ.get("RING", "1") == "1":
        main_ring()
    if os.environ.get("FWD", "1") == "1":
        main_fwd()
    main()
