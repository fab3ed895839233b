#!/usr/bin/env python
"""Micro-benchmarks of the hot HIP kernels at the headline model's shapes.

Reports achieved TFLOP/s (GEMM-shaped) or GB/s (memory-bound) per kernel, and
the hipBLASLt number for the plain-GEMM equivalent (torch.matmul) as a yardstick.
Usage (GPU box): python tools/bench_kernels.py [--rows 160000] [--iters 20]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

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
    return s.elapsed_time(e) / iters  # ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=160000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only-attn", action="store_true")
    args = ap.parse_args()
    dev = "cuda"
    B = 200
    L = args.rows // B
    R = B * L
    res = []
    shapes = [  # name, Cin, N, ks
        ("ffn.w1 (k9 256->1024)", 256, 1024, 9),
        ("ffn.w2 (k1 1024->256)", 1024, 256, 1),
        ("ffn.w1 dgrad (k9 1024->256)", 1024, 256, 9),
        ("ffn.w2 dgrad (k1 256->1024)", 256, 1024, 1),
        ("qkv (256->768)", 256, 768, 1),
        ("attn fc (256->256)", 256, 256, 1),
        ("postnet (k5 512->512)", 512, 512, 5),
        ("postnet in (k5 80->512)", 80, 512, 5),
    ]
    for name, Cin, N, ks in ([] if args.only_attn else shapes):
        x = torch.randn(B, L, Cin, device=dev).to(torch.bfloat16)
        w = torch.randn(N, ks, Cin, device=dev).to(torch.bfloat16)
        bias = torch.randn(N, device=dev)
        pad = (ks - 1) // 2
        flops = 2.0 * R * N * ks * Cin
        hip.lib().ssamd_gemm_set_variant(0)
        t_lds = timeit(lambda: hip.conv_gemm_raw(x, w, bias, B, L, Cin, ks, 1, pad, N, 1), args.iters)
        hip.lib().ssamd_gemm_set_variant(2)
        t_ring = timeit(lambda: hip.conv_gemm_raw(x, w, bias, B, L, Cin, ks, 1, pad, N, 1), args.iters)
        hip.lib().ssamd_gemm_set_variant(3)
        t_big = timeit(lambda: hip.conv_gemm_raw(x, w, bias, B, L, Cin, ks, 1, pad, N, 1), args.iters)
        hip.lib().ssamd_gemm_set_variant(4)
        t_b64 = timeit(lambda: hip.conv_gemm_raw(x, w, bias, B, L, Cin, ks, 1, pad, N, 1), args.iters)
        hip.lib().ssamd_gemm_set_variant(5)
        t_pers = timeit(lambda: hip.conv_gemm_raw(x, w, bias, B, L, Cin, ks, 1, pad, N, 1), args.iters)
        hip.lib().ssamd_gemm_set_variant(-1)
        t = timeit(lambda: hip.conv_gemm_raw(x, w, bias, B, L, Cin, ks, 1, pad, N, 1), args.iters)
        t_lds = min(t_lds, timeit(lambda: hip.conv_gemm_raw(x, w, bias, B, L, Cin, ks, 1, pad, N, 1), 1) * 0 + t_lds)
        dy = torch.randn(B, L, N, device=dev).to(torch.bfloat16)
        tw = timeit(lambda: hip.conv_wgrad_raw(x, dy, B, L, Cin, ks, 1, pad, N, with_bias=True), args.iters)
        hip.lib().ssamd_wgrad_set_variant(0)
        tw_old = timeit(lambda: hip.conv_wgrad_raw(x, dy, B, L, Cin, ks, 1, pad, N, with_bias=True), args.iters)
        hip.lib().ssamd_wgrad_set_variant(1)
        tw_r = timeit(lambda: hip.conv_wgrad_raw(x, dy, B, L, Cin, ks, 1, pad, N, with_bias=True), args.iters)
        hip.lib().ssamd_wgrad_set_variant(2)
        tw_32 = timeit(lambda: hip.conv_wgrad_raw(x, dy, B, L, Cin, ks, 1, pad, N, with_bias=True), args.iters)
        hip.lib().ssamd_wgrad_set_variant(-1)
        hip.lib().ssamd_wgrad_set_blocks(256)
        tw_256 = timeit(lambda: hip.conv_wgrad_raw(x, dy, B, L, Cin, ks, 1, pad, N, with_bias=True), args.iters)
        hip.lib().ssamd_wgrad_set_blocks(0)
        row = {"op": name, "fwd_ms": round(t, 3), "fwd_TF": round(flops / t / 1e9, 1),
               "fwd_regstage_TF": round(flops / t_lds / 1e9, 1), "fwd_ring256_TF": round(flops / t_ring / 1e9, 1),
               "fwd_big256x256_TF": round(flops / t_big / 1e9, 1),
               "fwd_big_bk64_TF": round(flops / t_b64 / 1e9, 1),
               "fwd_persistent_TF": round(flops / t_pers / 1e9, 1), "wgrad_ms": round(tw, 3),
               "wgrad_TF": round(flops / tw / 1e9, 1), "wgrad_128x128_TF": round(flops / tw_old / 1e9, 1),
               "wgrad_256x128_TF": round(flops / tw_r / 1e9, 1), "wgrad_bk32_TF": round(flops / tw_32 / 1e9, 1),
               "wgrad_256blocks_TF": round(flops / tw_256 / 1e9, 1)}
        if ks > 1:  # packed-sequence geometry (rinfo table), same data
            from speakingstyle_amd.ops.packing import PackInfo

            ri = PackInfo.build(torch.full((B,), L, device=dev), L, R).rinfo
            tpf = timeit(lambda: hip.conv_gemm_raw(x, w, bias, 1, R, Cin, ks, 1, pad, N, 1, rinfo=ri), args.iters)
            tpw = timeit(lambda: hip.conv_wgrad_raw(x, dy, 1, R, Cin, ks, 1, pad, N, with_bias=True, rinfo=ri),
                         args.iters)
            row["fwd_packed_TF"] = round(flops / tpf / 1e9, 1)
            row["wgrad_packed_TF"] = round(flops / tpw / 1e9, 1)
        if ks == 1:
            a2 = x.view(R, Cin)
            w2 = w.view(N, Cin)
            tb = timeit(lambda: torch.matmul(a2, w2.t()), args.iters)
            row["hipblaslt_ms"] = round(tb, 3)
            row["hipblaslt_TF"] = round(flops / tb / 1e9, 1)
        res.append(row)
        print(json.dumps(row), flush=True)
    # attention
    for H, D in ((2, 128), (8, 32)):
        Lq = 800
        qkv = torch.randn(B, Lq, 3 * H * D, device=dev).to(torch.bfloat16)
        lens = torch.randint(Lq // 2, Lq + 1, (B,), device=dev)
        lens[0] = Lq
        fl = 4.0 * B * H * Lq * Lq * D * (lens.float().mean().item() / Lq)
        qh = qkv.clone().requires_grad_(True)
        tf = timeit(lambda: hip.attention(qh, lens, H), args.iters)
        o = hip.attention(qh, lens, H)
        g = torch.randn_like(o)
        tb = timeit(lambda: torch.autograd.grad(o, qh, g, retain_graph=True), args.iters)
        row = {"op": f"attention H{H} D{D} L{Lq}", "fwd_ms": round(tf, 3), "fwd_TF": round(fl / tf / 1e9, 1),
               "bwd_ms": round(tb, 3), "bwd_TF": round(2.5 * fl / tb / 1e9, 1)}
        if D == 128:  # forward variants: register-staged (NF=1) / LDS-DMA NF=1 / NF=2
            for dma, nf in ((0, 1), (1, 1), (1, 2)):
                hip.lib().ssamd_attn_set_fwd(dma, nf)
                row[f"fwd_ms_dma{dma}_nf{nf}"] = round(timeit(lambda: hip.attention(qh, lens, H), args.iters), 3)
            hip.lib().ssamd_attn_set_fwd(1, 2)
        if D == 128:  # dK/dV kernel (register-staged / LDS-DMA) x fragments per wave; dQ NF = 1
            for dma, nkv in ((0, 2), (1, 1), (1, 2)):
                hip.lib().ssamd_attn_set_kv_dma(dma)
                hip.lib().ssamd_attn_set_nf(nkv, 1)
                t2 = timeit(lambda: torch.autograd.grad(o, qh, g, retain_graph=True), args.iters)
                row[f"bwd_ms_kvdma{dma}_nf{nkv}"] = round(t2, 3)
            hip.lib().ssamd_attn_set_kv_dma(1)
            hip.lib().ssamd_attn_set_nf(1, 2)
            for qd, nq in ((0, 1), (1, 1), (1, 2)):  # dQ kernel variants
                hip.lib().ssamd_attn_set_q_dma(qd, nq)
                t2 = timeit(lambda: torch.autograd.grad(o, qh, g, retain_graph=True), args.iters)
                row[f"bwd_ms_qdma{qd}_nf{nq}"] = round(t2, 3)
            hip.lib().ssamd_attn_set_q_dma(1, 2)
        if D == 32:  # query / key fragments per wave of the D = 32 kernels
            for nf in (1, 2, 4):
                hip.lib().ssamd_attn_set_nf32(nf, nf)
                row[f"fwd_ms_nf{nf}"] = round(timeit(lambda: hip.attention(qh, lens, H), args.iters), 3)
                o2 = hip.attention(qh, lens, H)
                row[f"bwd_ms_nf{nf}"] = round(timeit(lambda: torch.autograd.grad(o2, qh, g, retain_graph=True),
                                                     args.iters), 3)
            hip.lib().ssamd_attn_set_nf32(2, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
