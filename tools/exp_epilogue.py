"""Timing experiment: GEMM with vs without epilogue stores (big64 / persistent)."""
import os, sys, json, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from speakingstyle_amd.ops import hip
from bench_kernels import timeit  # noqa
lib = hip.lib()
lib.ssamd_gemm_debug_nostore.argtypes = [ctypes.c_int]
B, L = 200, 800
for Cin, N, ks in ((256, 768, 1), (256, 256, 1), (1024, 256, 1), (256, 1024, 9)):
    x = torch.randn(B, L, Cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, ks, Cin, device="cuda").to(torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    fl = 2.0 * B * L * N * ks * Cin
    row = {"shape": f"{Cin}->{N} k{ks}"}
    for v in (4, 5):
        lib.ssamd_gemm_set_variant(v)
        for ns in (0, 1):
            lib.ssamd_gemm_debug_nostore(ns)
            t = timeit(lambda: hip.conv_gemm_raw(x, w, bias, B, L, Cin, ks, 1, (ks - 1) // 2, N, 1), 20)
            row[f"v{v}{'_nostore' if ns else ''}_TF"] = round(fl / t / 1e9, 1)
    lib.ssamd_gemm_debug_nostore(0)
    lib.ssamd_gemm_set_variant(-1)
    print(json.dumps(row), flush=True)
