#!/usr/bin/env python
"""hipBLASLt (torch.matmul) on plain GEMMs of the training step's implicit-GEMM sizes (GPU box):
the library ceiling our conv kernels are compared against (k9 conv as an im2col GEMM)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tools.gemm_census import timeit, timeit_cold  # noqa: E402


def main():
    dev = "cuda"
    for M, K, N in ((64607, 2304, 1024), (64607, 9216, 256), (106600, 2560, 512), (64607, 256, 768),
                    (64607, 1024, 256), (64607, 256, 1024), (65536, 4096, 4096)):
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        b = torch.randn(K, N, device=dev).to(torch.bfloat16)
        fl = 2.0 * M * N * K
        t = timeit(lambda: torch.matmul(a, b), 10)
        tc = timeit_cold(lambda: torch.matmul(a, b), 10)
        print(json.dumps({"M": M, "K": K, "N": N, "us": round(t, 1), "TF": round(fl / t / 1e6, 1),
                          "cold_us": round(tc, 1), "cold_TF": round(fl / tc / 1e6, 1)}), flush=True)
        del a, b


if __name__ == "__main__":
    main()
