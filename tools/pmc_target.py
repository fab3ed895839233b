"""Tiny driver for rocprofv3 --pmc runs: a few launches of the headline kernels."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.ops import hip  # noqa: E402

B, L = 200, 800
dev = "cuda"
for Cin, N, ks in ((256, 1024, 9), (256, 256, 1)):
    x = torch.randn(B, L, Cin, device=dev).to(torch.bfloat16)
    w = torch.randn(N, ks, Cin, device=dev).to(torch.bfloat16)
    dy = torch.randn(B, L, N, device=dev).to(torch.bfloat16)
    for _ in range(3):
        hip.conv_gemm_raw(x, w, None, B, L, Cin, ks, 1, (ks - 1) // 2, N, 1)
        hip.conv_wgrad_raw(x, dy, B, L, Cin, ks, 1, (ks - 1) // 2, N, with_bias=True)
        hip.lib().ssamd_wgrad_set_variant(0)  # 128x128 kernels for comparison
        hip.conv_wgrad_raw(x, dy, B, L, Cin, ks, 1, (ks - 1) // 2, N, with_bias=True)
        hip.lib().ssamd_wgrad_set_variant(-1)
qkv = torch.randn(B, L, 768, device=dev).to(torch.bfloat16).requires_grad_(True)
lens = torch.full((B,), L, device=dev)
o = hip.attention(qkv, lens, 2)
for _ in range(3):
    torch.autograd.grad(o, qkv, torch.randn_like(o), retain_graph=True)
torch.cuda.synchronize()
print("done")
