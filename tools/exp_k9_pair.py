#!/usr/bin/env python
"""The decoder's k9 FFN conv (256 -> 1024, packed rows) as forward and as weight gradient, the same FLOPs each,
five launches of each: a target for PMC passes comparing the two main loops (tools/gpu.sh pmcpy:...)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd import ops  # noqa: E402
from speakingstyle_amd.ops import hip  # noqa: E402

torch.manual_seed(0)
B = 200
lens = torch.clamp(torch.normal(565.0, 150.0, (B,)), 100, 1000).to(torch.int64).cuda()
M, R = int(lens.max()), int(lens.sum())
pk = ops.PackInfo.build(lens, M, R)
Cin, N, ks = 256, 1024, 9
x = torch.randn(1, R, Cin, device="cuda").to(torch.bfloat16)
dy = torch.randn(1, R, N, device="cuda").to(torch.bfloat16)
w = (torch.randn(N, ks, Cin, device="cuda") / 48).to(torch.bfloat16)
for _ in range(5):
    hip.conv_gemm_raw(x, w, None, 1, R, Cin, ks, 1, 4, N, 0, rinfo=pk.rinfo)
    hip.conv_wgrad_raw(x, dy, 1, R, Cin, ks, 1, 4, N, with_bias=False, rinfo=pk.rinfo, cu=pk.cu)
torch.cuda.synchronize()
print("ok")
