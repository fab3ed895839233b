"""Isolated timing of the square 3-tap upsampler conv (csrc/k_vocoder.hip conv3_sq_kernel) against the generic
implicit-GEMM path (hip.conv1d_infer, what the upsamplers ran on before) at HiFi-GAN V1 ups 3 / ups 4 shapes
(C = 128 at 64x the mel rate, C = 64 at 128x; 32 utterances of 530 mel frames).  GPU box."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.ops import hip  # noqa: E402


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best * 1000


for C, T in ((128, 530 * 64), (64, 530 * 128)):
    B = 32
    torch.manual_seed(0)
    w = (torch.randn(C, C, 3, device="cuda") / math.sqrt(3 * C)).to(torch.bfloat16).float()
    b = torch.randn(C, device="cuda") * 0.1
    x = torch.randn(B, T, C, device="cuda").to(torch.bfloat16)
    wimg = w.permute(0, 2, 1).to(torch.bfloat16).contiguous()
    with torch.no_grad():
        us_sq = timeit(lambda: hip.conv3_sq(x, wimg, b))
        us_gemm = timeit(lambda: hip.conv1d_infer(x, w, b, 1, 1, None, wimg=wimg))
    rows = B * T
    gb = 2 * rows * C * 2 / 1e9
    tf = 2 * rows * C * 3 * C / 1e12
    print(json.dumps({"C": C, "rows": rows, "us_conv3_sq": round(us_sq, 1), "us_gemm": round(us_gemm, 1),
                      "conv3_sq_TBps": round(gb / us_sq * 1e3, 2), "conv3_sq_TFps": round(tf / us_sq * 1e6, 1),
                      "gemm_TBps": round(gb / us_gemm * 1e3, 2)}), flush=True)
