"""Isolated timing of the upsamplers' 3-tap GEMM (hifigan convT_as_conv3) with and without the per-tile zero-tap
skip (ConvGeom::ksplit, csrc/k_gemm.hip) at HiFi-GAN V1 ups 1 / ups 2 shapes, 32 utterances x 530 mel frames."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.models.hifigan import convT_as_conv3  # noqa: E402
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


for Cin, Cout, s, T, dual in ((512, 256, 8, 530, True), (256, 128, 8, 530 * 8, False)):
    B = 32
    w = (torch.randn(Cin, Cout, 2 * s, device="cuda") / math.sqrt(Cin * 2)).float()
    b = torch.randn(Cout, device="cuda") * 0.1
    x = torch.randn(B, T, Cin, device="cuda").to(torch.bfloat16)
    wu = convT_as_conv3(w, s, s // 2)
    wimg = wu.permute(0, 2, 1).to(torch.bfloat16).contiguous()
    bt = b.repeat(s).contiguous()
    with torch.no_grad():
        us = {k: timeit(lambda: hip.conv1d_infer(x, wu, bt, 1, 1, None, wimg=wimg, dual_lrelu=dual,
                                                 ksplit=k * (s // 2) * Cout)) for k in (0, 1)}
    tf = 2 * B * T * s * Cout * 3 * Cin / 1e12
    print(json.dumps({"Cin": Cin, "N": s * Cout, "rows": B * T, "dual_lrelu": dual, "us_full": round(us[0], 1),
                      "us_skip": round(us[1], 1), "TFps_3tap_equiv_full": round(tf / us[0] * 1e6, 1),
                      "TFps_3tap_equiv_skip": round(tf / us[1] * 1e6, 1)}), flush=True)
