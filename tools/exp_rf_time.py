"""Isolated timing of the whole-ResBlock kernel (csrc/k_vocoder.hip resblock_fused_kernel) at synthesis-sized inputs,
with the MRF accumulator (the in-place acc_in epilogue).  Same-box A/B: run once per kernel library
(SSAMD_KERNEL_LIB=<base .so> for A).  Usage: python tools/exp_rf_time.py [C K ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.models import hifigan as H  # noqa: E402
from speakingstyle_amd.ops import hip  # noqa: E402

args = [int(a) for a in sys.argv[1:]] or [64, 7]
for C, K in zip(args[::2], args[1::2]):
    torch.manual_seed(0)
    B, T = 16, (65536 if C == 64 else 131072 if C == 32 else 32768)
    blk = H.ResBlock1(C, K, (1, 3, 5)).cuda()
    for m in blk.modules():  # weight norm folded: its .weight attribute would stay a host tensor under .cuda()
        if isinstance(m, torch.nn.Conv1d) and hasattr(m, "weight_g"):
            torch.nn.utils.remove_weight_norm(m)
    x = (torch.randn(B, T, C, device="cuda") * 0.5).to(torch.bfloat16)
    acc = (torch.randn(B, T, C, device="cuda") * 0.5).to(torch.bfloat16)
    with torch.no_grad():
        run = lambda: hip.resblock_fused(x, blk.convs1, blk.convs2, blk.dilation, H.LRELU_SLOPE, acc=acc,  # noqa: E731
                                         out_scale=1.0)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        best = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                run()
            e1.record()
            torch.cuda.synchronize()
            best.append(e0.elapsed_time(e1) / 5)
    print(json.dumps({"C": C, "K": K, "rows": B * T, "lib": os.environ.get("SSAMD_KERNEL_LIB", "tree"),
                      "us_min": round(min(best) * 1000, 1), "us_med": round(sorted(best)[2] * 1000, 1)}), flush=True)
