"""A/B of the whole-ResBlock kernel vs three per-layer fused kernels at the vocoder bench shapes
(one MRF branch of each narrow stage: C = 32 at 256x, C = 64 at 128x the mel rate)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.models import hifigan as H  # noqa: E402
from speakingstyle_amd.ops import hip  # noqa: E402

dev = "cuda"
B, TM = 64, 680  # utterances x mel frames
res = []
for C, K, up in ((32, 3, 256), (32, 7, 256), (32, 11, 256), (64, 3, 128), (64, 7, 128), (64, 11, 128), (128, 3, 64),
                  (128, 7, 64)):
    blk = H.ResBlock1(C, K, (1, 3, 5)).to(dev)
    for m in blk.modules():
        if isinstance(m, torch.nn.Conv1d) and hasattr(m, "weight_g"):
            torch.nn.utils.remove_weight_norm(m)
    T = TM * up
    x = torch.randn(B, T, C, device=dev).to(torch.bfloat16)
    acc = torch.randn(B, T, C, device=dev).to(torch.bfloat16)
    row = {"C": C, "K": K, "T": T, "B": B}
    for whole in (False, True):
        if whole and not hip.resblock_fusable(C, K):
            continue
        H._WHOLE_BLOCK[0] = whole
        with torch.no_grad():
            for _ in range(2):
                blk.forward_cl(x, acc=acc, out_scale=1.0)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(5):
                blk.forward_cl(x, acc=acc, out_scale=1.0)
            torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / 5 * 1e3
        fl = 6 * 2 * B * T * C * C * K
        row["whole_ms" if whole else "layers_ms"] = round(ms, 3)
        row["whole_TF" if whole else "layers_TF"] = round(fl / ms / 1e9, 1)
    H._WHOLE_BLOCK[0] = True
    print(json.dumps(row), flush=True)
    res.append(row)
