"""PostNet BatchNorm + tanh + dropout fused op at the LJSpeech bench size ([200 x 750, 512] bf16):
forward and backward kernel times (rocprof-free: HIP events around each phase, 10 repetitions)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.ops import hip  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
R, C = 200 * 750, 512
bn = torch.nn.BatchNorm1d(C).to(dev)
h = torch.randn(1, R, C, device=dev).to(torch.bfloat16).requires_grad_(True)
g = torch.randn(1, R, C, device=dev).to(torch.bfloat16)
res = {}
for name in ("fwd", "bwd"):
    ts = []
    for it in range(12):
        x = h.detach().requires_grad_(True)
        if name == "fwd":
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            y = hip.bn_act(x, bn, True, True, 0.5)
            e1.record()
        else:
            y = hip.bn_act(x, bn, True, True, 0.5)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            y.backward(g)
            e1.record()
        torch.cuda.synchronize()
        if it >= 2:
            ts.append(e0.elapsed_time(e1) * 1000)
    res[name + "_us"] = round(sorted(ts)[len(ts) // 2], 1)
res["bytes_bwd_MB"] = round(2 * 3 * R * C * 2 / 1e6, 1)  # reduce (h, dy) + apply (h, dy, dh)
print(json.dumps(res))
