"""rocprofv3 --pmc driver: the fused HiFi-GAN ResBlock layer kernel at synthesis-like sizes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.ops import hip  # noqa: E402

dev = "cuda"
for C, K, d, T in ((64, 11, 5, 72704), (32, 11, 5, 145408)):
    B = 16
    c1 = torch.nn.Conv1d(C, C, K, dilation=d, padding=d * (K - 1) // 2).to(dev)
    c2 = torch.nn.Conv1d(C, C, K, padding=(K - 1) // 2).to(dev)
    x = torch.randn(B, T, C, device=dev).to(torch.bfloat16)
    with torch.no_grad():
        for _ in range(3):
            hip.resblock_layer(x, c1, c2, d, 0.1)
torch.cuda.synchronize()
print("done")
