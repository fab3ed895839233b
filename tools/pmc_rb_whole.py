"""rocprofv3 --pmc driver: the whole-ResBlock kernel (every instance) and the layer kernels of the
remaining geometries, one MRF branch each at synthesis-like sizes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.models import hifigan as H  # noqa: E402

dev = "cuda"
B, TM = 16, 680
for C, K, up in ((32, 3, 256), (32, 7, 256), (32, 11, 256), (64, 3, 128), (64, 7, 128), (64, 11, 128),
                 (128, 3, 64), (128, 7, 64), (128, 11, 64)):
    blk = H.ResBlock1(C, K, (1, 3, 5)).to(dev)
    for m in blk.modules():
        if isinstance(m, torch.nn.Conv1d) and hasattr(m, "weight_g"):
            torch.nn.utils.remove_weight_norm(m)
    x = torch.randn(B, TM * up, C, device=dev).to(torch.bfloat16)
    acc = torch.randn_like(x)
    with torch.no_grad():
        for _ in range(2):
            blk.forward_cl(x, acc=acc)
torch.cuda.synchronize()
print("done")
