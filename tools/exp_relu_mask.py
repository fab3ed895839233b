import sys, json
sys.path.insert(0, "/root/repo")
import torch
from speakingstyle_amd.ops import hip
from tools.gemm_census import timeit, timeit_cold
dev = "cuda"
B, L, C, H = 1, 64607, 256, 1024
dz = torch.randn(B, L, C, device=dev).to(torch.bfloat16)
w2 = (torch.randn(H, 1, C, device=dev) / C ** 0.5).to(torch.bfloat16)
h = torch.relu(torch.randn(B, L, H, device=dev)).to(torch.bfloat16)
mask = torch.randint(0, 255, (L, H // 8), device=dev, dtype=torch.uint8)
for name, fn in (("aux", lambda: hip.conv_gemm_raw(dz, w2, None, B, L, C, 1, 1, 0, H, 0, aux=h)),
                 ("mask", lambda: hip.conv_gemm_mask_raw(dz, w2, None, B, L, C, 1, 0, H, 0, mask_in=mask)),
                 ("plain", lambda: hip.conv_gemm_raw(dz, w2, None, B, L, C, 1, 1, 0, H, 0)),
                 ("aux", lambda: hip.conv_gemm_raw(dz, w2, None, B, L, C, 1, 1, 0, H, 0, aux=h)),
                 ("mask", lambda: hip.conv_gemm_mask_raw(dz, w2, None, B, L, C, 1, 0, H, 0, mask_in=mask))):
    print(json.dumps({"kind": name, "us": round(timeit(fn, 20), 1), "cold_us": round(timeit_cold(fn, 10), 1)}), flush=True)
