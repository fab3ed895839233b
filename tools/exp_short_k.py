"""Short-K GEMM shapes of the FastSpeech2 decoder (K = Cin = 256, ks = 1) on the big64 kernel:
plain epilogue vs the ReLU-bitmask epilogue vs hipBLASLt (torch.matmul) as a ceiling.
Prints one JSON line per shape."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from speakingstyle_amd.ops import hip  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) * 1000.0 / reps


def main():
    dev = "cuda"
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 113000
    for K, N in ((256, 1024), (256, 768), (256, 256), (1024, 256), (768, 256)):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
        b = torch.zeros(N, device=dev)
        mask = torch.randint(0, 255, (M, N // 8), device=dev, dtype=torch.uint8)
        fl = 2.0 * M * K * N
        rec = {"M": M, "K": K, "N": N}
        rec["plain_us"] = timeit(lambda: hip.conv_gemm_raw(x, w, b, 1, M, K, 1, 1, 0, N))  # hand-written kernel
        rec["mask_in_us"] = timeit(lambda: hip.conv_gemm_mask_raw(x, w, None, 1, M, K, 1, 0, N, 0, mask_in=mask))
        rec["relu_mask_out_us"] = timeit(lambda: hip.conv_gemm_mask_raw(x, w, b, 1, M, K, 1, 0, N, 1, mask_out=mask))
        rec["blaslt_us"] = timeit(lambda: torch.matmul(x, w.t()))
        w32 = w.float().view(N, K, 1).contiguous()
        res = torch.randn(M, N, device=dev).to(torch.bfloat16)
        acc = torch.randn(M, N, device=dev).to(torch.bfloat16)
        rec["resid_acc_us"] = timeit(lambda: hip.conv1d_infer(x.view(1, M, K), w32, b, 0, 1, None,
                                                              resid=res.view(1, M, N), acc=acc.view(1, M, N),
                                                              scale=0.5))
        for k in ("plain", "mask_in", "relu_mask_out", "blaslt", "resid_acc"):
            rec[k + "_TF"] = round(fl / rec[k + "_us"] / 1e6, 1)
            rec[k + "_us"] = round(rec[k + "_us"], 1)
        # bytes: x once, y once (+ mask): the memory floor at 5 TB/s
        rec["floor_us_5TBs"] = round((M * K * 2 + M * N * 2 + M * N / 8) / 5e12 * 1e6, 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
