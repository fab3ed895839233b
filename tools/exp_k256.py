"""Short-K (K = 256) GEMM shapes of the LJSpeech step on each main-loop variant: the 256x256 big64 kernel
(1 workgroup per CU), the 128x128 LDS-DMA kernel (2 workgroups per CU: one's epilogue overlaps the other's
main loop), the 256x128 ring.  Interleaved rounds, random operands, one JSON line per shape.
Usage (GPU box): python tools/exp_k256.py [rows]"""
import json
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from speakingstyle_amd.ops import hip  # noqa: E402


def timeit(fn, reps=20):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) * 1000.0 / reps


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 113000
    dev = "cuda"
    lib = hip.lib()
    for name, K, N, resid in (("fc 256->256", 256, 256, False), ("fc+resid 256->256", 256, 256, True),
                              ("qkv 256->768", 256, 768, False), ("w2 dgrad 256->1024", 256, 1024, False),
                              ("k1 1024->256", 1024, 256, False)):
        x = torch.randn(1, M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        r = torch.randn(1, M, N, device=dev).to(torch.bfloat16) if resid else None

        def run():
            return hip.conv_gemm_raw(x, w, b, 1, M, K, 1, 1, 0, N, 0, resid=r)

        t = {}
        outs = {}
        for v in (4, 1, 2):
            lib.ssamd_gemm_set_variant(v)
            outs[v] = run()
            t[v] = []
        for _ in range(5):
            for v in (4, 1, 2):
                lib.ssamd_gemm_set_variant(v)
                run()
                t[v].append(timeit(run))
        lib.ssamd_gemm_set_variant(-1)
        byts = 2.0 * M * (K + N * (2 if resid else 1))
        rec = {"shape": name, "M": M}
        for v, tag in ((4, "big64"), (1, "glds128"), (2, "ring256x128")):
            med = statistics.median(t[v])
            rec[tag + "_us"] = round(med, 1)
            rec[tag + "_TBps"] = round(byts / med / 1e6, 2)
            rec[tag + "_maxdiff"] = float((outs[v].float() - outs[4].float()).abs().max())
        print(json.dumps(rec), flush=True)
    # the ReLU-mask data gradient (w2 dgrad, N = 1024): generic epilogue vs EPI_MASK (prefetched mask bytes)
    K, N = 256, 1024
    x = torch.randn(1, M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    mask = torch.randint(0, 256, (M, N // 8), device=dev, dtype=torch.uint8)

    def runm():
        return hip.conv_gemm_mask_raw(x, w, None, 1, M, K, 1, 0, N, 0, mask_in=mask)

    t = {0: [], 1: []}
    outs = {}
    for v in (0, 1):
        lib.ssamd_gemm_set_mask_pre(v)
        outs[v] = runm()
    for _ in range(5):
        for v in (0, 1):
            lib.ssamd_gemm_set_mask_pre(v)
            runm()
            t[v].append(timeit(runm))
    lib.ssamd_gemm_set_mask_pre(1)
    print(json.dumps({"shape": "w2 dgrad + ReLU mask 256->1024", "M": M, "generic_us": round(statistics.median(t[0]), 1),
                      "mask_pre_us": round(statistics.median(t[1]), 1), "bitwise_equal": bool(torch.equal(outs[0], outs[1]))}),
          flush=True)


if __name__ == "__main__":
    main()
