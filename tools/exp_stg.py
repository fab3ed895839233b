"""A/B of the big64 GEMM main loops on the LJSpeech step's shapes: the two-stage double buffer (one
vmcnt(0) + barrier per 64-deep k-tile) vs the staggered 8-phase loop (``ssamd_gemm_set_stg``).
Both accumulate every output in the same order, so the outputs must be bitwise equal.  Interleaved
rounds in one process (random operands), one JSON line per shape with the median / min times.
Usage (GPU box): python tools/exp_stg.py [rounds]"""
import json
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from speakingstyle_amd.ops import hip  # noqa: E402


def timeit(fn, reps=10):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) * 1000.0 / reps


def packed_rinfo(lens, dev):
    t = torch.cat([torch.arange(int(n), dtype=torch.int32) for n in lens])
    ln = torch.cat([torch.full((int(n),), int(n), dtype=torch.int32) for n in lens])
    return torch.stack([t, ln], 1).contiguous().to(dev)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    lens = (torch.randn(200, generator=g) * 150 + 568).clamp(150, 1000).round().int()
    R = int(lens.sum())
    rinfo = packed_rinfo(lens.tolist(), dev)
    shapes = [  # name, rows, Cin, N, ks, packed, act(relu=1)
        ("dec k9 fwd 256->1024", R, 256, 1024, 9, True, 1),
        ("dec k9 dgrad 1024->256", R, 1024, 256, 9, True, 0),
        ("dec k1 w2 1024->256", R, 1024, 256, 1, False, 0),
        ("dec qkv 256->768", R, 256, 768, 1, False, 0),
        ("dec fc 256->256", R, 256, 256, 1, False, 0),
        ("dec w2 dgrad 256->1024", R, 256, 1024, 1, False, 0),
        ("postnet k5 512->512", 200 * 760, 512, 512, 5, False, 0),
    ]
    for name, M, Cin, N, ks, packed, act in shapes:
        x = torch.randn(1, M, Cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, ks * Cin, device=dev) / (ks * Cin) ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        pad = (ks - 1) // 2
        ri = rinfo if packed else None
        if packed:
            assert M == R
        B, L = (1, M)

        def run():
            return hip.conv_gemm_raw(x, w, b, B, L, Cin, ks, 1, pad, N, act, rinfo=ri)

        lib = hip.lib()
        lib.ssamd_gemm_set_stg(0)
        y0 = run()
        lib.ssamd_gemm_set_stg(1)
        y1 = run()
        torch.cuda.synchronize()
        same = bool(torch.equal(y0, y1))
        t = {0: [], 1: []}
        for _ in range(rounds):
            for v in (0, 1):
                lib.ssamd_gemm_set_stg(v)
                run()
                t[v].append(timeit(run))
        lib.ssamd_gemm_set_stg(1)  # restore the default
        fl = 2.0 * M * N * ks * Cin
        rec = {"shape": name, "M": M, "bitwise_equal": same}
        for v, tag in ((0, "dbuf"), (1, "stg")):
            med = statistics.median(t[v])
            rec[tag + "_us_med"] = round(med, 1)
            rec[tag + "_us_min"] = round(min(t[v]), 1)
            rec[tag + "_TF"] = round(fl / med / 1e6, 1)
        rec["speedup"] = round(rec["dbuf_us_med"] / rec["stg_us_med"], 3)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
