#!/usr/bin/env python
"""A/B of the 256x256 weight-gradient main loops (ssamd_wgrad_set_pp: 0 double buffer, 1 ping-pong; 2 was
the staggered 8-phase loop of the measurement in profiles/r5_exp_wgrad_staggered.txt -- rejected, so in the
current library 2 selects the ping-pong loop again) on the training step's weight-gradient shapes: dW must be
bitwise equal across loops (same per-accumulator row order), db within fp32 rounding of an fp32 column sum;
then time each (kernel + reduce (+ colsum), warm, alternating).  JSON per shape.
Usage (GPU): python tools/exp_wgrad_stg.py [--iters 20]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from speakingstyle_amd import ops  # noqa: E402
from speakingstyle_amd.ops import hip  # noqa: E402
from exp_wgrad_pp import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--loops", type=int, nargs="*", default=[0, 1, 2])
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    B = 200
    lens = torch.clamp(torch.normal(565.0, 150.0, (B,)), 100, 1000).to(torch.int64).to(dev)
    M, R = int(lens.max()), int(lens.sum())
    pk = ops.PackInfo.build(lens, M, R)
    shapes = [  # name, Cin, N, ks, packed, rows
        ("dec ffn.w1 k9 256->1024 packed", 256, 1024, 9, True, R),
        ("dec ffn.w2 k1 1024->256", 1024, 256, 1, False, R),
        ("dec qkv 256->768", 256, 768, 1, False, R),
        ("postnet k5 512->512", 512, 512, 5, False, 140000),
        ("postnet k5 80->512", 80, 512, 5, False, 140000),
        ("enc ffn.w1 k9 256->1024", 256, 1024, 9, False, 14000),
    ]
    for name, Cin, N, ks, packed, rows in shapes:
        if packed:
            Bq, L, rinfo, cu = 1, rows, pk.rinfo, pk.cu
        else:
            Bq, L, rinfo, cu = 200, rows // 200, None, None
        x = torch.randn(Bq, L, Cin, device=dev).to(torch.bfloat16)
        dy = torch.randn(Bq, L, N, device=dev).to(torch.bfloat16)
        pad = (ks - 1) // 2
        flops = 2.0 * Bq * L * N * ks * Cin

        def run():
            return hip.conv_wgrad_raw(x, dy, Bq, L, Cin, ks, 1, pad, N, with_bias=True, rinfo=rinfo, cu=cu)

        ref_db = dy.float().reshape(-1, N).sum(0)
        res = {"shape": name, "rows": Bq * L}
        outs = {}
        for v in a.loops:
            hip.lib().ssamd_wgrad_set_pp(v)
            w, b = run()
            outs[v] = w.clone()
            res[f"db_rel_{v}"] = float((b - ref_db).norm() / ref_db.norm())
        base = a.loops[0]
        res["dW_bitwise"] = {v: bool(torch.equal(outs[base], outs[v])) for v in a.loops}
        for rep in range(2):
            for v in a.loops:
                hip.lib().ssamd_wgrad_set_pp(v)
                res.setdefault(f"pp{v}_us", []).append(round(timeit(run, a.iters), 1))
        for v in a.loops:  # kernel + reduce only (no bias: no fused sums, no colsum)
            hip.lib().ssamd_wgrad_set_pp(v)
            res[f"pp{v}_nobias_us"] = round(timeit(lambda: hip.conv_wgrad_raw(x, dy, Bq, L, Cin, ks, 1, pad, N,
                                                                           rinfo=rinfo, cu=cu), a.iters), 1)
        res["colsum_us"] = round(timeit(lambda: hip.colsum_raw(dy.reshape(-1, N), N), a.iters), 1)
        hip.lib().ssamd_wgrad_set_pp(-1)
        for v in a.loops:
            res[f"pp{v}_TF"] = round(flops / min(res[f"pp{v}_us"]) / 1e6, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
