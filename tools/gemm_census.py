#!/usr/bin/env python
"""GEMM census of one training step (GPU box): records every implicit-GEMM launch of a real
``Trainer.train_step`` (forward / dgrad through ``conv_gemm_raw``, weight
gradients through ``conv_wgrad_raw``), then replays each distinct shape on random data and times
it under every GEMM variant, so the auto-selection in ``csrc/k_gemm.hip`` can be checked per
shape against the step's real mix.

Usage: python tools/gemm_census.py [--config LJSpeech] [--batch N] [--iters 10]
Prints one JSON line per distinct shape (calls per step, us per call per variant, TF/s) and a
summary line (total GEMM us per step for the auto choice vs the per-shape best variant).
"""
import argparse
import json
import os
import sys
from collections import OrderedDict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from speakingstyle_amd.ops import hip  # noqa: E402

FWD_VARIANTS = (-1, 0, 1, 2, 4, 5)
WGRAD_VARIANTS = (-1, 0, 1, 2)


_FLUSH = None


def timeit_cold(fn, iters):
    """Mean time of fn with the L2 / Infinity Cache flushed before every call (a 1 GiB write),
    events around fn only: what a GEMM costs inside the step, where its operands come from HBM."""
    global _FLUSH
    if _FLUSH is None:
        _FLUSH = torch.empty(256 << 20, device="cuda", dtype=torch.float32)
    fn()
    tot = 0.0
    for _ in range(iters):
        _FLUSH.zero_()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        tot += s.elapsed_time(e)
    return tot / iters * 1000.0


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0  # us


def record_step(args):
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.train.trainer import Trainer

    pp, mc, tc = load_named(args.config)
    batch = args.batch or int(tc["optimizer"]["batch_size"])
    torch.manual_seed(0)
    model = FastSpeech2(pp, mc).to("cuda").set_compute_dtype(torch.bfloat16)
    tr = Trainer(model, (pp, mc, tc), seed=1)
    gen = SyntheticBatches(batch, device="cuda", max_seq_len=mc["max_seq_len"], seed=5,
                           frame_level=pp["preprocessing"]["pitch"]["feature"] == "frame_level")
    b = gen.make_batch()
    tr.train_step(b)  # warm (weight images, allocator)
    calls = OrderedDict()
    orig = (hip.conv_gemm_raw, hip.conv_wgrad_raw)

    def key_add(k):
        calls[k] = calls.get(k, 0) + 1

    def g(x, wimg, bias, B, L, Cin, ks, dil, pad, N, act=0, aux=None, resid=None, lens=None, out_f32=False,
          rinfo=None):
        key_add(("fwd", B, L, Cin, ks, dil, pad, N, int(act), aux is not None, resid is not None, lens is not None,
                 bool(out_f32), rinfo is not None))
        return orig[0](x, wimg, bias, B, L, Cin, ks, dil, pad, N, act, aux, resid, lens, out_f32, rinfo)

    def w(x, dy, B, L, Cin, ks, dil, pad, N, with_bias=False, dW=None, db=None, rinfo=None, cu=None):
        key_add(("wgrad", B, L, Cin, ks, dil, pad, N, int(bool(with_bias)), False, False, False, False,
                 rinfo is not None))
        return orig[1](x, dy, B, L, Cin, ks, dil, pad, N, with_bias, dW, db, rinfo, cu)

    hip.conv_gemm_raw, hip.conv_wgrad_raw = g, w
    try:
        tr.train_step(b)
        torch.cuda.synchronize()
    finally:
        hip.conv_gemm_raw, hip.conv_wgrad_raw = orig
    del tr, model
    torch.cuda.empty_cache()
    return calls


def replay(k, n, iters):
    from speakingstyle_amd.ops.packing import PackInfo

    kind, B, L, Cin, ks, dil, pad, N, act, has_aux, has_res, has_lens, f32, packed = k
    dev = "cuda"
    M = B * L
    x = torch.randn(B, L, Cin, device=dev).to(torch.bfloat16)
    ri = cu = None
    if packed:  # one long packed row block: sequences of ~800 rows
        per = 800
        nseq = max(1, M // per)
        lens = torch.full((nseq,), per, device=dev, dtype=torch.int64)
        lens[-1] += M - nseq * per
        pk = PackInfo.build(lens, int(lens.max()), M)
        ri, cu = pk.rinfo, pk.cu
    flops = 2.0 * M * N * ks * Cin
    rec = {"kind": kind, "M": M, "Cin": Cin, "ks": ks, "N": N, "calls": n, "packed": packed}
    if kind == "wgrad":
        dy = torch.randn(B, L, N, device=dev).to(torch.bfloat16)
        fn = lambda: orig_wgrad(x, dy, B, L, Cin, ks, dil, pad, N, with_bias=bool(act), rinfo=ri, cu=cu)  # noqa: E731
        setv = hip.lib().ssamd_wgrad_set_variant
        variants = WGRAD_VARIANTS
    else:
        wimg = (torch.randn(N, ks, Cin, device=dev) / (ks * Cin) ** 0.5).to(torch.bfloat16)
        bias = torch.zeros(N, device=dev)
        aux = torch.randn(B, L, N, device=dev).to(torch.bfloat16) if has_aux else None
        res = torch.randn(B, L, N, device=dev).to(torch.bfloat16) if has_res else None
        ln = torch.full((B,), L, device=dev, dtype=torch.int64) if has_lens else None
        fn = lambda: hip.conv_gemm_raw(x, wimg, bias, B, L, Cin, ks, dil, pad, N, act, aux, res, ln, f32,  # noqa: E731
                                       ri)
        setv = hip.lib().ssamd_gemm_set_variant
        variants = FWD_VARIANTS
    for v in variants:
        setv(v)
        try:
            t = timeit(fn, iters)
            rec[f"v{v}_us"] = round(t, 1)
        except Exception as e:  # noqa: BLE001 (variant not applicable to this shape)
            rec[f"v{v}_us"] = None
            rec[f"v{v}_err"] = str(e)[:60]
    setv(-1)
    # the first timed variant runs on a cold clock / cache: re-time the auto choice last, keep the min
    t = timeit(fn, iters)
    rec["v-1_us"] = round(min(rec["v-1_us"], t), 1) if rec.get("v-1_us") else round(t, 1)
    ts = {v: rec[f"v{v}_us"] for v in variants if rec.get(f"v{v}_us")}
    best = min(ts, key=ts.get)
    rec["auto_TF"] = round(flops / ts[-1] / 1e6, 1)
    rec["cold_us"] = round(timeit_cold(fn, iters), 1)
    rec["cold_TF"] = round(flops / rec["cold_us"] / 1e6, 1)
    rec["best"] = best
    rec["best_TF"] = round(flops / ts[best] / 1e6, 1)
    return rec


orig_wgrad = hip.conv_wgrad_raw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="LJSpeech")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    calls = record_step(args)
    tot_auto = tot_best = tot_cold = 0.0
    for k, n in calls.items():
        rec = replay(k, n, args.iters)
        tot_auto += n * rec["v-1_us"]
        tot_best += n * rec[f"v{rec['best']}_us"]
        tot_cold += n * rec["cold_us"]
        print(json.dumps(rec), flush=True)
    print(json.dumps({"summary": args.config, "distinct": len(calls), "calls": sum(calls.values()),
                      "gemm_us_auto": round(tot_auto, 1), "gemm_us_best_variant": round(tot_best, 1),
                      "gemm_us_cold": round(tot_cold, 1)}), flush=True)


if __name__ == "__main__":
    main()
