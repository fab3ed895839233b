"""Phase timing of the fused HiFi-GAN ResBlock layer kernel (csrc/k_vocoder.hip resblock_layer_kernel, the
diagnostic PROF instantiation): per workgroup s_memtime stamps at the phase boundaries -- x staged (global ->
lrelu -> LDS), conv1, t1 epilogue, conv2, output-tile staging, epilogue (residual / acc loads, stores).
Prints median cycles per phase and the share of a tile's time, for one tile per workgroup and for the
persistent grid of the production launch (GPU box).
Usage: python tools/exp_rb_phases.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.ops import hip  # noqa: E402

PH = ["x_stage", "conv1", "t1_epi", "conv2", "out_stage", "epilogue"]
for C, K, d, acc in ((128, 11, 1, False), (128, 11, 5, True), (128, 7, 3, False), (64, 11, 3, False)):
    B, T = (16, 32768) if C == 128 else (16, 65536)
    torch.manual_seed(0)
    c1 = torch.nn.Conv1d(C, C, K).cuda()
    c2 = torch.nn.Conv1d(C, C, K).cuda()
    x = (torch.randn(B, T, C, device="cuda") * 0.5).to(torch.bfloat16)
    a = (torch.randn(B, T, C, device="cuda") * 0.5).to(torch.bfloat16) if acc else None
    out = torch.empty_like(x)
    w1, w2 = hip.weight_fwd(c1.weight), hip.weight_fwd(c2.weight)
    b1, b2 = c1.bias.detach().float().contiguous(), c2.bias.detach().float().contiguous()
    BM = hip.lib().ssamd_resblock_layer_tile(C, K)
    tiles = (T + BM - 1) // BM
    prof = torch.zeros(B * (T // 16 + 1) * 8, dtype=torch.int64, device="cuda")  # any tile height

    def run(p):
        # p = 0: production launch; 1: stamped, one tile per workgroup; 2: stamped, the production launch's
        # persistent grid (resident workgroups)
        f = hip.lib().ssamd_resblock_layer_prof if p else hip.lib().ssamd_resblock_layer
        args = [hip._ptr(x), hip._ptr(w1), hip._ptr(b1), hip._ptr(w2), hip._ptr(b2), hip._ptr(a),
                hip._ptr(out if a is None else a), B, T, C, K, d, 0.1, 1.0, 0]
        if p:
            args += [hip._ptr(prof), prof.numel(), 0 if p == 1 else (256 if C == 128 else 512)]
        hip._check(f(*args, hip._stream()), "resblock")

    ms = {}
    for p in (0, 1, 2):
        for _ in range(3):
            run(p)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            run(p)
        e1.record()
        torch.cuda.synchronize()
        ms[p] = e0.elapsed_time(e1) / 5
        if p == 0:
            continue
        st = prof.view(-1, 8).cpu().double()
        d_ = st[:, 1:7] - st[:, 0:6]
        tot = (st[:, 6] - st[:, 0])
        med = d_.median(0).values
        rec = {"C": C, "K": K, "d": d, "acc": acc, "grid": "one_tile_per_block" if p == 1 else "persistent",
               "rows": B * T, "tiles": B * tiles, "us_plain": round(ms[0] * 1000, 1),
               "us_prof": round(ms[p] * 1000, 1), "tile_cycles_med": int(tot.median()),
               "phase_cycles_med": {k: int(v) for k, v in zip(PH, med.tolist())},
               "phase_share": {k: round(float(v) / float(med.sum()), 3) for k, v in zip(PH, med.tolist())}}
        print(json.dumps(rec), flush=True)
