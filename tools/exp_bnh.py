"""PostNet BatchNorm backward costs at the LJSpeech shape (R = 200 x 680 padded rows, C = 512, k5): the
plain data-gradient GEMM vs the GEMM with the BatchNorm-backward head (EPI_BNH: dz + column partials in
the epilogue), the dz apply pass, and the unfused reduce + apply pair (ssamd_bn_bwd) for reference.
Usage (GPU box): python tools/exp_bnh.py [pmc]   (pmc: 3 launches per arm, no timing -- for rocprofv3 --pmc)
(The per-block s_memrealtime stamp build behind profiles/r4_exp_bnh_stamps.jsonl was a diagnostic build, removed.)"""
import json
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from speakingstyle_amd.ops import hip  # noqa: E402
from speakingstyle_amd.ops.hip import _ptr, _stream  # noqa: E402


def timeit(fn, reps=10):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) * 1000.0 / reps


def main():
    dev = "cuda"
    R, C, ks = 200 * 680, 512, 5
    lib = hip.lib()
    dout = torch.randn(1, R, C, device=dev).to(torch.bfloat16)
    wimg = (torch.randn(C, ks * C, device=dev) / (ks * C) ** 0.5).to(torch.bfloat16)
    h = (torch.randn(1, R, C, device=dev) * 2).to(torch.bfloat16)
    stats = torch.stack([torch.zeros(C), torch.ones(C), torch.ones(C) * 0.5, torch.zeros(C)]).to(dev).contiguous()
    nparts = (R + 255) // 256
    part = torch.empty(2 * nparts * C, device=dev)
    dz = torch.empty_like(h)
    dh = torch.empty_like(h)
    gamma = torch.ones(C, device=dev)
    dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
    ws = hip._bn_ws(h.device, R, C)

    def plain():
        return hip.conv_gemm_raw(dout, wimg, None, 1, R, C, ks, 1, 2, C)

    def plain_nostg():
        lib.ssamd_gemm_set_stg(0)
        plain()
        lib.ssamd_gemm_set_stg(1)

    def bnh(p, act=1):
        return lambda: lib.ssamd_conv_gemm_bnbwd(_ptr(dout), _ptr(wimg), _ptr(dz), 1, R, C, ks, 1, 2, C, _ptr(h),
                                                 _ptr(stats), _ptr(part), act, p, 1234, _stream())

    def apply_dz():
        return lib.ssamd_bn_bwd_dz(_ptr(dz), _ptr(h), _ptr(gamma), _ptr(stats), _ptr(part), nparts, _ptr(dh),
                                   _ptr(dg), _ptr(db), R, C, 1, _stream())

    def unfused():
        return lib.ssamd_bn_bwd(_ptr(dout), 0, _ptr(h), _ptr(gamma), _ptr(stats[2]), _ptr(stats[3]), _ptr(stats[0]),
                                _ptr(stats[1]), _ptr(dh), _ptr(dg), _ptr(db), R, C, 1, 1, 0.5, 1234, _ptr(ws),
                                _stream())

    arms = {"gemm_plain": plain, "gemm_plain_nostg": plain_nostg, "gemm_bnh_p0.5": bnh(0.5), "gemm_bnh_p0": bnh(0.0), "gemm_bnh_p0_noact": bnh(0.0, 0), "apply_dz": apply_dz,
            "bn_bwd_unfused(reduce+apply)": unfused}
    if len(sys.argv) > 1 and sys.argv[1] == "pmc":
        for f in arms.values():
            for _ in range(3):
                f()
            torch.cuda.synchronize()
        return
    t = {k: [] for k in arms}
    for f in arms.values():
        f()
    torch.cuda.synchronize()
    for _ in range(5):
        for k, f in arms.items():
            t[k].append(timeit(f))
    # apply-dz geometry sweep: (rows per thread, grid cap)
    cfgs = [(8, 8192), (4, 8192), (16, 8192), (8, 2048), (8, 1024), (4, 2048), (16, 1024)]
    td = {c: [] for c in cfgs}
    for _ in range(5):
        for c in cfgs:
            lib.ssamd_bn_set_dz_cfg(*c)
            td[c].append(timeit(apply_dz))
    lib.ssamd_bn_set_dz_cfg(8, 8192)
    rec = {k: round(statistics.median(v), 1) for k, v in t.items()}
    for c, v in td.items():
        rec[f"apply_dz_u{c[0]}_g{c[1]}_TBps"] = round(3 * R * C * 2 / statistics.median(v) / 1e6, 2)
    rec["apply_dz_TBps"] = round(3 * R * C * 2 / rec["apply_dz"] / 1e6, 2)
    rec["unfused_TBps"] = round(5 * R * C * 2 / rec["bn_bwd_unfused(reduce+apply)"] / 1e6, 2)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
