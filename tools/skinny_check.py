"""Debug aid: run one batch-1 GST synthesis forward with every conv_gemm call executed twice (skinny kernel on /
off) and print the geometry of calls whose outputs differ beyond bf16 rounding."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.config import load_named  # noqa: E402
from speakingstyle_amd.data.synthetic import SyntheticBatches  # noqa: E402
from speakingstyle_amd.models.fastspeech2 import FastSpeech2  # noqa: E402
from speakingstyle_amd.ops import hip  # noqa: E402

orig = hip.conv_gemm_raw
bad = []


def twice(x, wimg, bias, B, L, Cin, ks, dil, pad, N, act=0, aux=None, resid=None, lens=None, out_f32=False, rinfo=None):
    hip.lib().ssamd_gemm_set_skinny(0)
    y0 = orig(x, wimg, bias, B, L, Cin, ks, dil, pad, N, act, aux, resid, lens, out_f32, rinfo)
    hip.lib().ssamd_gemm_set_skinny(1)
    y1 = orig(x, wimg, bias, B, L, Cin, ks, dil, pad, N, act, aux, resid, lens, out_f32, rinfo)
    d = ((y1.float() - y0.float()).norm() / (y0.float().norm() + 1e-12)).item()
    tag = dict(B=B, L=L, Cin=Cin, ks=ks, dil=dil, pad=pad, N=N, act=act, aux=aux is not None,
               resid=resid is not None, lens=lens is not None, f32=out_f32, rinfo=rinfo is not None,
               xc=x.is_contiguous(), xal=x.data_ptr() % 16, wal=wimg.data_ptr() % 16, wshape=tuple(wimg.shape))
    print(f"{d:.3e} {tag}", flush=True)
    if d > 1e-2:
        bad.append(tag)
    return y1


hip.conv_gemm_raw = twice
dev = torch.device("cuda", 0)
pp, mc, tc = load_named(sys.argv[1] if len(sys.argv) > 1 else "BC2013_GST")
torch.manual_seed(0)
model = FastSpeech2(pp, mc).to(dev)
with torch.no_grad():
    lin = model.variance_adaptor.duration_predictor.linear_layer
    lin.weight.normal_(0.0, 0.005)
    lin.bias.fill_(math.log(9.1))
model.eval().set_compute_dtype(torch.bfloat16)
model.requires_grad_(False)
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 1
b = SyntheticBatches(nb, device=dev, seed=3, max_seq_len=mc["max_seq_len"]).make_batch()
args = (b[2], b[3], b[4], b[5], b[6], b[7], b[8])
if len(sys.argv) > 3 and sys.argv[3] == "packed":  # infer_packed with the skinny kernel on vs off, per stage
    hip.conv_gemm_raw = orig
    outs = {}
    for sk in (0, 1):
        hip.lib().ssamd_gemm_set_skinny(sk)
        with torch.no_grad():
            front = model.infer_front(*args)
            outs[sk] = [t.float().clone() if isinstance(t, torch.Tensor) and t.is_floating_point() else t
                        for t in front]
            lens = [int(v) for v in front[2].cpu().tolist()]
            outs[sk].append(model.infer_back(front, lens).float().clone())
    for i, (a, c) in enumerate(zip(outs[0], outs[1])):
        if isinstance(a, torch.Tensor) and a.is_floating_point():
            d = ((c - a).norm() / (a.norm() + 1e-12)).item()
            print("front/back output", i, tuple(a.shape), f"{d:.3e}")
        elif isinstance(a, torch.Tensor):
            print("output", i, tuple(a.shape), "equal" if torch.equal(a, c) else "DIFF")
    sys.exit(0)
if len(sys.argv) > 3 and sys.argv[3] == "slice":  # utterance 0 of the batch alone, whole model on vs off
    args = tuple(a[0:1] if isinstance(a, torch.Tensor) else a for a in args)
    hip.conv_gemm_raw = orig
    res = {}
    for sk in (0, 1):
        hip.lib().ssamd_gemm_set_skinny(sk)
        with torch.no_grad():
            res[sk] = model(*args)
    for i, (a, c) in enumerate(zip(res[0], res[1])):
        if isinstance(a, torch.Tensor) and a.is_floating_point():
            print("output", i, tuple(a.shape), f"{((c.float() - a.float()).norm() / (a.float().norm() + 1e-12)).item():.3e}")
    hip.conv_gemm_raw = twice
with torch.no_grad():
    model(*args)
torch.cuda.synchronize()
print("BAD", len(bad))
for t in bad:
    print(t)
