import sys
sys.path.insert(0, "/root/repo")
import torch
from speakingstyle_amd.ops import hip
from speakingstyle_amd.config import load_named
from speakingstyle_amd.data.synthetic import SyntheticBatches
from speakingstyle_amd.models.fastspeech2 import FastSpeech2
from speakingstyle_amd.train.trainer import Trainer
pp, mc, tc = load_named("LJSpeech")
m = FastSpeech2(pp, mc).to("cuda").set_compute_dtype(torch.bfloat16)
tr = Trainer(m, (pp, mc, tc), seed=1)
b = SyntheticBatches(200, device="cuda", max_seq_len=mc["max_seq_len"], seed=5).make_batch()
calls = []
orig = hip.conv_gemm_mask_raw
def f(*a, **k):
    calls.append(("out" if k.get("mask_out") is not None else "in", a[4], a[7], a[8]))
    return orig(*a, **k)
hip.conv_gemm_mask_raw = f
tr.train_step(b)
torch.cuda.synchronize()
print(len(calls), calls[:20])
