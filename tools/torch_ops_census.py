"""Which torch ops (not HIP kernels) a steady-state training step still issues, with their Python call
sites: torch.profiler over 2 Trainer steps, grouped by op and 6-frame stack (GPU box).
Usage: python tools/torch_ops_census.py [config]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from speakingstyle_amd.config import load_named  # noqa: E402
from speakingstyle_amd.data.synthetic import SyntheticBatches  # noqa: E402
from speakingstyle_amd.models.fastspeech2 import FastSpeech2  # noqa: E402
from speakingstyle_amd.train.trainer import Trainer  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "LJSpeech"
pp, mc, tc = load_named(cfg)
torch.manual_seed(0)
model = FastSpeech2(pp, mc).to("cuda").set_compute_dtype(torch.bfloat16)
tr = Trainer(model, (pp, mc, tc), seed=1)
tr.use_priority_stream(True)
gen = SyntheticBatches(int(tc["optimizer"]["batch_size"]), device="cuda", max_seq_len=mc["max_seq_len"], seed=5)
pool = [gen.make_batch() for _ in range(3)]
for b in pool:
    tr.train_step(b)
torch.cuda.synchronize()
WATCH = ("aten::copy_", "aten::clone", "aten::contiguous", "aten::cat", "aten::zeros", "aten::fill_", "aten::add",
         "aten::add_", "aten::mul", "aten::sum", "aten::to", "aten::_to_copy", "aten::zero_", "aten::index",
         "aten::stack", "aten::sub", "aten::div", "aten::where", "aten::ne", "aten::lt", "aten::arange")
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    for b in pool[:2]:
        tr.train_step(b)
    torch.cuda.synchronize()
rows = prof.key_averages(group_by_stack_n=6)
out = []
for r in rows:
    if r.key in WATCH:
        out.append((r.count, r.key, r.cpu_time_total, r.stack))
out.sort(key=lambda x: -x[0])
for cnt, key, cpu, st in out[:40]:
    print(f"{cnt:4d}  {key:18s} cpu {cpu / 1000 / 2:7.3f} ms/step")
    for fr in st[:6]:
        if "site-packages/torch" in fr:
            continue
        print("        " + fr)
