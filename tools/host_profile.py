"""Host-side (Python) cost of a training step: cProfile over N steady-state Trainer steps (GPU box).
Usage: python tools/host_profile.py [config] [steps] [batch]   (prints the unprofiled host ms/step first)"""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.config import load_named  # noqa: E402
from speakingstyle_amd.data.synthetic import SyntheticBatches  # noqa: E402
from speakingstyle_amd.models.fastspeech2 import FastSpeech2  # noqa: E402
from speakingstyle_amd.train.trainer import Trainer  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "LJSpeech"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
pp, mc, tc = load_named(cfg)
torch.manual_seed(0)
model = FastSpeech2(pp, mc).to("cuda").set_compute_dtype(torch.bfloat16)
tr = Trainer(model, (pp, mc, tc), seed=1)
bs = int(sys.argv[3]) if len(sys.argv) > 3 else int(tc["optimizer"]["batch_size"])
gen = SyntheticBatches(bs, device="cuda", max_seq_len=mc["max_seq_len"], seed=5)
b = gen.make_batch()
for _ in range(3):
    tr.train_step(b)
torch.cuda.synchronize()
import time  # noqa: E402

t0 = time.perf_counter()
for _ in range(20):
    tr.train_step(b)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"{cfg} batch {bs}: host {1e3 * (t1 - t0) / 20:.2f} ms/step, wall {1e3 * (t2 - t0) / 20:.2f} ms/step", flush=True)
if os.environ.get("SAME_THREAD_BWD", "1") == "1":  # backward on this thread so cProfile sees it
    torch.autograd.set_multithreading_enabled(False)
pr = cProfile.Profile()
pr.enable()
for _ in range(n):
    tr.train_step(b)
pr.disable()
torch.cuda.synchronize()
s = io.StringIO()
ps = pstats.Stats(pr, stream=s).sort_stats("tottime")
ps.print_stats(35)
print(s.getvalue())
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
print(s.getvalue())
