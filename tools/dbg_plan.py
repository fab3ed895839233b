"""Debug: fused-Adam plan rebuilds and weight_prep refreshes per training step (GPU box)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.config import load_named  # noqa: E402
from speakingstyle_amd.data.synthetic import SyntheticBatches  # noqa: E402
from speakingstyle_amd.models.fastspeech2 import FastSpeech2  # noqa: E402
from speakingstyle_amd.ops import hip  # noqa: E402
from speakingstyle_amd.train.trainer import Trainer  # noqa: E402

pp, mc, tc = load_named("LJSpeech")
torch.manual_seed(0)
model = FastSpeech2(pp, mc).to("cuda").set_compute_dtype(torch.bfloat16)
tr = Trainer(model, (pp, mc, tc), seed=1)
gen = SyntheticBatches(200, device="cuda", max_seq_len=mc["max_seq_len"], seed=5)
b = gen.make_batch()
refresh = [0]
orig = hip._refresh_all


def cnt(dev):
    refresh[0] += 1
    return orig(dev)


hip._refresh_all = cnt
for i in range(6):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train_step(b)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"step {i}: host {1e3 * (t1 - t0):.2f} ms, total {1e3 * (t2 - t0):.2f} ms, plan builds "
          f"{hip._adam_plan_builds[0]}, refreshes {refresh[0]}, epoch {hip._wepoch}, cache {len(hip._wcache)}")
