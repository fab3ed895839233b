"""Host-synchronising torch calls inside steady-state training steps (GPU box): runs Trainer steps
over a pool of differently shaped batches with torch.cuda.set_sync_debug_mode('warn') and prints
each distinct warning site."""
import os
import sys
import traceback
import warnings

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.config import load_named  # noqa: E402
from speakingstyle_amd.data.synthetic import SyntheticBatches  # noqa: E402
from speakingstyle_amd.models.fastspeech2 import FastSpeech2  # noqa: E402
from speakingstyle_amd.train.trainer import Trainer  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "LJSpeech"
pp, mc, tc = load_named(cfg)
torch.manual_seed(0)
model = FastSpeech2(pp, mc).to("cuda").set_compute_dtype(torch.bfloat16)
tr = Trainer(model, (pp, mc, tc), seed=1)
gen = SyntheticBatches(int(tc["optimizer"]["batch_size"]), device="cuda", max_seq_len=mc["max_seq_len"], seed=5)
pool = [gen.make_batch() for _ in range(4)]
for b in pool:
    tr.train_step(b)
torch.cuda.synchronize()
seen = {}


def hook(message, category, filename, lineno, file=None, line=None):
    st = "".join(traceback.format_stack(limit=12)[:-1])
    key = st[-600:]
    seen.setdefault(key, [str(message)[:120], 0])[1] += 1


warnings.showwarning = hook
warnings.simplefilter("always")
torch.cuda.set_sync_debug_mode("warn")
for b in pool:
    tr.train_step(b)
torch.cuda.set_sync_debug_mode(0)
torch.cuda.synchronize()
print("distinct sync sites:", len(seen))
for k, (msg, n) in seen.items():
    print("=" * 60, n, msg)
    print(k)
