"""Python call sites of the aten ops that launch GPU work in one steady-state training step (GPU box):
a TorchDispatchMode logs every op with a CUDA tensor result (views / empty / metadata ops excluded) with the
innermost repo frames of its stack.  Usage: python tools/aten_sites.py [config] [batch]"""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

from speakingstyle_amd.config import load_named  # noqa: E402
from speakingstyle_amd.data.synthetic import SyntheticBatches  # noqa: E402
from speakingstyle_amd.models.fastspeech2 import FastSpeech2  # noqa: E402
from speakingstyle_amd.train.trainer import Trainer  # noqa: E402

SKIP = ("empty", "view", "as_strided", "_reshape_alias", "detach", "alias", "slice", "select", "unsqueeze",
        "squeeze", "expand", "permute", "transpose", "t.default", "split", "unbind", "_unsafe_view", "set_", "lift",
        "_local_scalar_dense", "is_same_size", "record_stream", "size", "stride", "numel", "dim", "new_empty")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.sites = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func)
        if not any(s in name for s in SKIP):
            outs = out if isinstance(out, (tuple, list)) else [out]
            if any(isinstance(o, torch.Tensor) and o.is_cuda for o in outs):
                fr = [f for f in traceback.extract_stack()[:-1] if f.filename.startswith(REPO) and "aten_sites" not in f.filename]
                site = " <- ".join(f"{os.path.relpath(f.filename, REPO)}:{f.lineno}" for f in fr[-3:][::-1])
                self.sites[(name, site)] += 1
        return out


cfg = sys.argv[1] if len(sys.argv) > 1 else "LJSpeech"
pp, mc, tc = load_named(cfg)
bs = int(sys.argv[2]) if len(sys.argv) > 2 else int(tc["optimizer"]["batch_size"])
torch.manual_seed(0)
model = FastSpeech2(pp, mc).to("cuda").set_compute_dtype(torch.bfloat16)
tr = Trainer(model, (pp, mc, tc), seed=1)
tr.use_priority_stream(True)
gen = SyntheticBatches(bs, device="cuda", max_seq_len=mc["max_seq_len"], seed=5,
                       frame_level=pp["preprocessing"]["pitch"]["feature"] == "frame_level")
pool = [gen.make_batch() for _ in range(3)]
for b in pool:
    tr.train_step(b)
torch.cuda.synchronize()
log = Log()
with log:
    tr.train_step(pool[0])
torch.cuda.synchronize()
for (name, site), n in sorted(log.sites.items(), key=lambda kv: -kv[1]):
    print(f"{n:4d}  {name:40s} {site}")
