"""Diagnose side-stream weight gradients: plain trainer with/without the side stream (bitwise?), the
slot-copy counter, and the 1-rank RCCL bucket path with the side stream."""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speakingstyle_amd.config import load_named  # noqa: E402
from speakingstyle_amd.data.synthetic import SyntheticBatches  # noqa: E402
from speakingstyle_amd.models.fastspeech2 import FastSpeech2  # noqa: E402
from speakingstyle_amd.ops import hip  # noqa: E402
from speakingstyle_amd.parallel import ddp  # noqa: E402
from speakingstyle_amd.train.trainer import Trainer  # noqa: E402

pp, mc, tc = load_named("LJSpeech")
mc["transformer"]["encoder_layer"] = mc["transformer"]["decoder_layer"] = 2
cfg = (pp, mc, tc)
batches = [SyntheticBatches(8, device="cuda", seed=3 + i).make_batch() for i in range(3)]


def run(side, buckets=False):
    hip.set_wgrad_stream(side)
    torch.manual_seed(11)
    m = FastSpeech2(pp, mc).to("cuda").set_compute_dtype(torch.bfloat16)
    tr = Trainer(m, cfg, seed=1234)
    if buckets:
        tr.buckets = ddp.GradBuckets(tr.opt.arena, bucket_mb=4.0, force=True)
    grads = []
    orig = tr.opt.step_and_update_lr

    def hook():
        grads.append(tr.opt.arena.grad.clone())
        return orig()

    tr.opt.step_and_update_lr = hook
    for b in batches:
        tr.train_step(b)
    torch.cuda.synchronize()
    names = {id(p): n for n, p in m.named_parameters()}
    return grads, tr.opt.arena.copied, tr, names


g0, c0, t0, names = run(False)
g1, c1, t1, _ = run(True)
print("plain: copies no-side", c0, "side", c1, "equal", [torch.equal(a, b) for a, b in zip(g0, g1)])
s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
import torch.distributed as dist  # noqa: E402
dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}")
for side in (False, True):
    g2, c2, t2, names2 = run(side, buckets=True)
    eq = [torch.equal(a, b) for a, b in zip(g0, g2)]
    print("buckets side", side, "copies", c2, "equal", eq)
    if not all(eq):
        a = t2.opt.arena
        bad = []
        for i, p in enumerate(a.params):
            s_, e_ = a.slice(i)
            if not torch.equal(g2[-1][s_:e_], g0[-1][s_:e_]):
                bad.append(names2.get(id(p), "?"))
        print("  differing params (last step):", bad[:20], len(bad))
dist.destroy_process_group()
