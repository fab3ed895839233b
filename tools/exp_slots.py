"""Which parameters' gradients land outside their arena slot (copied by finalize_grads at the step end)?
Usage (GPU box): python tools/exp_slots.py [config]"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from speakingstyle_amd.config import load_named  # noqa: E402
from speakingstyle_amd.data.synthetic import SyntheticBatches  # noqa: E402
from speakingstyle_amd.models.fastspeech2 import FastSpeech2  # noqa: E402
from speakingstyle_amd.train.trainer import Trainer  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "LJSpeech"
    pp, mc, tc = load_named(cfg)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = FastSpeech2(pp, mc).to(dev)
    model.set_compute_dtype(torch.bfloat16)
    tr = Trainer(model, (pp, mc, tc), seed=0)
    tr.use_priority_stream(True)
    gen = SyntheticBatches(int(tc["optimizer"]["batch_size"]), device=dev, max_seq_len=mc["max_seq_len"], seed=1)
    names = {id(p): n for n, p in model.named_parameters()}
    a = tr.opt.arena
    got = []
    orig = a.ensure_slot

    def spy(p, i=None):
        if p.grad is not None and p.grad.data_ptr() != a._slot_ptr[id(p)]:
            got.append(f"{names.get(id(p), '?')}{tuple(p.shape)}")
        return orig(p, i)

    a.ensure_slot = spy
    for i in range(4):
        got.clear()
        tr.train_step(gen.make_batch())
        torch.cuda.synchronize()
        print(f"step {i}: copied {len(got)}: " + ", ".join(got), flush=True)


if __name__ == "__main__":
    main()
