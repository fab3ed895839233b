#!/usr/bin/env python
"""Which parameter gradients of a training step are produced outside their arena slot (and
copied in by ``ensure_slot``), and which torch ops run on the GPU during one step (GPU box)."""
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.train.trainer import Trainer

    cfg = sys.argv[1] if len(sys.argv) > 1 else "LJSpeech"
    pp, mc, tc = load_named(cfg)
    torch.manual_seed(0)
    model = FastSpeech2(pp, mc).to("cuda").set_compute_dtype(torch.bfloat16)
    tr = Trainer(model, (pp, mc, tc), seed=1)
    gen = SyntheticBatches(int(tc["optimizer"]["batch_size"]), device="cuda", max_seq_len=mc["max_seq_len"], seed=5)
    b = gen.make_batch()
    tr.train_step(b)
    names = {id(p): n for n, p in model.named_parameters()}
    copied = []
    arena = tr.opt.arena
    orig = arena.ensure_slot

    def ens(p, i=None):
        g = p.grad
        if g is not None and g.data_ptr() != arena._slot_ptr[id(p)]:
            copied.append(names.get(id(p), "?"))
        return orig(p, i)

    arena.ensure_slot = ens
    ops = Counter()

    import traceback

    skip = ("view", "detach", "slice", "empty", "select", "unsqueeze", "alias", "lift_fresh", "as_strided",
            "expand", "t.default", "permute", "reshape", "squeeze", "_unsafe_view", "transpose")
    sites = Counter()

    class Mode(torch.utils._python_dispatch.TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            ops[str(func)] += 1
            if not any(k in str(func) for k in skip):
                fr = [f for f in traceback.extract_stack() if "speakingstyle_amd" in f.filename]
                where = f"{os.path.relpath(fr[-1].filename)}:{fr[-1].lineno}" if fr else "?"
                sites[(str(func), where)] += 1
            return func(*args, **(kwargs or {}))

    with Mode():
        tr.train_step(b)
    torch.cuda.synchronize()
    print("slot copies:", len(copied))
    for n in copied:
        print("  ", n)
    print("torch ops dispatched in one step:", sum(ops.values()))
    for k, v in ops.most_common(40):
        print(f"  {v:4d}  {k}")
    print("compute ops by call site:")
    for (f, w), v in sites.most_common(60):
        print(f"  {v:4d}  {f:40s} {w}")


if __name__ == "__main__":
    main()
