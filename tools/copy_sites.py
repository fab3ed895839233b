"""Census of the runtime copy kernels (__amd_rocclr_copyBuffer, hipMemcpyAsync under torch copies) and torch
elementwise / cat / fill kernels of one training step, attributed to their Python call sites (GPU box):
python tools/copy_sites.py [config] [batch]  -> per call site: count of copyBuffer / other torch kernels."""
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.train.trainer import Trainer

    cfg = sys.argv[1] if len(sys.argv) > 1 else "LJSpeech"
    synth = cfg.startswith("synth:")  # synth:<config>: one batch-1 packed synthesis (eager) instead of a train step
    cfg = cfg.split(":", 1)[1] if synth else cfg
    pp, mc, tc = load_named(cfg)
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else (1 if synth else int(tc["optimizer"]["batch_size"]))
    torch.manual_seed(0)
    model = FastSpeech2(pp, mc).to("cuda").set_compute_dtype(torch.bfloat16)
    gen = SyntheticBatches(bs, device="cuda", max_seq_len=mc["max_seq_len"], seed=5,
                           frame_level=pp["preprocessing"]["pitch"]["feature"] == "frame_level")
    bats = [gen.make_batch() for _ in range(3)]
    if synth:
        import math

        from speakingstyle_amd.utils.model import get_vocoder

        with torch.no_grad():
            lin = model.variance_adaptor.duration_predictor.linear_layer
            lin.weight.normal_(0.0, 0.005)
            lin.bias.fill_(math.log(9.1))
        model.eval().requires_grad_(False)
        voc = get_vocoder(mc, torch.device("cuda"))

        def step(b):
            rows, lens, _ = model.infer_packed(b[2], b[3], b[4], b[5], b[6], b[7], b[8])
            voc.infer_packed(rows, lens, int16_scale=32768.0).cpu()
    else:
        tr = Trainer(model, (pp, mc, tc), seed=1)
        tr.use_priority_stream(True)
        step = tr.train_step
    for b in bats[:2]:
        step(b)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step(bats[2])
        torch.cuda.synchronize()
    sites, kinds = Counter(), Counter()
    total = Counter()
    for e in prof.events():
        ks = [k.name for k in getattr(e, "kernels", [])]
        if not ks:
            continue
        for k in ks:
            torchk = k.startswith("__amd_rocclr") or "at::native" in k
            if not torchk:
                continue
            kind = "copyBuffer" if "copyBuffer" in k else ("fill" if "Fill" in k else
                   ("cat" if "Cat" in k else ("copy" if "copy" in k else "elementwise/other")))
            total[kind] += 1
            st = [f for f in (e.stack or []) if "speakingstyle_amd" in f or "tools/" in f]
            site = " <- ".join(s.split("speakingstyle_amd/")[-1] for s in st[:3]) or e.name
            sites[(kind, e.name, site)] += 1
    print("per step:", dict(total))
    for (kind, op, site), n in sites.most_common(60):
        print(f"{n:4d} {kind:12s} {op:24s} {site}")


if __name__ == "__main__":
    main()
