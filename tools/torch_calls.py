"""Python call sites of the torch tensor ops that launch copy / fill / elementwise kernels on the GPU during one
training step (or one batch-1 packed synthesis: ``synth:<config>``): Tensor.copy_ / clone / to / contiguous /
float / fill_ / zero_ / __add__ ... and torch.cat / zeros / full / stack are wrapped and their callers counted.
python tools/torch_calls.py [LJSpeech | LibriTTS | synth:BC2013_GST] [batch]"""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SITES = collections.Counter()
ON = [False]


def _site():
    fr = [f for f in traceback.extract_stack()[:-2] if "speakingstyle_amd" in f.filename]
    return " <- ".join(f"{f.filename.split('speakingstyle_amd/')[-1]}:{f.lineno}" for f in fr[-2:][::-1]) or "?"


def wrap(owner, name, test):
    orig = getattr(owner, name)

    def w(*a, **k):
        r = orig(*a, **k)
        if ON[0] and test(a, k, r):
            SITES[(name, _site())] += 1
        return r

    setattr(owner, name, w)


def cuda_any(a, k, r):
    ts = [x for x in list(a) + list(k.values()) + [r] if isinstance(x, torch.Tensor)]
    return any(t.is_cuda for t in ts)


def launched(a, k, r):
    """A kernel (or runtime copy) ran: conversions / slicing count only when they made new storage."""
    if not cuda_any(a, k, r):
        return False
    src = a[0] if a and isinstance(a[0], torch.Tensor) else None
    if isinstance(r, torch.Tensor) and src is not None:
        if r is src:
            return False
        try:
            if r.untyped_storage().data_ptr() == src.untyped_storage().data_ptr():
                return False  # a view
        except Exception:  # noqa: BLE001
            pass
    return True


def main():
    for n in ("copy_", "clone", "to", "contiguous", "float", "fill_", "zero_", "__add__", "__mul__", "__sub__",
              "__truediv__", "__floordiv__", "__rshift__", "add_", "mul_", "masked_fill", "masked_fill_",
              "__getitem__", "sum", "clamp", "repeat", "index_select", "long", "int"):
        wrap(torch.Tensor, n, launched)
    for n in ("cat", "zeros", "full", "stack", "zeros_like", "ones", "arange", "tensor"):
        wrap(torch, n, cuda_any)
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.train.trainer import Trainer

    cfg = sys.argv[1] if len(sys.argv) > 1 else "LJSpeech"
    synth = cfg.startswith("synth:")
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
    ON[0] = True
    step(bats[2])
    torch.cuda.synchronize()
    ON[0] = False
    print("total calls:", sum(SITES.values()))
    for (n, site), c in SITES.most_common(70):
        print(f"{c:4d} {n:14s} {site}")


if __name__ == "__main__":
    main()
