"""RCCL + the bench's allocator setting on one GPU (GPU box): expandable segments, a single-rank
RCCL communicator, the full LJSpeech Trainer with forced gradient buckets (hook-driven async
all-reduces during backward) for a few steps -- the multi-GPU bench path minus the peers."""
import os
import socket
import sys

os.environ.setdefault("PYTORCH_HIP_ALLOC_CONF", "expandable_segments:True")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from speakingstyle_amd.config import load_named  # noqa: E402
from speakingstyle_amd.data.synthetic import SyntheticBatches  # noqa: E402
from speakingstyle_amd.models.fastspeech2 import FastSpeech2  # noqa: E402
from speakingstyle_amd.parallel import ddp  # noqa: E402
from speakingstyle_amd.train.trainer import Trainer  # noqa: E402

s = socket.socket()
s.bind(("127.0.0.1", 0))
port = s.getsockname()[1]
s.close()
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}")
try:
    pp, mc, tc = load_named(sys.argv[1] if len(sys.argv) > 1 else "LJSpeech")
    torch.manual_seed(0)
    m = FastSpeech2(pp, mc).to("cuda").set_compute_dtype(torch.bfloat16)
    tr = Trainer(m, (pp, mc, tc), seed=1)
    tr.buckets = ddp.GradBuckets(tr.opt.arena, force=True)
    gen = SyntheticBatches(int(tc["optimizer"]["batch_size"]), device="cuda", max_seq_len=mc["max_seq_len"], seed=2,
                           frame_level=pp["preprocessing"]["pitch"]["feature"] == "frame_level")
    for i in range(4):
        losses, _, _ = tr.train_step(gen.make_batch())
        torch.cuda.synchronize()
        print(f"step {i}: loss {float(losses[0]):.4f} buckets issued in backward "
              f"{len(tr.buckets.last_launch_order)}/{len(tr.buckets.buckets)} calibrated={tr.buckets.calibrated()}",
              flush=True)
        assert torch.isfinite(losses[0])
    print("alloc conf:", os.environ["PYTORCH_HIP_ALLOC_CONF"], "ok")
finally:
    dist.destroy_process_group()
