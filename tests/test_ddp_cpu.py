"""Multi-process data parallelism on CPU (gloo, world_size 2).

DP=2 with bucketed, backward-overlapped all-reduce of the flat gradient arena and
global-count loss normalisation must equal the single-process gradient of the
same two shards (BatchNorm statistics are per replica, like the reference's
DataParallel), and the optimizer step must keep replicas bit-identical."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(name="BC2013"):
    from speakingstyle_amd.config import load_named

    pp, mc, tc = load_named(name)
    mc["transformer"].update(encoder_layer=1, decoder_layer=1)
    if mc.get("reference_encoder"):
        mc["reference_encoder"].update(encoder_layer=1, conv_layer=1, dropout=0.0)
    mc["transformer"].update(encoder_dropout=0.0, decoder_dropout=0.0)
    mc["variance_predictor"]["dropout"] = 0.0
    pp["path"]["preprocessed_path"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                   "preprocessed_data", "BC2013")
    return pp, mc, tc


def _model(cfg):
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2

    torch.manual_seed(0)
    m = FastSpeech2(cfg[0], cfg[1])
    m.postnet.dropout = 0.0
    return m


def _shards():
    from speakingstyle_amd.data.synthetic import SyntheticBatches

    a = SyntheticBatches(2, seed=1, phone_counts=[11, 15, 9], max_seq_len=1000).make_batch()
    b = SyntheticBatches(2, seed=2, phone_counts=[13, 7, 10], max_seq_len=1000).make_batch()
    return a, b


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from speakingstyle_amd.parallel import ddp
    from speakingstyle_amd.train.trainer import Trainer

    ddp.init_distributed("gloo")
    cfg = _setup()
    model = _model(cfg)
    tr = Trainer(model, cfg, bucket_mb=1.0)  # small buckets -> many overlapped all-reduces
    shard = _shards()[rank]
    # capture the reduced gradient just before the optimizer consumes it
    captured = {}
    orig = tr.opt.step_and_update_lr

    def hook():
        captured["g"] = tr.opt.arena.grad.clone()
        return orig()

    tr.opt.step_and_update_lr = hook
    tr.train_step(shard)
    q.put((rank, captured["g"].numpy().copy(), tr.opt.arena.data.numpy().copy(), len(tr.buckets.buckets)))
    torch.distributed.destroy_process_group()


def test_dp2_matches_single_process():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, g, data, nb = q.get(timeout=600)
        res[r] = (torch.from_numpy(g), torch.from_numpy(data), nb)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res[0][2] > 1, "expected several gradient buckets"
    torch.testing.assert_close(res[0][0], res[1][0])          # all-reduced grads identical
    torch.testing.assert_close(res[0][1], res[1][1])          # replicas stay in sync after Adam

    # single-process reference: sum of the two shards' grads with global-count normalisation
    from speakingstyle_amd.models.loss import FastSpeech2Loss
    from speakingstyle_amd.train.optim import FlatArena

    cfg = _setup()
    model = _model(cfg)
    model.train()
    arena = FlatArena(list(reversed([p for p in model.parameters() if p.requires_grad])),
                      groups=model.fused_param_groups())
    shards = _shards()
    n_mel = 80
    counts = torch.zeros(3)
    for s in shards:
        fr = s[7].clamp(max=1000).sum()
        counts += torch.stack([fr * n_mel, s[4].sum(), fr]).float()
    lf = FastSpeech2Loss(cfg[0], cfg[2])
    for s in shards:
        out = model(*s[2:])
        named = model.film_scalars()
        loss = lf(s, out, named, global_counts=counts)[0]
        loss = loss - 0.5 * lf.lambda_f * torch.sum(named ** 2)
        loss.backward()
        arena.finalize_grads()
    torch.testing.assert_close(res[0][0], arena.grad, rtol=1e-4, atol=1e-6)


def _flat_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from speakingstyle_amd.parallel import ddp

    ddp.init_distributed("gloo")
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.zeros(n)) for n in (5, 300, 7, 1000)]
    ps.append(torch.nn.Parameter(torch.zeros(3)))  # no grad: skipped
    for i, p in enumerate(ps[:-1]):
        p.grad = torch.full_like(p, float(rank + 1) * (i + 1)) + torch.arange(p.numel()).float() * rank
    ddp.allreduce_grads_flat(ps, bucket_mb=1e-3)  # ~262 floats per bucket: several buckets, one oversized
    # numpy copies: torch CPU tensors travel by fd passing, which breaks once this process has exited
    q.put((rank, [p.grad.numpy().copy() if p.grad is not None else None for p in ps]))
    torch.distributed.destroy_process_group()


def test_allreduce_grads_flat_averages_over_ranks():
    """The HiFi-GAN HIP path's discriminator-gradient all-reduce (vocoder/train.py:hip_step): flat buckets,
    the rank average, grads without .grad skipped."""
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_flat_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = {r: [None if g is None else torch.from_numpy(g) for g in gs] for r, gs in res.items()}
    for i, n in enumerate((5, 300, 7, 1000)):
        want = (torch.full((n,), 1.0 * (i + 1)) + torch.full((n,), 2.0 * (i + 1)) + torch.arange(n).float()) / 2
        torch.testing.assert_close(res[0][i], want)
        torch.testing.assert_close(res[1][i], want)
    assert res[0][4] is None
