"""GradBuckets on the GPU gradient path, rehearsed on the CPU (gloo, world 2).

On MI355X the HIP backward kernels ``claim`` a parameter's arena slot and write
the weight gradient in place (``ops/gradslots.py``); AccumulateGrad adopts that
view, later uses of the same parameter accumulate into it, and the
post-accumulate hooks drive the bucket all-reduces.  This test forces exactly
that path with a custom autograd Function that writes into claimed slots, uses
one parameter twice and leaves one unused, and checks:

* the first step calibrates (no collective in hooks), later steps launch buckets
  from the hooks, always in bucket-index order;
* the reduced gradient equals the single-process sum over both shards;
* replicas stay identical after the optimizer step."""
import os
import socket

import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SIDE = [False]  # simulate the side-stream weight-gradient path (hip.wgrad_async) in SlotMatmul


class SlotMatmul(torch.autograd.Function):
    """y = x @ w.T with the weight gradient written into w's arena slot when claimable."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        ctx.w = w
        return x @ w.t()

    @staticmethod
    def backward(ctx, gy):
        from speakingstyle_amd.ops import gradslots

        x, w = ctx.saved_tensors
        gw = gy.t() @ x
        slot = gradslots.claim(ctx.w)
        if slot is not None:
            slot.copy_(gw)  # "kernel" writes in place
            gw = slot
            if SIDE[0] and gradslots.single_contribution(ctx.w):
                gradslots.mark_side([ctx.w])  # what hip.wgrad_async records when it takes the side stream
        return gy @ w, gw


class Toy(torch.nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.w = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(16, 16) * 0.2) for _ in range(6)])
        self.shared = torch.nn.Parameter(torch.randn(16, 16) * 0.2)   # used twice per step
        self.plain = torch.nn.Parameter(torch.randn(16) * 0.1)        # gradient from a plain torch op
        self.unused = torch.nn.Parameter(torch.randn(16))             # never receives a gradient

    def forward(self, x):
        h = SlotMatmul.apply(x, self.shared)
        for w in self.w:
            h = torch.tanh(SlotMatmul.apply(h, w))
        h = SlotMatmul.apply(h, self.shared) + self.plain
        return (h ** 2).mean()


def _data(rank, step):
    g = torch.Generator().manual_seed(100 * step + rank)
    return torch.randn(8, 16, generator=g)


def _arena(model):
    from speakingstyle_amd.train.optim import FlatArena

    return FlatArena(list(reversed(list(model.parameters()))))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from speakingstyle_amd.parallel import ddp

    ddp.init_distributed("gloo")
    model = Toy()
    arena = _arena(model)
    gb = ddp.GradBuckets(arena, bucket_mb=16 * 16 * 4 * 1.5 / 2 ** 20)  # ~1 parameter per bucket
    res = []
    for step in range(3):
        loss = model(_data(rank, step))
        loss.backward()
        in_hooks = list(gb.launch_order)  # launched before finish()
        gb.finish()
        res.append((gb.calibrated(), in_hooks, list(gb.last_launch_order), arena.grad.clone()))
        with torch.no_grad():
            arena.data.add_(arena.grad, alpha=-0.1)
        arena.zero_grad()
    q.put((rank, [(c, h, o, g.numpy()) for c, h, o, g in res], arena.data.numpy().copy(), len(gb.buckets)))
    torch.distributed.destroy_process_group()


def test_slot_path_buckets_dp2():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, steps, data, nb = q.get(timeout=300)
        out[r] = (steps, data, nb)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nb = out[0][2]
    assert nb >= 6
    for r in range(world):
        steps = out[r][0]
        # step 0: calibration -- nothing launched from hooks, everything at finish in index order
        assert steps[0][1] == [] and steps[0][2] == list(range(nb))
        for cal, in_hooks, order, _ in steps[1:]:
            assert cal
            assert order == list(range(nb))         # strictly in bucket-index order
            assert len(in_hooks) >= nb // 2         # overlapped with backward
    torch.testing.assert_close(torch.from_numpy(out[0][1]), torch.from_numpy(out[1][1]))

    # single process: summed gradients of both shards, same update rule
    model = Toy()
    arena = _arena(model)
    for step in range(3):
        for r in range(world):
            model(_data(r, step)).backward()
        arena.finalize_grads()
        torch.testing.assert_close(torch.from_numpy(out[0][0][step][3]), arena.grad, rtol=1e-5, atol=1e-6)
        with torch.no_grad():
            arena.data.add_(arena.grad, alpha=-0.1)
        arena.zero_grad()


class Toy2(Toy):
    """``use_shared=False`` drops ``shared`` from the graph (it accumulates once per backward in the
    calibration step)."""

    def forward(self, x, use_shared=True):
        h = SlotMatmul.apply(x, self.shared) if use_shared else x
        for w in self.w:
            h = torch.tanh(SlotMatmul.apply(h, w))
        return (h ** 2).mean() + self.plain.sum()


def _worker_changed(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from speakingstyle_amd.parallel import ddp

    ddp.init_distributed("gloo")
    model = Toy2()
    arena = _arena(model)
    gb = ddp.GradBuckets(arena, bucket_mb=16 * 16 * 4 * 1.5 / 2 ** 20)
    out = {}
    # step 0 calibrates; step 1 leaves `shared` out (fewer accumulations: its bucket is held back to
    # finish(), still correct)
    for step, use in ((0, True), (1, False)):
        model(_data(rank, step), use).backward()
        gb.finish()
        out[step] = arena.grad.clone().numpy()
        arena.zero_grad()
    out["mismatched"] = gb.mismatched_steps
    # step 2 runs a second backward before finish(): every parameter accumulates twice, into buckets
    # the first backward already put on the wire -> must raise instead of corrupting them
    model(_data(rank, 2)).backward()
    try:
        model(_data(rank, 3)).backward()
        out["raised"] = None
    except RuntimeError as e:
        out["raised"] = str(e)
    q.put((rank, out))
    torch.distributed.destroy_process_group()


def test_graph_change_after_calibration_dp2():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker_changed, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, o = q.get(timeout=300)
        res[r] = o
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert res[r]["mismatched"] == 1
        assert res[r]["raised"] is not None and "calibration" in res[r]["raised"]
    model = Toy2()
    arena = _arena(model)
    for step, use in ((0, True), (1, False)):
        for r in range(world):
            model(_data(r, step), use).backward()
        arena.finalize_grads()
        torch.testing.assert_close(torch.from_numpy(res[0][step]), arena.grad, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(torch.from_numpy(res[1][step]), arena.grad, rtol=1e-5, atol=1e-6)
        arena.zero_grad()


def test_race_suspect_poisons_slot_and_adam_skips():
    """A parameter whose previous backward ended with its single slot view (so its next weight gradient may
    be written by the side stream) but that now receives a second, main-stream-summed contribution: the
    arena slot is poisoned before the optimizer -> the non-finite guard skips the step, the replica is
    unchanged, the warning fires, and the flag flip puts it back on the main stream for the next step."""
    import warnings

    import pytest

    from speakingstyle_amd.ops import gradslots
    from speakingstyle_amd.train.optim import FlatArena

    torch.manual_seed(1)
    w = torch.nn.Parameter(torch.randn(8, 8))
    arena = FlatArena([w])
    x = torch.randn(4, 8)

    def backward(twice):
        y = SlotMatmul.apply(x, w)
        if twice:
            y = y + SlotMatmul.apply(x, w)  # graph changed: a second contribution (autograd sums them)
        y.sum().backward()

    backward(False)
    arena.finalize_grads()
    gradslots.note_contributions(arena)
    assert gradslots.single_contribution(w)
    arena.zero_grad()
    before = gradslots.race_suspects[0]
    # the side stream was off this step (e.g. the side_wgrad auto policy): nothing can have raced -> copied
    backward(True)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        arena.finalize_grads()
    assert gradslots.race_suspects[0] == before and torch.isfinite(arena.grad[: w.numel()]).all()
    arena.zero_grad()
    # single flag restored, side stream on: the slot was written on the side stream -> poisoned
    backward(False)
    arena.finalize_grads()
    gradslots.note_contributions(arena)
    arena.zero_grad()
    SIDE[0] = True
    try:
        backward(True)
    finally:
        SIDE[0] = False
    with pytest.warns(RuntimeWarning, match="skipped"):
        arena.finalize_grads()
    assert gradslots.race_suspects[0] == before + 1
    assert torch.isnan(arena.grad[: w.numel()]).all()
    gradslots.note_contributions(arena)
    assert not gradslots.single_contribution(w)  # next step: main stream, no race
    arena.zero_grad()
    backward(True)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        arena.finalize_grads()
    assert torch.isfinite(arena.grad[: w.numel()]).all()
