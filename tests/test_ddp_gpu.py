"""The data-parallel gradient path on a real GPU with RCCL (single-rank communicator -- a 1-GPU
box cannot host two RCCL ranks): the HIP backward kernels write weight gradients into arena slots,
post-accumulate hooks drive asynchronous RCCL all-reduces of arena slices in bucket order while
the backward continues, ``finish()`` orders the compute stream after them.  With one rank every
all-reduce is an identity, so the reduced gradients must equal a plain (non-DP) step's bitwise.

The multi-rank launcher / gloo path is covered on the CPU (tests/test_bench_cpu.py,
tests/test_ddp_cpu.py, tests/test_ddp_slots_cpu.py)."""
import os
import socket
import warnings

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _side_stream_on():
    """These tests are about buckets behind queued side-stream weight gradients: force the side stream on
    (the automatic policy turns it off for steps this small, experimental.side_wgrad)."""
    from speakingstyle_amd import experimental

    with experimental.overrides(side_wgrad="1"):
        yield


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _trainer(cfg, seed=11):
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.train.trainer import Trainer

    torch.manual_seed(seed)
    m = FastSpeech2(*cfg[:2]).to("cuda").set_compute_dtype(torch.bfloat16)
    return Trainer(m, cfg, seed=1234)


def _capture(tr, step=True):
    """Record the reduced gradient of every step; ``step=False`` also skips Adam (weights stay put)."""
    grads = []
    orig = tr.opt.step_and_update_lr

    def hook():
        grads.append(tr.opt.arena.grad.clone())
        return orig() if step else 0.0

    tr.opt.step_and_update_lr = hook
    return grads


@pytest.mark.parametrize("name,prio", [("LJSpeech", False), ("BC2013", False), ("LJSpeech", True)])
def test_rccl_bucket_path_single_rank(name, prio, monkeypatch):
    """BC2013 adds the FiLM sites: scalar gradients folded with the L2 term into their slots and the
    shared style gamma/beta buffer must keep the per-parameter hook counts stable across steps.

    ``prio``: the bench / train.py stream layout (high-priority compute stream, weight gradients on the
    side stream).  Buckets whose weight gradients are still queued on the side stream are issued with
    the side stream current (ordered after both streams, the compute stream does not wait): the
    reduced gradients must still equal the plain step's bitwise."""
    import torch.distributed as dist

    from speakingstyle_amd.ops import hip

    side_issued = []
    orig_side = hip.side_stream_for_collective

    def counting(dev):
        s = orig_side(dev)
        side_issued.append(s is not None)
        return s

    monkeypatch.setattr(hip, "side_stream_for_collective", counting)

    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.parallel import ddp

    pp, mc, tc = load_named(name)
    mc["transformer"]["encoder_layer"] = mc["transformer"]["decoder_layer"] = 2
    cfg = (pp, mc, tc)
    fl = pp["preprocessing"]["pitch"]["feature"] == "frame_level"
    batches = [SyntheticBatches(8, device="cuda", seed=3 + i, frame_level=fl).make_batch() for i in range(3)]

    ref = _trainer(cfg)
    if prio:
        ref.use_priority_stream()
    g_ref = _capture(ref)
    for b in batches:
        ref.train_step(b)

    dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{_port()}")
    try:
        tr = _trainer(cfg)
        if prio:
            tr.use_priority_stream()
        tr.buckets = ddp.GradBuckets(tr.opt.arena, bucket_mb=4.0, force=True)  # many buckets
        nb = len(tr.buckets.buckets)
        assert nb >= 4
        g = _capture(tr)
        in_hooks = []
        for i, b in enumerate(batches):
            orig_finish = tr.buckets.finish

            def finish():
                in_hooks.append(list(tr.buckets.launch_order))  # issued during backward
                return orig_finish()

            tr.buckets.finish = finish
            tr.train_step(b)
            tr.buckets.finish = orig_finish
            assert tr.buckets.last_launch_order == list(range(nb))
        torch.cuda.synchronize()
        assert in_hooks[0] == [] and tr.buckets.calibrated()
        assert len(in_hooks[1]) >= nb // 2 and len(in_hooks[2]) >= nb // 2  # overlapped with backward
        for a, r in zip(g, g_ref):
            assert torch.equal(a, r)
        assert torch.equal(tr.opt.arena.data, ref.opt.arena.data)
        if prio:
            assert any(side_issued), "no bucket was issued behind queued side-stream weight gradients"
    finally:
        dist.destroy_process_group()
        if prio:
            torch.cuda.set_stream(torch.cuda.default_stream())


class _StreamWork:
    """Work handle of a stream-ordered test reduction: wait() orders the caller's stream after it."""

    def __init__(self):
        self.ev = torch.cuda.Event()
        self.ev.record()

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


class _GatherX2Work:
    """wait(): the caller's stream waits for the ProcessGroup's all_gather, then t = 2 * (what RCCL read)."""

    def __init__(self, work, out, t):
        self.work, self.out, self.t = work, out, t

    def wait(self):
        self.work.wait()
        torch.mul(self.out, 2.0, out=self.t)

    def is_completed(self):
        return self.work.is_completed()


def test_rccl_bucket_order_non_idempotent_with_late_side_stream(record_property):
    """The 1-rank RCCL bucket path with a reduction that is NOT an identity (x2: RCCL PREMUL_SUM, or -- if
    this RCCL lacks it -- an in-place x2 on the same stream the collective would use) and a ~20 ms spin
    injected on the weight-gradient side stream ahead of a step's side-stream launches.  A bucket reduced
    before its last side-stream weight gradient landed would be doubled from a partial slot and then
    overwritten by the late kernel: the reduced gradients would not equal exactly 2x the plain step's."""
    import torch.distributed as dist

    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.ops import hip
    from speakingstyle_amd.parallel import ddp

    pp, mc, tc = load_named("LJSpeech")
    mc["transformer"]["encoder_layer"] = mc["transformer"]["decoder_layer"] = 2
    cfg = (pp, mc, tc)
    batches = [SyntheticBatches(8, device="cuda", seed=30 + i).make_batch() for i in range(3)]
    ref = _trainer(cfg)
    ref.use_priority_stream()
    g_ref = _capture(ref, step=False)  # no Adam: both runs see the same weights every step
    for b in batches:
        ref.train_step(b)
    torch.cuda.set_stream(torch.cuda.default_stream())

    dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{_port()}")
    try:
        tr = _trainer(cfg)
        tr.use_priority_stream()
        tr.buckets = ddp.GradBuckets(tr.opt.arena, bucket_mb=4.0, force=True)
        probe = torch.ones(4, device="cuda")
        try:
            dist.all_reduce(probe, op=dist._make_nccl_premul_sum(2.0))
            torch.cuda.synchronize()
            premul = bool((probe == 2).all())
        except Exception:  # noqa: BLE001 -- RCCL without ncclRedOpCreatePreMulSum
            premul = False

        branch = "premul_sum" if premul else "all_gather_x2"
        # which branch ran goes into the test log (warnings summary) and the junit properties
        warnings.warn(f"RCCL non-idempotent bucket reduction branch: {branch}", UserWarning)
        print(f"RCCL non-idempotent bucket reduction branch: {branch}", flush=True)
        record_property("rccl_branch", branch)

        def doubled(t):
            if premul:
                return dist.all_reduce(t, op=dist._make_nccl_premul_sum(2.0), async_op=True)
            # no PREMUL_SUM: still a collective of the ProcessGroup, on its internal stream -- a 1-rank
            # all_gather copies t as the RCCL kernel sees it (ordered exactly like the real all-reduce), and the
            # x2 write-back happens after the work's wait(): a bucket read before its last side-stream weight
            # gradient landed would be written back doubled from the partial slot
            out = torch.empty_like(t)
            w = dist.all_gather_into_tensor(out, t, async_op=True)
            return _GatherX2Work(w, out, t)

        tr.buckets.collective = doubled
        g = _capture(tr, step=False)
        delayed = [0]
        orig_async = hip.wgrad_async

        def late(launch, inputs, slots_ok, params=()):
            side_ok = (hip._SIDE_WGRAD[0] and slots_ok
                       and all(hip.gradslots.single_contribution(p) for p in params))
            if side_ok and armed[0] and delayed[0] == 0:
                with torch.cuda.stream(hip._side_stream(inputs[0].device)):
                    torch.cuda._sleep(40_000_000)  # ~20 ms spin ahead of this step's side-stream kernels
                delayed[0] += 1
            return orig_async(launch, inputs, slots_ok, params)

        armed = [False]
        hip.wgrad_async = late
        try:
            for i, b in enumerate(batches):
                armed[0] = i >= 1  # after the calibration step: buckets go out from the hooks
                delayed[0] = 0
                tr.train_step(b)
                if i >= 1:
                    assert delayed[0] == 1, "no side-stream weight gradient to delay"
        finally:
            hip.wgrad_async = orig_async
        torch.cuda.synchronize()
        assert tr.buckets.calibrated()
        # step 0 (calibration) launches every bucket at finish() -- also doubled
        for a, r in zip(g, g_ref):
            assert torch.equal(a, 2.0 * r), (a - 2.0 * r).abs().max().item()
    finally:
        dist.destroy_process_group()
        torch.cuda.set_stream(torch.cuda.default_stream())
