"""Per-GPU frame budget (``mi355x.frames_per_gpu``) -- the MI355X batch semantics next to the
reference's global-batch split (``train.py:27-45``).

* ``FrameBudgetSampler``: every rank gets the same number of steps, batches are disjoint, within
  the padded-frame budget, deterministic per (seed, epoch) and resumable;
* ``SyntheticBatches(frames_per_batch=...)`` obeys the same budget;
* DP=2 (gloo) on budget-sized batches of DIFFERENT utterance counts per rank equals the
  single-process gradient of the union (global-count loss normalisation);
* ``train.py --synthetic`` at world 2 sizes each rank's batch by frames, not batch_size / world."""
import json
import os
import re
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lens(n=3000, seed=0):
    rng = np.random.default_rng(seed)
    return np.clip(rng.normal(570, 180, n), 40, 1200).astype(np.int64)


def test_sampler_budget_equal_steps_disjoint():
    from speakingstyle_amd.data.dataset import FrameBudgetSampler

    lens = _lens()
    budget = 40000
    world = 4
    per_rank = []
    for r in range(world):
        s = FrameBudgetSampler(None, budget, rank=r, world=world, seed=7, pool=1024, mel_lens=lens)
        per_rank.append(list(s))
    n = len(per_rank[0])
    assert n > 10 and all(len(p) == n for p in per_rank)
    seen = set()
    capped = np.minimum(lens, 1000)
    for p in per_rank:
        for b in p:
            assert len(b) * capped[b].max() <= budget          # padded frames within the budget
            assert not (set(b) & seen)
            seen |= set(b)
    assert len(seen) > 0.9 * len(lens)                          # only a small tail is dropped
    # deterministic and resumable: start=k continues the same plan
    again = list(FrameBudgetSampler(None, budget, rank=1, world=world, seed=7, pool=1024, mel_lens=lens))
    assert again == per_rank[1]
    tail = list(FrameBudgetSampler(None, budget, rank=1, world=world, seed=7, pool=1024, mel_lens=lens, start=5))
    assert tail == per_rank[1][5:]
    other = list(FrameBudgetSampler(None, budget, rank=1, world=world, seed=7, epoch=1, pool=1024, mel_lens=lens))
    assert other != per_rank[1]
    # utterance cap
    capd = list(FrameBudgetSampler(None, budget, rank=0, world=1, seed=7, mel_lens=lens, max_batch=20))
    assert max(len(b) for b in capd) <= 20


def test_sampler_rejects_budget_below_longest():
    from speakingstyle_amd.data.dataset import FrameBudgetSampler

    with pytest.raises(ValueError):
        FrameBudgetSampler(None, 500, mel_lens=_lens())


def test_global_batch_split_requires_bs_ge_world():
    from speakingstyle_amd.data.dataset import ShardedGroupSampler

    class _DS:
        def text_lengths(self):
            return np.arange(1, 100)

    with pytest.raises(ValueError):
        ShardedGroupSampler(_DS(), batch_size=2, rank=0, world=4)


def test_synthetic_budget():
    from speakingstyle_amd.data.synthetic import SyntheticBatches

    g = SyntheticBatches(8, frames_per_batch=30000, seed=3)
    sizes = []
    for _ in range(6):
        b = g.make_batch()
        n, M = len(b[0]), int(b[8])
        assert n * M <= 30000 and b[3].shape[0] == n and b[11].shape[0] == n
        sizes.append(n)
    assert len(set(sizes)) > 1  # utterance count follows the lengths


# ------------------------------------------------------------------ DP=2 gradient equality
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    from speakingstyle_amd.config import load_named

    pp, mc, tc = load_named("LJSpeech")
    mc["transformer"].update(encoder_layer=1, decoder_layer=1, encoder_dropout=0.0, decoder_dropout=0.0)
    mc["variance_predictor"]["dropout"] = 0.0
    return pp, mc, tc


def _shards():
    """Budget-sized batches of different utterance counts on the two ranks."""
    from speakingstyle_amd.data.synthetic import SyntheticBatches

    out = []
    for r, budget in ((0, 1200), (1, 2400)):
        g = SyntheticBatches(1, seed=50 + r, frames_per_batch=budget, max_seq_len=1000,
                             phone_counts=np.array([9, 12, 15, 20]), frames_per_phone=6.0)
        out.append(g.make_batch())
    return out


def _model(cfg):
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2

    torch.manual_seed(0)
    m = FastSpeech2(cfg[0], cfg[1])
    m.postnet.dropout = 0.0
    return m


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from speakingstyle_amd.parallel import ddp
    from speakingstyle_amd.train.trainer import Trainer

    ddp.init_distributed("gloo")
    cfg = _setup()
    tr = Trainer(_model(cfg), cfg, bucket_mb=1.0)
    captured = {}
    orig = tr.opt.step_and_update_lr

    def hook():
        captured["g"] = tr.opt.arena.grad.clone()
        return orig()

    tr.opt.step_and_update_lr = hook
    shard = _shards()[rank]
    tr.train_step(shard)
    q.put((rank, len(shard[0]), captured["g"].numpy().copy()))
    torch.distributed.destroy_process_group()


def test_dp2_frame_budget_matches_single_process():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, n, g = q.get(timeout=600)
        res[r] = (n, torch.from_numpy(g))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res[0][0] != res[1][0], "the two ranks should hold different utterance counts"
    torch.testing.assert_close(res[0][1], res[1][1])

    from speakingstyle_amd.models.loss import FastSpeech2Loss
    from speakingstyle_amd.train.optim import FlatArena

    cfg = _setup()
    model = _model(cfg)
    model.train()
    arena = FlatArena(list(reversed([p for p in model.parameters() if p.requires_grad])),
                      groups=model.fused_param_groups())
    shards = _shards()
    counts = torch.zeros(3)
    for s in shards:
        fr = s[7].clamp(max=1000).sum()
        counts += torch.stack([fr * 80, s[4].sum(), fr]).float()
    lf = FastSpeech2Loss(cfg[0], cfg[2])
    for s in shards:
        out = model(*s[2:])
        lf(s, out, None, global_counts=counts)[0].backward()
        arena.finalize_grads()
    torch.testing.assert_close(res[0][1], arena.grad, rtol=1e-4, atol=1e-6)


# ------------------------------------------------------------------ train.py at world 2
def test_train_cli_world2_frame_budget(tmp_path):
    from speakingstyle_amd.config import config_dir_triplet, load_yaml

    p, m, t = (load_yaml(x) for x in config_dir_triplet("LJSpeech"))
    p["path"]["preprocessed_path"] = os.path.join(ROOT, "preprocessed_data", "LJSpeech")
    m["transformer"].update(encoder_layer=1, decoder_layer=1, conv_filter_size=64, encoder_hidden=32,
                            decoder_hidden=32, encoder_head=2, decoder_head=2)
    m["variance_predictor"]["filter_size"] = 32
    t["optimizer"]["batch_size"] = 4           # global-split semantics would give 2 per rank
    t["mi355x"]["frames_per_gpu"] = 6000       # ~10 LJSpeech-length utterances per rank
    t["step"].update(total_step=2, log_step=1, synth_step=1000, val_step=1000, save_step=1000)
    for k in ("ckpt_path", "log_path", "result_path"):
        t["path"][k] = str(tmp_path / k)
    files = []
    for nm, obj in (("preprocess", p), ("model", m), ("train", t)):
        f = tmp_path / f"{nm}.yaml"
        f.write_text(yaml.safe_dump(obj))
        files.append(str(f))
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "train.py", "-p", files[0], "-m", files[1],
           "-t", files[2], "--synthetic", "--cpu", "--no_vocoder"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    # the two ranks print concurrently: their lines may interleave, so match the records, not lines
    recs = re.findall(r"\[rank (\d)\] first batch: (\d+) utterances, (\d+) padded mel frames \(frames_per_gpu=(\d+)\)",
                      r.stdout)
    assert sorted(int(x[0]) for x in recs) == [0, 1], r.stdout
    for _, n, frames, budget in recs:
        assert int(n) > 2 and int(frames) <= 6000 and budget == "6000"
    assert "Step 2/2" in r.stdout
