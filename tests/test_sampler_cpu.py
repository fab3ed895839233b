"""ShardedGroupSampler: shard-before-load grouping with the reference loader's order
(``train.py:27-41`` shuffle -> groups of batch_size*4 -> sort by text length ->
4 batches), resumable from (epoch, group)."""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dataset(bs=16):
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.data.dataset import Dataset

    pp, mc, tc = load_named("LJSpeech")
    pp["path"]["preprocessed_path"] = os.path.join(ROOT, "preprocessed_data", "LJSpeech")
    tc["optimizer"]["batch_size"] = bs
    return Dataset("train.txt", pp, tc, sort=True, drop_last=True)


def test_shards_partition_sorted_groups():
    from speakingstyle_amd.data.dataset import ShardedGroupSampler

    ds = _dataset()
    bs, world = 16, 3
    tl = ds.text_lengths()
    full = list(ShardedGroupSampler(ds, bs, 4, 0, 1, seed=5))
    assert len(full) == len(tl) // (bs * 4)
    shards = [list(ShardedGroupSampler(ds, bs, 4, r, world, seed=5)) for r in range(world)]
    for gi in (0, 1, len(full) - 1):
        g = full[gi]
        assert list(tl[g]) == sorted(tl[g], reverse=True)  # sorted by text length, longest first
        for k in range(4):
            batch = g[k * bs:(k + 1) * bs]
            got = []
            for r in range(world):
                n = len(range(r, bs, world))
                got.extend(shards[r][gi][k * n:(k + 1) * n])
            assert sorted(got) == sorted(batch)
            for r in range(world):
                n = len(range(r, bs, world))
                assert shards[r][gi][k * n:(k + 1) * n] == batch[r::world]


def test_resume_position_and_epochs_differ():
    from speakingstyle_amd.data.dataset import ShardedGroupSampler

    ds = _dataset()
    a = list(ShardedGroupSampler(ds, 16, 4, 1, 2, seed=9, epoch=2))
    b = list(ShardedGroupSampler(ds, 16, 4, 1, 2, seed=9, epoch=2, start=5))
    assert b == a[5:]
    c = list(ShardedGroupSampler(ds, 16, 4, 1, 2, seed=9, epoch=3))
    assert c[0] != a[0]


def test_collate_local_splits_per_batch():
    from speakingstyle_amd.data.dataset import ShardedGroupSampler

    ds = _dataset()
    s = ShardedGroupSampler(ds, 16, 4, 0, 3, seed=1)
    idx = next(iter(s))
    fake = [{"id": str(i), "raw_text": "", "speaker": 0, "text": np.ones(int(ds.text_lengths()[i]), np.int64),
             "mel": np.zeros((3, 80), np.float32), "pitch": np.zeros(2, np.float32),
             "energy": np.zeros(2, np.float32), "duration": np.ones(2, np.int64)} for i in idx]
    out = ds.collate_local(fake)
    assert len(out) == 4 and all(len(b[0]) == 6 for b in out)  # ceil(16/3) rows of rank 0 per batch
    assert [b[0] for b in out][0] == [str(i) for i in idx[:6]]
