"""Length-bucketed vocoding (``Generator.infer(..., lengths=)``): each length-sorted group is
vocoded at ``min(T, max_len + receptive_radius())`` frames instead of the padded batch.  The
valid samples must equal the padded-batch result (the reference vocodes padded and trims,
``utils/model.py:97-115``), and the halo must be necessary."""
import numpy as np
import torch

from speakingstyle_amd.models.hifigan import AttrDict, Generator, default_config


def _tiny():
    h = AttrDict(default_config())
    h.update(upsample_rates=[4, 2], upsample_kernel_sizes=[8, 4], upsample_initial_channel=32,
             resblock_kernel_sizes=[3, 5], resblock_dilation_sizes=[[1, 2], [1, 3]], num_mels=8)
    torch.manual_seed(0)
    g = Generator(h).eval()
    with torch.no_grad():  # larger weights than the 0.01 init so far-away frames actually matter
        for p in g.parameters():
            p.mul_(8.0)
    return g, 8


def test_receptive_radius_hifigan_v1():
    g = Generator(default_config())
    r = g.receptive_radius()
    # conv_pre 3 + ConvT 1 + 8x-stage MRF 60/8 + ... (see receptive_radius) -> a dozen-odd frames
    assert 10 <= r <= 20, r


def test_buckets_equal_padded_on_valid_samples():
    g, hop = _tiny()
    lengths = [40, 12, 25, 7, 33, 18]
    B, T = len(lengths), max(lengths)
    mel = torch.randn(B, T, 8)
    ref = g.infer(mel)
    out = g.infer(mel, lengths=lengths, max_buckets=3, bucket_cost=0)
    assert len(g.length_buckets(lengths, T, g.receptive_radius(), 3, 0)) == 3
    assert out.shape == ref.shape
    for b, L in enumerate(lengths):
        torch.testing.assert_close(out[b, : L * hop], ref[b, : L * hop], rtol=1e-5, atol=1e-6)


def test_halo_is_necessary():
    g, hop = _tiny()
    lengths = [40, 9, 9, 9]
    mel = torch.randn(4, 40, 8)
    ref = g.infer(mel)
    g.receptive_radius = lambda: 0  # truncate exactly at the valid length
    out = g.infer(mel, lengths=lengths, max_buckets=2, bucket_cost=0)
    err = max((out[b, : L * hop] - ref[b, : L * hop]).abs().max().item() for b, L in enumerate(lengths))
    assert err > 1e-4


def test_bucket_dp_is_optimal_small():
    rng = np.random.default_rng(3)
    L = rng.integers(5, 200, 9)
    T, halo, k, c = int(L.max()), 7, 3, 50
    groups = Generator.length_buckets(L, T, halo, k, c)
    assert sorted(np.concatenate([g[0] for g in groups]).tolist()) == list(range(9))
    got = sum(len(i) * w + c for i, w in groups)
    for i, w in groups:
        assert w == min(T, int(L[i].max()) + halo)
    # brute force over contiguous partitions of the sorted lengths into <= k groups
    s = np.sort(L)
    import itertools
    best = np.inf
    for m in range(1, k + 1):
        for cuts in itertools.combinations(range(1, 9), m - 1):
            edges = (0,) + cuts + (9,)
            best = min(best, sum((edges[j + 1] - edges[j]) * min(T, s[edges[j + 1] - 1] + halo) + c for j in range(m)))
    assert got == best


def test_vocpack_tile_tables_cover_each_utterance_exactly():
    """hip.VocPack (the packed vocoder's work tables): per (rate, tile rows) every utterance's rows [0, L*rate) are
    covered by consecutive tiles of its own (t0 = 0, BM, 2BM, ...; never straddling two utterances), row offsets are
    the packed prefix sums, and the whole set lives in one buffer (one host-to-device copy)."""
    import numpy as np
    import torch

    from speakingstyle_amd.ops.hip import VocPack

    lens = [300, 41, 0, 170, 1, 90]
    geoms = [(1, 256), (64, 118), (256, 408), (64, 118)]  # duplicate key: built once
    vp = VocPack(lens, torch.device("cpu"), geoms)
    assert vp.R == sum(lens) and vp.cu.tolist() == [0, 300, 341, 341, 511, 512, 602]
    for rate, bm in geoms:
        tab, n = vp.tiles(rate, bm)
        t = tab.view(n, 4).numpy()
        assert n == sum(-(-L * rate // bm) for L in lens)
        for u, L in enumerate(lens):
            mine = t[t[:, 3] == u]
            assert len(mine) == -(-L * rate // bm)
            if L:
                assert (mine[:, 0] == vp.cu_host[u] * rate).all() and (mine[:, 1] == L * rate).all()
                assert mine[:, 2].tolist() == list(range(0, L * rate, bm))
        assert np.all(np.diff(t[:, 3]) >= 0)  # utterance-major
