"""Packed decoder (valid frames only, ``ops/packing.py``) == padded decoder.

Training forward + backward with and without the host lengths that enable packing
must give the same outputs (every element of mel / postnet, incl. padded frames) and
the same parameter gradients (fp32 CPU reference ops; dropout off)."""
import copy

import numpy as np
import pytest
import torch


def _cfg(name):
    from speakingstyle_amd.config import load_named

    pp, mc, tc = load_named(name)
    mc["transformer"].update(encoder_layer=1, decoder_layer=2, encoder_dropout=0.0, decoder_dropout=0.0)
    mc["variance_predictor"]["dropout"] = 0.0
    if mc.get("reference_encoder"):
        mc["reference_encoder"].update(encoder_layer=1, conv_layer=1, dropout=0.0)
    return pp, mc, tc


@pytest.mark.parametrize("name", ["LJSpeech", "BC2013"])
def test_packed_decoder_matches_padded(name):
    from speakingstyle_amd.data.synthetic import SyntheticBatches
    from speakingstyle_amd.models.fastspeech2 import FastSpeech2
    from speakingstyle_amd.models.loss import FastSpeech2Loss

    pp, mc, tc = _cfg(name)
    torch.manual_seed(0)
    m1 = FastSpeech2(pp, mc)
    m1.postnet.dropout = 0.0
    m2 = copy.deepcopy(m1)
    m1.train()
    m2.train()
    b = SyntheticBatches(3, seed=4, phone_counts=[12, 30, 7]).make_batch()
    assert getattr(b[7], "host_lengths", None) is not None
    lossf = FastSpeech2Loss(pp, tc)
    calls = []
    orig = m1.decoder.forward_packed
    m1.decoder.forward_packed = lambda *a, **k: calls.append(1) or orig(*a, **k)
    out_p = m1(*b[2:])  # host lengths attached -> packed decoder
    assert calls, "packed decoder path not taken"
    b_nohost = list(b)
    b_nohost[7] = b[7].clone()  # no host_lengths attribute -> padded decoder
    out_d = m2(*b_nohost[2:])
    for i in (0, 1, 9):
        torch.testing.assert_close(out_p[i], out_d[i], rtol=1e-5, atol=1e-5)
    lp = lossf(b, out_p, m1.film_scalars())[0]
    ld = lossf(b, out_d, m2.film_scalars())[0]
    torch.testing.assert_close(lp, ld, rtol=1e-5, atol=1e-6)
    lp.backward()
    ld.backward()
    g2 = dict(m2.named_parameters())
    for n, p in m1.named_parameters():
        if p.grad is None:
            assert g2[n].grad is None or g2[n].grad.abs().max() == 0, n
            continue
        torch.testing.assert_close(p.grad, g2[n].grad, rtol=1e-4, atol=1e-6, msg=n)


def test_pack_info_cpu():
    from speakingstyle_amd.ops.packing import PackInfo, pack, unpack

    lens = torch.tensor([3, 5, 1])
    pk = PackInfo.build(lens, 4, 3 + 4 + 1)
    assert pk.cu.tolist() == [0, 3, 7, 8]
    assert pk.rinfo[:, 0].tolist() == [0, 1, 2, 0, 1, 2, 3, 0]
    assert pk.rinfo[:, 1].tolist() == [3, 3, 3, 4, 4, 4, 4, 1]
    x = torch.randn(3, 4, 2)
    y = unpack(pack(x, pk), pk, fill=torch.tensor([7.0, 8.0]))
    mask = torch.arange(4)[None] < lens.clamp(max=4)[:, None]
    torch.testing.assert_close(y[mask], x[mask])
    assert (y[~mask] == torch.tensor([7.0, 8.0])).all()


def test_positional_rows_cast_cache_and_idcache():
    """The per-dtype positional table copy is made once and sliced (no cast per forward); IdCache is keyed by
    tensor identity (a WeakKeyDictionary would compare tensor keys elementwise) and follows in-place updates."""
    import torch

    from speakingstyle_amd.models.fastspeech2 import positional_rows
    from speakingstyle_amd.ops import IdCache

    p = torch.nn.Parameter(torch.randn(1, 10, 4), requires_grad=False)
    a = positional_rows(p, 5, 4, "cpu", torch.bfloat16)
    b = positional_rows(p, 3, 4, "cpu", torch.bfloat16)
    assert a.dtype == torch.bfloat16 and a.data_ptr() == b.data_ptr()
    assert torch.equal(a, p[0, :5].to(torch.bfloat16))
    with torch.no_grad():
        p.add_(1.0)  # version bump -> fresh copy
    c = positional_rows(p, 5, 4, "cpu", torch.bfloat16)
    assert torch.equal(c, p[0, :5].to(torch.bfloat16))
    cache = IdCache()
    t1, t2 = torch.zeros(3), torch.zeros(3)
    cache.put(t1, "one")
    assert cache.get(t1) == "one" and cache.get(t2) is None


def test_postnet_folded_batchnorm_packed_matches_eval():
    """PostNet.forward_packed folds eval BatchNorm into the convs: same output as the eval forward on the padded
    batch (valid frames), and the fold follows in-place updates of the running statistics."""
    from speakingstyle_amd.models.layers import PostNet
    from speakingstyle_amd.ops.packing import PackInfo, pack, unpack

    torch.manual_seed(0)
    pn = PostNet(n_mel_channels=16, emb=32, k=5, n=5)
    for _, bn in pn.convolutions:
        bn.running_mean.uniform_(-0.5, 0.5)
        bn.running_var.uniform_(0.5, 2.0)
        bn.weight.data.uniform_(0.5, 1.5)
        bn.bias.data.uniform_(-0.2, 0.2)
    pn.eval()
    lens = torch.tensor([9, 4, 13])
    L = 13
    x = torch.randn(3, L, 16)
    mask = torch.arange(L)[None] < lens[:, None]
    pk = PackInfo.build(lens, L, int(lens.sum()))
    for _ in range(2):
        with torch.no_grad():
            ref = torch.stack([pn(x[b:b + 1, : int(lens[b])]).squeeze(0).new_zeros(L, 16).index_copy(
                0, torch.arange(int(lens[b])), pn(x[b:b + 1, : int(lens[b])]).squeeze(0)) for b in range(3)])
            got = unpack(pn.forward_packed(pack(x, pk), pk), pk)
        assert got.dtype == torch.float32
        torch.testing.assert_close(got[mask], ref[mask], rtol=1e-5, atol=1e-5)
        pn.convolutions[2][1].running_mean.add_(0.3)  # in place: the cached fold must be rebuilt
    assert "_fold" not in pn.state_dict()
