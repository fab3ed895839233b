"""FiLM reference encoder on valid frames only (reference ``model/modules.py:307-406``): the conv stack
runs on rows packed with a halo of (k-1)/2*(layers-1) pad frames per sequence, because the reference
zeroes pad frames only after the whole stack (``modules.py:366-371``) -- the last valid frames of
layer 3 depend on layer-1/2 values inside the padding.  fp32 CPU: the halo-packed path must equal the
padded one; without the halo it must not (the test would be vacuous otherwise)."""
import copy

import torch


def _enc():
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.models.style import ReferenceEncoder

    pp, mc, _ = load_named("BC2013")
    mc["reference_encoder"].update(dropout=0.0, conv_filter_size=64, encoder_hidden=32, encoder_head=2,
                                   encoder_layer=1)
    torch.manual_seed(5)
    return ReferenceEncoder(pp, mc).eval()


def _batch():
    lens_h = [37, 12, 50, 3]
    B, M = len(lens_h), max(lens_h) + 4
    torch.manual_seed(6)
    mel = torch.randn(B, M, 80)
    for i, n in enumerate(lens_h):
        mel[i, n:] = 0.0
    return mel, torch.tensor(lens_h), lens_h


def test_halo_packed_conv_stack_equals_padded():
    e = _enc()
    mel, lens, host = _batch()
    assert e.halo() == 2
    with torch.no_grad():
        g_pad, b_pad = e(mel, lens)
        g_pk, b_pk = e._forward_packed(mel, lens, host)
    torch.testing.assert_close(g_pk, g_pad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(b_pk, b_pad, rtol=1e-4, atol=1e-5)


def test_without_halo_differs():
    e = _enc()
    e2 = copy.deepcopy(e)
    e2.halo = lambda: 0
    mel, lens, host = _batch()
    with torch.no_grad():
        g_pad, _ = e(mel, lens)
        g0, _ = e2._forward_packed(mel, lens, host)
    assert not torch.allclose(g0, g_pad, rtol=1e-4, atol=1e-5)
