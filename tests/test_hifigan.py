"""HiFi-GAN: polyphase ConvTranspose == torch conv_transpose1d, channel-last inference path
== the NCL training forward, reference-key compatibility, discriminators + losses run."""
import pytest
import torch
import torch.nn.functional as F

from speakingstyle_amd.models import hifigan as H


@pytest.mark.parametrize("k,s,cin,cout,T", [(16, 8, 16, 8, 9), (4, 2, 8, 8, 13), (16, 8, 8, 4, 1), (7, 3, 4, 4, 5)])
def test_polyphase_conv_transpose(k, s, cin, cout, T):
    torch.manual_seed(0)
    x = torch.randn(2, T, cin)
    w = torch.randn(cin, cout, k)
    b = torch.randn(cout)
    pad = (k - s) // 2
    y = H.conv_transpose_polyphase(x, w, b, s, pad)
    yr = F.conv_transpose1d(x.transpose(1, 2), w, b, stride=s, padding=pad).transpose(1, 2)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("k,s,cin,cout,T", [(16, 8, 16, 8, 9), (4, 2, 8, 8, 13), (16, 8, 8, 4, 1), (8, 4, 8, 8, 6)])
def test_conv_transpose_as_3tap_conv(k, s, cin, cout, T):
    """The GPU upsampler form: one 3-tap conv with N = s*Cout whose output rows are the phases."""
    from speakingstyle_amd.ops import reference as R

    torch.manual_seed(0)
    x = torch.randn(2, T, cin)
    w = torch.randn(cin, cout, k)
    b = torch.randn(cout)
    pad = (k - s) // 2
    wu = H.convT_as_conv3(w, s, pad)
    assert wu is not None and wu.shape == (s * cout, cin, 3)
    y = R.conv1d(x, wu, b.repeat(s), 1, 1, None).reshape(2, T * s, cout)
    yr = F.conv_transpose1d(x.transpose(1, 2), w, b, stride=s, padding=pad).transpose(1, 2)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    assert H.convT_as_conv3(torch.randn(4, 4, 7), 3, 1) is None  # K != s + 2*pad: polyphase fallback


def _small_cfg():
    h = H.default_config()
    h.update(upsample_initial_channel=32, resblock_kernel_sizes=[3, 7], resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5]])
    return h


def test_infer_matches_forward():
    torch.manual_seed(1)
    g = H.Generator(_small_cfg()).eval().fold_weight_norm()
    mel = torch.randn(2, 80, 11)
    with torch.no_grad():
        a = g(mel).squeeze(1)
        b = g.infer(mel.transpose(1, 2).contiguous())
    assert a.shape == b.shape == (2, 11 * 256)
    torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


def test_reference_generator_keys(reference_modules):
    h = H.default_config()
    ours = H.Generator(h)
    ref = reference_modules.hifigan_models.Generator(h)
    assert set(ours.state_dict()) == set(ref.state_dict())
    ref.load_state_dict(ours.state_dict())
    mel = torch.randn(1, 80, 5)
    with torch.no_grad():
        torch.testing.assert_close(ours(mel), ref(mel), rtol=1e-4, atol=1e-5)


def test_discriminators_and_losses():
    torch.manual_seed(2)
    y = torch.randn(2, 1, 2048)
    y_hat = torch.randn(2, 1, 2048, requires_grad=True)
    mpd, msd = H.MultiPeriodDiscriminator(), H.MultiScaleDiscriminator()
    r, g, fr, fg = mpd(y, y_hat)
    r2, g2, fr2, fg2 = msd(y, y_hat)
    ld, _, _ = H.discriminator_loss(r + r2, g + g2)
    lg, _ = H.generator_loss(g + g2)
    lf = H.feature_loss(fr + fr2, fg + fg2)
    (lg + lf).backward()
    assert torch.isfinite(ld) and y_hat.grad is not None
