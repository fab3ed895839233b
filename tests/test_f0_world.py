"""Native DIO + StoneMask F0 (csrc/host_f0.cpp) -- the reference's pyworld pair
(preprocessor/preprocessor.py:182-187).  pyworld is not installable here, so parity
with it is unpinned; these tests check the estimator against signals whose F0 is
known by construction (steady harmonic tones, a glide, silence) and the pyworld
call contract (frame grid, 0 = unvoiced)."""
import numpy as np
import pytest

from speakingstyle_amd.data.preprocess import extract_f0
from speakingstyle_amd.utils import native

FS, HOP = 22050, 256
FP = HOP / FS * 1000.0


@pytest.fixture(scope="module", autouse=True)
def _built():
    if native.lib() is None:
        import subprocess
        import sys

        subprocess.run([sys.executable, "csrc/build.py"], check=True)
        native._tried = False
    assert native.lib() is not None


def _tone(f_of_t, dur=1.5, harmonics=5, seed=0):
    t = np.arange(int(FS * dur)) / FS
    f = np.broadcast_to(np.asarray(f_of_t(t), dtype=np.float64), t.shape)
    ph = 2 * np.pi * np.cumsum(f) / FS
    x = sum(np.sin(k * ph + 0.3 * k) / k for k in range(1, harmonics + 1)) * 0.3
    x = x + 1e-4 * np.random.default_rng(seed).standard_normal(len(x))
    return x, t, f


def test_frame_grid_contract():
    x, _, _ = _tone(lambda t: 150.0, dur=1.0)
    f0, t = native.dio(x, FS, frame_period=FP)
    assert len(f0) == int(1000.0 * len(x) / FS / FP) + 1
    np.testing.assert_allclose(t, np.arange(len(f0)) * FP / 1000.0)
    assert f0.dtype == np.float64 and np.all(f0 >= 0)


@pytest.mark.parametrize("F", [85.0, 150.0, 230.0, 410.0])
def test_steady_tone(F):
    x, _, _ = _tone(lambda t: F)
    f0, t = native.dio(x, FS, frame_period=FP)
    v = f0 > 0
    inner = (t > 0.1) & (t < t[-1] - 0.1)  # away from the abrupt signal edges
    assert v[inner].all()
    assert np.max(np.abs(f0[v & inner] - F) / F) < 0.01
    assert np.max(np.abs(f0[v] - F) / F) < 0.1
    f1 = native.stonemask(x, f0, t, FS)
    assert np.array_equal(f1 > 0, v)
    assert np.median(np.abs(f1[v] - F) / F) < 0.003


def test_glide_and_silence():
    x, tt, f = _tone(lambda t: np.where(t < 1.0, 140.0, 140.0 + 80.0 * (t - 1.0)), dur=2.0)
    x[tt < 0.4] = 1e-5 * np.random.default_rng(1).standard_normal(int((tt < 0.4).sum()))
    f0, t = native.dio(x, FS, frame_period=FP)
    f1 = native.stonemask(x, f0, t, FS)
    ref = np.interp(t, tt, f)
    v = f1 > 0
    assert not v[t < 0.35].any()  # silence stays unvoiced
    assert v[(t > 0.5) & (t < 1.9)].all()
    inner = v & (t > 0.5) & (t < 1.9)
    assert np.max(np.abs(f1[inner] - ref[inner]) / ref[inner]) < 0.02
    assert np.median(np.abs(f1[v] - ref[v]) / ref[v]) < 0.005


def test_stonemask_corrects_a_biased_estimate():
    x, _, _ = _tone(lambda t: 137.3, dur=1.0)
    t = np.arange(20, 60) * FP / 1000.0
    for guess in (137.3 * 1.05, 137.3 * 0.96):
        f1 = native.stonemask(x, np.full(len(t), guess), t, FS)
        assert np.median(np.abs(f1 - 137.3)) < 0.01 * 137.3
    # unvoiced frames stay unvoiced
    assert np.all(native.stonemask(x, np.zeros(len(t)), t, FS) == 0)


def test_bad_arguments_raise():
    with pytest.raises(ValueError):
        native.dio(np.zeros(100), FS, f0_floor=500.0, f0_ceil=100.0)
    with pytest.raises(ValueError):
        native.stonemask(np.zeros(100), np.zeros(3), np.zeros(4), FS)


def test_preprocessor_extractor_choice():
    x, _, _ = _tone(lambda t: 180.0, dur=1.0)
    d = extract_f0(x.astype(np.float32), FS, HOP, "dio")
    y = extract_f0(x.astype(np.float32), FS, HOP, "yin")
    vd, vy = d > 0, y > 0
    assert abs(np.median(d[vd]) - 180.0) < 1.0 and abs(np.median(y[vy]) - 180.0) < 2.0
    with pytest.raises(ValueError):
        extract_f0(x, FS, HOP, "crepe")
