"""Native host library (csrc/host_collate.cpp) == numpy reference padding."""
import numpy as np
import pytest

from speakingstyle_amd.utils import native, tools


def _np_pad(arrs, max_rows=None):
    max_rows = max_rows or max(a.shape[0] for a in arrs)
    out = np.zeros((len(arrs), max_rows) + arrs[0].shape[1:], dtype=arrs[0].dtype)
    for i, a in enumerate(arrs):
        out[i, : a.shape[0]] = a
    return out


@pytest.fixture(scope="module", autouse=True)
def _built():
    if native.lib() is None:
        import subprocess
        import sys

        subprocess.run([sys.executable, "csrc/build.py"], check=True)
        native._tried = False
    assert native.lib() is not None, "libssamd_host.so must build with g++"


@pytest.mark.parametrize("dtype,tail", [(np.float32, (80,)), (np.int64, ()), (np.float32, ())])
def test_pad_rows_matches_numpy(dtype, tail):
    rng = np.random.default_rng(0)
    arrs = [rng.standard_normal((int(n),) + tail).astype(dtype) for n in rng.integers(0, 900, 300)]
    out = native.pad_rows(arrs)
    np.testing.assert_array_equal(out, _np_pad(arrs))
    out2 = native.pad_rows(arrs, max_rows=1000)
    np.testing.assert_array_equal(out2, _np_pad(arrs, 1000))


def test_pad_rows_too_long_raises():
    with pytest.raises(ValueError):
        native.pad_rows([np.zeros((5, 3), np.float32)], max_rows=4)


@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_host_runtime_under_sanitizers(san):
    """csrc/host_collate.cpp under ASan+UBSan / TSan (host-only sanitizers; the GPU
    sanitizers are unavailable on the target pool): the self-test must run clean."""
    import os
    import shutil
    import subprocess
    import sys

    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "csrc"))
    import build

    exe = build.build_sanitized()[san]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "selftest_host_collate ok" in r.stdout


def test_tools_pad_uses_native():
    arrs = [np.arange(n, dtype=np.int64) + 1 for n in (3, 7, 1)]
    np.testing.assert_array_equal(tools.pad_1d(arrs), _np_pad(arrs))
    mels = [np.ones((n, 4), np.float32) for n in (2, 5)]
    np.testing.assert_array_equal(tools.pad_2d(mels), _np_pad(mels))
