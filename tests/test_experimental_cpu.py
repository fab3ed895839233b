"""Experiment / diagnostic switches: one validated registry (speakingstyle_amd/experimental.py).
A plain run reaches only the defaults; a typo or an unparsable value raises instead of silently
selecting a path."""
import pytest

from speakingstyle_amd import experimental


@pytest.fixture(autouse=True)
def _clean(monkeypatch):
    monkeypatch.delenv("SSAMD_EXPERIMENTAL", raising=False)
    experimental.reset_for_tests()
    yield
    experimental.reset_for_tests()


def test_defaults_are_production():
    assert experimental.overridden() == {}
    assert experimental.get("wgrad_first") == "auto"
    assert experimental.get("bn_fuse") is True
    assert experimental.get("hifigan_hip_train") is True


def test_env_parsing_and_validation(monkeypatch):
    monkeypatch.setenv("SSAMD_EXPERIMENTAL", "wgrad_first=1, bn_fuse=false")
    assert experimental.get("wgrad_first") == "1" and experimental.get("bn_fuse") is False
    assert experimental.overridden() == {"wgrad_first": "1", "bn_fuse": False}
    for bad in ("wgrad_frist=1", "wgrad_first=off", "bn_fuse=maybe", "wgrad_cu_frac=1.5", "novalue"):
        experimental.reset_for_tests()
        monkeypatch.setenv("SSAMD_EXPERIMENTAL", bad)
        with pytest.raises((KeyError, ValueError)):
            experimental.get("wgrad_first")


def test_config_block_env_precedence(monkeypatch):
    monkeypatch.setenv("SSAMD_EXPERIMENTAL", "wgrad_first=0")
    experimental.configure({"wgrad_first": "1", "wgrad_cu_frac": 0.5})
    assert experimental.get("wgrad_first") == "0" and experimental.get("wgrad_cu_frac") == 0.5
    with pytest.raises(KeyError):
        experimental.configure({"not_a_switch": 1})


def test_configure_replaces_previous_block_and_applies_kernel_switches(monkeypatch):
    calls = []

    class FakeLib:
        def ssamd_gemm_set_stg(self, v):
            calls.append(("stg", v))

        def ssamd_gemm_set_mask_pre(self, v):
            calls.append(("mask_pre", v))

    monkeypatch.setattr(experimental, "_lib_ref", [None])
    experimental.apply_kernel_switches(FakeLib())
    assert ("stg", 1) in calls and ("mask_pre", 1) in calls
    calls.clear()
    experimental.configure({"gemm_stg": "0"})
    assert experimental.get("gemm_stg") is False and ("stg", 0) in calls
    calls.clear()
    experimental.configure({})  # a second Trainer without the block: back to the default
    assert experimental.get("gemm_stg") is True and ("stg", 1) in calls
    calls.clear()
    with experimental.overrides(gemm_mask_pre=False):
        assert ("mask_pre", 0) in calls
    assert calls[-1] == ("mask_pre", 1) or ("mask_pre", 1) in calls[-2:]


def test_side_wgrad_policy_threshold():
    """Automatic side-stream weight gradients (experimental.side_wgrad): on for steps with >= the frame
    threshold, off below it, forced by 0 / 1, undecided (None) without host lengths."""
    import numpy as np

    from speakingstyle_amd import experimental
    from speakingstyle_amd.train.trainer import side_wgrad_wanted

    small = np.full(16, 560)        # LibriTTS batch 16: ~9k frames
    big = np.full(200, 570)         # LJSpeech batch 200: ~114k frames
    capped = np.full(30, 5000)      # lengths past max_seq_len count as max_seq_len
    with experimental.overrides(side_wgrad="auto", side_wgrad_min_frames=20000):
        assert side_wgrad_wanted(small, 1000) is False
        assert side_wgrad_wanted(big, 1000) is True
        assert side_wgrad_wanted(capped, 600) is False   # 30 * 600 = 18000
        assert side_wgrad_wanted(None, 1000) is None
    with experimental.overrides(side_wgrad="1"):
        assert side_wgrad_wanted(small, 1000) is True
    with experimental.overrides(side_wgrad="0"):
        assert side_wgrad_wanted(big, 1000) is False
