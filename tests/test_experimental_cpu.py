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
    assert experimental.get("ln_fuse") is False
    assert experimental.get("hifigan_hip_train") is True


def test_env_parsing_and_validation(monkeypatch):
    monkeypatch.setenv("SSAMD_EXPERIMENTAL", "wgrad_first=1, ln_fuse=true")
    assert experimental.get("wgrad_first") == "1" and experimental.get("ln_fuse") is True
    assert experimental.overridden() == {"wgrad_first": "1", "ln_fuse": True}
    for bad in ("wgrad_frist=1", "wgrad_first=off", "ln_fuse=maybe", "wgrad_cu_frac=1.5", "novalue"):
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
