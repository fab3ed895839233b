import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device and the built kernel library")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def reference_modules():
    """Import the read-only reference package as a numerical oracle (stubbing the
    unavailable `unidecode` / `inflect` text deps, which the model code never uses)."""
    if not os.path.isdir(REFERENCE):
        pytest.skip("reference tree not mounted")
    import types

    sys.modules.setdefault("unidecode", types.SimpleNamespace(unidecode=lambda s: s))
    sys.modules.setdefault("inflect", types.SimpleNamespace(engine=lambda: types.SimpleNamespace()))
    saved = {k: sys.modules.pop(k) for k in list(sys.modules) if k.split(".")[0] in ("utils", "model", "transformer", "text", "audio", "hifigan")}
    sys.path.insert(0, REFERENCE)
    try:
        import model as ref_model  # noqa
        import transformer as ref_transformer  # noqa
        import hifigan as ref_hifigan  # noqa
        mods = types.SimpleNamespace(model=ref_model, transformer=ref_transformer, hifigan=ref_hifigan,
                                     modules=sys.modules["model.modules"], loss=sys.modules["model.loss"],
                                     optimizer=sys.modules["model.optimizer"], hifigan_models=sys.modules["hifigan.models"])
        yield mods
    finally:
        sys.path.remove(REFERENCE)
        for k in list(sys.modules):
            if k.split(".")[0] in ("utils", "model", "transformer", "text", "audio", "hifigan"):
                sys.modules.pop(k)
        sys.modules.update(saved)
