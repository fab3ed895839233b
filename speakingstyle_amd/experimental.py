"""The one place experiment / diagnostic switches are read.

A plain run -- no ``SSAMD_EXPERIMENTAL`` in the environment, no ``mi355x.experimental`` block in
train.yaml -- takes the measured production path of every switch below and nothing else.  Setting
one is an explicit, validated act: unknown names and values that do not parse raise, instead of
silently selecting a default (or an untested path).

    SSAMD_EXPERIMENTAL="wgrad_first=1,gemm_stg=0" python bench.py ...

``mi355x.experimental: {wgrad_first: "0"}`` in train.yaml does the same for ``train.py`` (the trainer
calls ``configure`` with it; the environment wins on conflicts).

Three switches select kernel-library variants (``KERNEL_SWITCHES``: ``gemm_stg``, ``gemm_mask_pre``,
``gemm_bnh_stg``).
``apply_kernel_switches()`` pushes their current values into the library; it runs when the library
is first loaded (``ops/hip.py:lib``), after ``configure()`` and on entry to / exit from ``overrides``,
so every path -- training, synthesis, kernel tests -- sees the same values.  The library's other
``ssamd_*_set_*`` setters (``ops/hip.py:_SIGS``) are not framework switches: only the GPU tests (to
cover every variant against fp32) and the ``tools/exp_*.py`` experiments call them.

Infrastructure variables that are not experiments stay plain environment variables and are
documented where they are read: ``SSAMD_BACKEND`` (hip / reference op backend), ``SSAMD_KERNEL_LIB``
(A/B of a second kernel-library build), ``SSAMD_ALLOW_TORCH_FALLBACK``, ``SSAMD_DIST_BACKEND``,
``SSAMD_DIST_TIMEOUT_S``.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

# name -> (default, parser, help)
_BOOL = {"0": False, "1": True, "false": False, "true": True, "off": False, "on": True}


def _bool(v):
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s not in _BOOL:
        raise ValueError(f"expected 0/1, got {v!r}")
    return _BOOL[s]


def _tristate(v):
    s = str(v).strip().lower()
    if s not in ("0", "1", "auto"):
        raise ValueError(f"expected 0 / 1 / auto, got {v!r}")
    return s


def _pos_int(v):
    i = int(v)
    if i <= 0:
        raise ValueError(f"expected a positive integer, got {v!r}")
    return i


def _frac(v):
    f = float(v)
    if not 0.0 < f <= 1.0:
        raise ValueError(f"expected a fraction in (0, 1], got {v!r}")
    return f


KNOBS: Dict[str, tuple] = {
    # -- compute-path experiments (A/B of measured production choices)
    "wgrad_first": ("auto", _tristate,
                    "issue a layer's weight gradient (side stream) before its data gradient: 0 never, 1 always, "
                    "auto when the data-gradient GEMMs have fewer row tiles than wgrad_first_waves x CUs"),
    "wgrad_first_waves": (1.25, float, "auto threshold of wgrad_first, in waves of 256-row tiles per CU"),
    "side_wgrad": ("auto", _tristate,
                   "weight gradients (and LayerNorm weight reductions) on the side stream: 0 never, 1 always, auto "
                   "when the step has >= side_wgrad_min_frames valid mel frames (a small step is host-bound: the "
                   "side stream's event record / wait per launch costs more host time than its overlap saves)"),
    "side_wgrad_min_frames": (20000, _pos_int, "auto threshold of side_wgrad (valid mel frames per step and GPU)"),
    "wgrad_cu_frac": (0.75, _frac, "fraction of the CUs the side-stream weight-gradient split plan is sized for"),
    "wgrad_cus_all": (True, _bool, "apply the reduced weight-gradient CU plan to every stream (0: side stream "
                                   "only -- main-stream weight gradients then reduce in a different order)"),
    "gemm_stg": (True, _bool, "staggered 8-phase main loop of the 256x256 GEMM for K >= 512 (+0.7 % LJSpeech)"),
    "gemm_mask_pre": (True, _bool, "ReLU-mask data gradient with its mask bytes prefetched before the main loop"),
    "gemm_bnh_stg": (True, _bool, "PostNet BatchNorm-backward-head data gradient on the staggered main loop"),
    "gemm_ring_maxk": (0, int, "GEMMs with K <= this on the 256x128 ring kernel at any tile count (0: only <= 64 "
                               "big tiles)"),
    "gemm_ring_maxn": (256, int, "widest N of gemm_ring_maxk"),
    "gemm_skinny": (True, _bool, "small-M GEMMs on the skinny 16 x 16-tile kernel"),
    "gemm_skinny_maxm": (1024, int, "row limit of gemm_skinny"),
    "bn_fuse": (True, _bool, "PostNet BatchNorm backward started in the data-gradient GEMM's epilogue"),
    "defer_release": (False, _bool, "hand the side-stream weight-gradient inputs back to the trainer, freed "
                                    "during the next forward (holds a step's activations into it)"),
    "hifigan_hip_train": (True, _bool, "HiFi-GAN generator training on the HIP implicit-GEMM convs"),
    # -- diagnostics (instrumentation only; no effect on what is computed)
    "phase_timing": (False, _bool, "per-phase host/device step times (Perf/phase_* scalars)"),
    "host_tail": (False, _bool, "host timestamps of the step tail (backward return .. optimizer launch)"),
    "host_lead": (False, _bool, "bench: how far the host enqueue runs ahead of the GPU per step"),
    "tail_events": (False, _bool, "bench: device-side event timing of the step tail (joined backward .. Adam)"),
    "fail_rank": (None, int, "fault injection: this rank raises in its second timed bench step"),
}

# switch -> kernel-library setter it drives (applied by apply_kernel_switches)
KERNEL_SWITCHES = {"gemm_stg": "ssamd_gemm_set_stg", "gemm_mask_pre": "ssamd_gemm_set_mask_pre",
                   "gemm_bnh_stg": "ssamd_gemm_set_bnh_stg", "gemm_ring_maxk": "ssamd_gemm_set_ring_maxk",
                   "gemm_ring_maxn": "ssamd_gemm_set_ring_maxn", "gemm_skinny": "ssamd_gemm_set_skinny",
                   "gemm_skinny_maxm": "ssamd_gemm_set_skinny_maxm"}

_values: Dict[str, Any] = {}
_parsed = [False]
_lib_ref = [None]  # the loaded kernel library (set by ops/hip.py when it loads it)
_from_config = set()  # names the last configure() set (replaced by the next one)


def _parse_env() -> Dict[str, Any]:
    raw = os.environ.get("SSAMD_EXPERIMENTAL", "").strip()
    out = {}
    if not raw:
        return out
    for item in raw.split(","):
        item = item.strip()
        if not item:
            continue
        if "=" not in item:
            raise ValueError(f"SSAMD_EXPERIMENTAL: '{item}' is not name=value")
        k, v = (x.strip() for x in item.split("=", 1))
        out[k] = v
    return out


def _set(name: str, value, source: str):
    if name not in KNOBS:
        raise KeyError(f"{source}: unknown experimental switch '{name}' (known: {', '.join(sorted(KNOBS))})")
    try:
        _values[name] = KNOBS[name][1](value)
    except (TypeError, ValueError) as e:
        raise ValueError(f"{source}: {name}={value!r}: {e}") from None


def _ensure():
    if not _parsed[0]:
        for k, v in _parse_env().items():
            _set(k, v, "SSAMD_EXPERIMENTAL")
        _parsed[0] = True


def set_value(name: str, value, source: str = "set_value"):
    """Set a switch for the rest of the process (a CLI flag's programmatic equivalent); later ``configure``
    calls do not reset it (they replace only their own block's values)."""
    _ensure()
    _set(name, value, source)
    apply_kernel_switches()


def configure(block: Optional[dict]):
    """Apply a train.yaml ``mi355x.experimental`` block (the environment keeps precedence).  Replaces
    the values of an earlier ``configure`` call (a second Trainer in one process starts from the
    environment + its own block, not from the first one's)."""
    _ensure()
    for k in _from_config:
        _values.pop(k, None)
    _from_config.clear()
    env = _parse_env()
    for k, v in (block or {}).items():
        if k not in env:
            _set(k, v, "mi355x.experimental")
            _from_config.add(k)
    apply_kernel_switches()


def apply_kernel_switches(lib=None):
    """Push the current values of ``KERNEL_SWITCHES`` into the kernel library (no-op until it is loaded)."""
    if lib is not None:
        _lib_ref[0] = lib
    lib = _lib_ref[0]
    if lib is None:
        return
    for name, setter in KERNEL_SWITCHES.items():
        fn = getattr(lib, setter, None)
        if fn is not None:
            fn(int(get(name)))


def get(name: str):
    _ensure()
    if name not in KNOBS:
        raise KeyError(name)
    return _values.get(name, KNOBS[name][0])


def overridden() -> Dict[str, Any]:
    """Switches set away from their defaults (recorded in bench output / logs)."""
    _ensure()
    return {k: v for k, v in _values.items() if v != KNOBS[k][0]}


class overrides:
    """Context manager for tests / experiments in one process: ``with overrides(gemm_stg=False): ...``."""

    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        _ensure()
        self.saved = dict(_values)
        for k, v in self.kw.items():
            _set(k, v, "overrides")
        apply_kernel_switches()
        return self

    def __exit__(self, *a):
        _values.clear()
        _values.update(self.saved)
        apply_kernel_switches()


def reset_for_tests():
    _values.clear()
    _from_config.clear()
    _parsed[0] = False
    apply_kernel_switches()
