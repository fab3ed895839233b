"""Per-phase step timing (SURVEY §5 tracing): host time (perf_counter, no synchronisation) and
device time (HIP events on the current stream) of the phases of a training step.

Used by ``Trainer`` when enabled (``mi355x.phase_timing: true`` in train.yaml, ``bench.py
--phase-times`` or the ``phase_timing`` experiment switch): the training loop logs ``Perf/phase_*_ms``
scalars at every log step and the bench prints a per-phase table.  Disabled it costs one
attribute test per phase.

Device times come from events recorded at phase boundaries on the compute stream, read back
lazily (``summary()`` synchronises once), so enabling the timer does not add host-device
synchronisation inside the step.
"""
from __future__ import annotations

import time
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import torch


class PhaseTimer:
    def __init__(self, enabled: bool = False):
        self.enabled = enabled
        self._host: Dict[str, float] = OrderedDict()
        self._count: Dict[str, int] = OrderedDict()
        self._events: List[Tuple[str, object, object]] = []
        self._cur: Optional[Tuple[str, float, object]] = None

    def phase(self, name: str):
        """End the current phase (if any) and start ``name``."""
        if not self.enabled:
            return
        now = time.perf_counter()
        ev = None
        if torch.cuda.is_available():
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
        if self._cur is not None:
            pname, t0, e0 = self._cur
            self._host[pname] = self._host.get(pname, 0.0) + (now - t0)
            self._count[pname] = self._count.get(pname, 0) + 1
            if e0 is not None and ev is not None:
                self._events.append((pname, e0, ev))
        self._cur = (name, now, ev)

    def stop(self):
        if self.enabled and self._cur is not None:
            self.phase("__end__")
            self._cur = None

    def summary(self, reset: bool = True) -> Dict[str, Dict[str, float]]:
        """{phase: {"host_ms": mean host ms, "device_ms": mean device ms, "n": count}}."""
        if not self.enabled:
            return {}
        dev: Dict[str, float] = {}
        if self._events:
            self._events[-1][2].synchronize()
            for name, a, b in self._events:
                dev[name] = dev.get(name, 0.0) + a.elapsed_time(b)
        out = OrderedDict()
        for name, tot in self._host.items():
            n = max(1, self._count.get(name, 1))
            out[name] = {"host_ms": 1000.0 * tot / n, "device_ms": dev.get(name, 0.0) / n if dev else 0.0, "n": n}
        if reset:
            self._host.clear()
            self._count.clear()
            self._events.clear()
        return out
