"""Tracing / profiling hooks.

The reference disables SageMaker Debugger/Profiler and relies on CloudWatch graphs,
``NCCL_DEBUG=INFO`` and ``KMP_SETTINGS`` (NBHVD:90, PS:411).  Here:

* ``range(name)``  — roctx range (ROCm's NVTX-compatible markers, shown by
  ``rocprofv3 --marker-trace``) around a phase; a no-op on CPU;
* ``StepWindow``   — marks steps [a, b) (flag ``--profile_steps a:b`` via env
  ``HIPFM_PROFILE_STEPS``) so a kernel trace can be cut to the steady state;
* per-step host timers live in ``utils.logging.StepTimer`` and are written to metrics.jsonl;
* kernel-level evidence: ``scripts/profile.sh`` (``rocprofv3 --kernel-trace --stats``) and
  ``tools/prof_summary.py`` (-> profiles/*.md).
"""
from __future__ import annotations

import contextlib
import os

import torch
from ..utils.knobs import knob


def _nvtx():
    try:
        if torch.cuda.is_available():
            return torch.cuda.nvtx
    except Exception:  # noqa: BLE001
        pass
    return None


@contextlib.contextmanager
def range(name: str):  # noqa: A001  (mirrors nvtx.range)
    nv = _nvtx()
    if nv is None:
        yield
        return
    nv.range_push(name)
    try:
        yield
    finally:
        nv.range_pop()


class StepWindow:
    """Emit a marker range around the steps of a window (e.g. ``HIPFM_PROFILE_STEPS=100:120``)."""

    def __init__(self, spec: str = None):
        spec = spec if spec is not None else knob("HIPFM_PROFILE_STEPS")
        self.a = self.b = -1
        if spec and ":" in spec:
            a, b = spec.split(":", 1)
            self.a, self.b = int(a), int(b)
        self._open = False

    def step(self, step: int):
        nv = _nvtx()
        if nv is None or self.a < 0:
            return
        if step == self.a and not self._open:
            nv.range_push(f"hipfm_steps_{self.a}_{self.b}")
            self._open = True
        elif step == self.b and self._open:
            nv.range_pop()
            self._open = False
