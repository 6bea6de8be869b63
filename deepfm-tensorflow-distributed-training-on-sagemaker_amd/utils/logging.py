"""Logging / metrics: TF-Estimator-style console lines + structured JSONL.

The reference relies on Estimator's default hooks (``loss = ..., step = ...`` and
``global_step/sec`` every 100 steps) plus prints; ``log_steps`` was unused (Q5).  Here
``log_steps`` drives both the console line and a ``metrics.jsonl`` record with loss,
samples/s (rank and whole job), step time and comm bytes, for the benchmark harness.
"""
from __future__ import annotations

import json
import os
import sys
import time
from typing import Optional


class MetricsLogger:
    def __init__(self, path: Optional[str], rank: int = 0, echo: bool = True):
        self.rank = rank
        self.echo = echo and rank == 0
        self.f = None
        if path and rank == 0:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            self.f = open(path, "a", buffering=1)

    def info(self, msg: str):
        if self.echo:
            print(f"INFO:hipfm:{msg}", flush=True)

    def log(self, kind: str, **kv):
        rec = {"kind": kind, "time": time.time(), **kv}
        if self.f is not None:
            self.f.write(json.dumps(rec) + "\n")
        return rec

    def close(self):
        if self.f is not None:
            self.f.close()
            self.f = None


class StepTimer:
    """Wall-clock per-phase timers (host side): data wait, step enqueue, sync."""

    def __init__(self):
        self.t = {}
        self.n = {}

    def add(self, key: str, dt: float):
        self.t[key] = self.t.get(key, 0.0) + dt
        self.n[key] = self.n.get(key, 0) + 1

    def summary(self, reset: bool = True) -> dict:
        out = {k: self.t[k] / max(1, self.n[k]) * 1e3 for k in self.t}
        if reset:
            self.t.clear()
            self.n.clear()
        return {f"{k}_ms": round(v, 4) for k, v in out.items()}
