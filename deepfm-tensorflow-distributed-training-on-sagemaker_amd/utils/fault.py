"""Failure detection and fault injection.

The reference has no elastic recovery: Horovod's stall inspector warns after 60 s and any rank
failure shuts the job down (DOC p.21-22); spot checkpoints are commented out (NBPS:100-101).
Here:

* ``Watchdog`` — a heartbeat thread per rank: if no training step completes within
  ``timeout_s`` (a stalled collective, a hung kernel, a dead peer) it prints every thread's stack
  with the rank and the last completed step, then terminates the process so the launcher's
  fail-fast logic stops the job instead of hanging the GPUs;
* ``maybe_inject_fault(step, rank)`` — ``HIPFM_FAULT_STEP=s [HIPFM_FAULT_RANK=r]
  [HIPFM_FAULT_MODE=exit|raise]`` kills rank r at step s, to test that auto-resume from the last
  checkpoint reproduces the run (tests/test_fault.py).
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
from ..utils.knobs import knob


class Watchdog:
    def __init__(self, timeout_s: float = 900.0, rank: int = 0, exit_code: int = 86):
        self.timeout = float(timeout_s)
        self.rank = rank
        self.exit_code = exit_code
        self.last = time.time()
        self.step = -1
        self._stop = threading.Event()
        self._t = None

    def start(self):
        if self.timeout <= 0:
            return self
        self._t = threading.Thread(target=self._run, name="hipfm-watchdog", daemon=True)
        self._t.start()
        return self

    def beat(self, step: int):
        self.step = step
        self.last = time.time()

    def stop(self):
        self._stop.set()

    def _run(self):
        while not self._stop.wait(min(10.0, self.timeout / 4)):
            idle = time.time() - self.last
            if idle > self.timeout:
                sys.stderr.write(f"[hipfm watchdog] rank {self.rank}: no step completed for {idle:.0f}s "
                                 f"(last step {self.step}); dumping stacks and exiting\n")
                faulthandler.dump_traceback(all_threads=True)
                sys.stderr.flush()
                os._exit(self.exit_code)


class InjectedFault(RuntimeError):
    pass


def maybe_inject_fault(step: int, rank: int, prev: int = None) -> None:
    """Fires when the fault step lies in (prev, step]: a multi-step graph run advances the step
    by up to ``graph_steps`` at once (``prev`` = the step before the run; default step - 1)."""
    s = knob("HIPFM_FAULT_STEP")
    if prev is None:
        prev = step - 1
    if not s or not (prev < int(s) <= step):
        return
    r = knob("HIPFM_FAULT_RANK")
    if r is not None and int(r) != rank:
        return
    if knob("HIPFM_FAULT_MODE") == "raise":
        raise InjectedFault(f"injected fault at step {step} on rank {rank}")
    sys.stderr.write(f"[hipfm] injected fault: rank {rank} exits at step {step}\n")
    sys.stderr.flush()
    os._exit(17)
