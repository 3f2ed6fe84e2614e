"""Failure detection: step watchdog + RCCL async-error polling.

In the reference, one rank raising while the others sit in ``recv``/``gather`` hangs the job
until an external timeout (measured, SURVEY.md §3.5 failure (b)).  Here a daemon thread
(1) polls the native RCCL communicator for asynchronous errors and (2) checks that the training
loop made progress within ``timeout_s``; on either failure it aborts the communicator (so peers
blocked in a collective error out instead of hanging) and terminates the process non-zero.
"""
from __future__ import annotations

import os
import sys
import threading
import time


ABORT_GRACE_S = 15.0


class Watchdog:
    def __init__(self, timeout_s: float, native_comm=None, poll_s: float = 1.0, on_fail=None):
        self.timeout_s = float(timeout_s)
        self.comm = native_comm
        self.poll_s = poll_s
        self.on_fail = on_fail or self._default_fail
        self._last = time.monotonic()
        self._stop = threading.Event()
        self.failed = None
        self._t = threading.Thread(target=self._run, name="nnmpi-watchdog", daemon=True)
        self._t.start()

    def kick(self):
        self._last = time.monotonic()

    def stop(self):
        self._stop.set()
        self._t.join(timeout=2 * self.poll_s)

    def _run(self):
        while not self._stop.wait(self.poll_s):
            if self.comm is not None:
                try:
                    err = self.comm.poll_error(True)
                except Exception as e:  # pragma: no cover
                    err = repr(e)
                if err:
                    self._fail(f"RCCL async error {err}")
                    return
            if time.monotonic() - self._last > self.timeout_s:
                self._fail(f"no training progress for {self.timeout_s:.0f}s")
                return

    def _fail(self, why: str):
        self.failed = why
        # a backstop first: if ncclCommAbort itself never returns (a peer's kernel that ignores
        # the abort flag), the process still ends, non-zero, ABORT_GRACE_S later
        backstop = threading.Timer(ABORT_GRACE_S, self._backstop, args=(why,))
        backstop.daemon = True
        backstop.start()
        if self.comm is not None:
            print(f"[nnmpi watchdog] rank {os.environ.get('RANK', '?')}: {why}; aborting the "
                  "RCCL communicator", file=sys.stderr, flush=True)
            try:
                self.comm.abort()
            except Exception:
                pass
        self.on_fail(why)
        # (the default handler never returns; a custom one that does has taken the failure over)
        backstop.cancel()

    @staticmethod
    def _backstop(why: str):
        print(f"[nnmpi watchdog] rank {os.environ.get('RANK', '?')}: abort did not return in "
              f"{ABORT_GRACE_S:.0f} s after '{why}'; exiting", file=sys.stderr, flush=True)
        os._exit(3)

    @staticmethod
    def _default_fail(why: str):
        print(f"[nnmpi watchdog] rank {os.environ.get('RANK', '?')}: {why}; aborting",
              file=sys.stderr, flush=True)
        os._exit(3)
