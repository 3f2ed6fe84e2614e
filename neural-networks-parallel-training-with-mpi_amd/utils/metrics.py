"""Structured metrics (JSON lines) and step timers.

The reference only prints two lines per epoch per rank (ref.py:152,224).  The framework keeps
those lines and adds rank-0 JSON-lines metrics (loss, epoch time, whole-job samples/s) and
device-side step timers based on HIP events (fwd/bwd/comm/update breakdown when requested).
"""
from __future__ import annotations

import json
import time
from typing import Optional

import torch


class MetricsWriter:
    def __init__(self, path: Optional[str]):
        self.path = path
        self.f = open(path, "a") if path else None

    def write(self, **kw):
        if self.f:
            kw.setdefault("ts", time.time())
            self.f.write(json.dumps(kw) + "\n")
            self.f.flush()

    def close(self):
        if self.f:
            self.f.close()
            self.f = None


class EventTimer:
    """Named HIP-event intervals on a stream; read once at the end (no per-step host sync)."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self.marks = []

    def mark(self, name: str, stream=None):
        if not self.enabled:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        self.marks.append((name, e))

    def intervals_ms(self):
        if not self.marks:
            return {}
        self.marks[-1][1].synchronize()
        out = {}
        for (n0, e0), (n1, e1) in zip(self.marks, self.marks[1:]):
            key = f"{n0}->{n1}"
            out[key] = out.get(key, 0.0) + e0.elapsed_time(e1)
        return out
