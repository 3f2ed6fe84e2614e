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
    """Named device-side intervals of a step (HIP events on the engine's stream; on the CPU
    path the ops are synchronous, so wall-clock marks).  Marks accumulate over steps and are
    read once at the end (no per-step host sync): ``summary_ms()`` gives the mean time per
    step of every consecutive phase pair, e.g. ``{"start->fwd": 0.031, "fwd->head": ...}``."""

    def __init__(self, device: str = "cuda"):
        self.cuda = device.startswith("cuda") and torch.cuda.is_available()
        self.marks = []
        self.steps = 0

    def mark(self, name: str, stream=None):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            self.marks.append((name, e))
        else:
            self.marks.append((name, time.perf_counter()))
        if name == "start":
            self.steps += 1

    def _elapsed_ms(self, a, b) -> float:
        return a.elapsed_time(b) if self.cuda else (b - a) * 1e3

    def intervals_ms(self):
        """Total ms per phase pair over all recorded steps (pairs that cross a step boundary,
        i.e. the host gap between steps, are skipped)."""
        if not self.marks:
            return {}
        if self.cuda:
            self.marks[-1][1].synchronize()
        out = {}
        for (n0, e0), (n1, e1) in zip(self.marks, self.marks[1:]):
            if n1 == "start":
                continue
            key = f"{n0}->{n1}"
            out[key] = out.get(key, 0.0) + self._elapsed_ms(e0, e1)
        return out

    def summary_ms(self):
        n = max(self.steps, 1)
        return {k: v / n for k, v in self.intervals_ms().items()}


def comm_volume(grad_numel: int, world: int, grad_dtype: str = "fp32", sharded: bool = False,
                shadow: bool = False) -> dict:
    """Bytes one rank moves per step for the gradient synchronisation (ring algorithms:
    all-reduce 2(P-1)/P * S, reduce-scatter and all-gather (P-1)/P * S each).  ZeRO-1 = fp32
    reduce-scatter + all-gather of the bf16 shadow (fp32 master without one)."""
    if world <= 1:
        return {"grad_bytes": 0, "wire_bytes_per_rank": 0}
    f = (world - 1) / world
    if sharded:
        wire = f * grad_numel * 4 + f * grad_numel * (2 if shadow else 4)
        gb = grad_numel * 4
    else:
        gb = grad_numel * (2 if grad_dtype == "bf16" else 4)
        wire = 2 * f * gb
    return {"grad_bytes": int(gb), "wire_bytes_per_rank": int(wire)}


def comm_bus_gbps(wire_bytes_per_rank: int, comm_ms: Optional[float]) -> Optional[float]:
    """Achieved bus bandwidth (GB/s per rank) of a step's synchronisation phase."""
    if not comm_ms or comm_ms <= 0 or not wire_bytes_per_rank:
        return None
    return wire_bytes_per_rank / (comm_ms * 1e-3) / 1e9


def parallel_efficiency(samples_per_s: Optional[float], world: int,
                        ref_samples_per_s: Optional[float]) -> Optional[float]:
    """S(P) / (P * S(1)) -- the BASELINE metric's efficiency term."""
    if not samples_per_s or not ref_samples_per_s:
        return None
    return samples_per_s / (world * ref_samples_per_s)


def scaling_report(world: int, rows_per_rank: int, global_rows: int, step_ms: float,
                   compute_ms: Optional[float], comm_ms: Optional[float],
                   wire_bytes_per_rank: int) -> dict:
    """The BASELINE metric's derived terms for one measured configuration (BASELINE.md:66-70).

    * ``step_ms``    -- the full data-parallel step (max over ranks);
    * ``compute_ms`` -- the same per-rank work with the gradient synchronisation switched off
      (every rank alone = the single-GPU step of this shard size);
    * ``comm_ms``    -- the step's collectives alone (same buckets, dtype and order), no compute.

    Returns samples/s, ``parallel_efficiency`` = S(P) / (P * S(1)) with S(1) the single-GPU
    throughput of the same per-rank work (weak scaling: = compute_ms / step_ms),
    ``exposed_comm_ms`` = step - compute (communication time not hidden behind compute),
    ``overlap_pct`` = the share of the collectives' own time that the step hides, and the
    achieved all-reduce bus bandwidth ``comm_bus_gbps`` = wire bytes per rank / comm_ms.
    """
    out = {"samples_per_s": global_rows / (step_ms * 1e-3) if step_ms > 0 else None}
    if compute_ms:
        s1 = rows_per_rank / (compute_ms * 1e-3)
        out["single_gpu_samples_per_s"] = s1
        out["parallel_efficiency"] = out["samples_per_s"] / (world * s1)
        out["exposed_comm_ms"] = max(0.0, step_ms - compute_ms)
    if comm_ms and compute_ms:
        out["comm_only_ms"] = comm_ms
        hidden = comm_ms - out["exposed_comm_ms"]
        out["overlap_pct"] = 100.0 * min(1.0, max(0.0, hidden / comm_ms))
    if comm_ms:
        out["comm_bus_gbps"] = comm_bus_gbps(wire_bytes_per_rank, comm_ms)
    return out
