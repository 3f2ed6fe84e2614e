"""Gradient synchronisation strategies (the data-parallel core).

The reference averages gradients by pickling every rank's gradient list to rank 0
(``comm.gather``, ref.py:185), summing them there in rank order, dividing by P (ref.py:190-197)
and sending the mean back with P-1 serial ``comm.send`` calls (ref.py:199, recv ref.py:203):
2(P-1)·G bytes through the root every step, fully blocking.

Here the flat gradient arena is split into contiguous buckets in backward order
(:mod:`nnmpi_amd.engine.arena`); the engine calls :meth:`GradSync.ready` after each layer's
weight gradient, a bucket's all-reduce (SUM) is launched as soon as its last layer is ready and
overlaps the remaining backward, and :meth:`GradSync.finish` joins before the optimizer, which
folds the 1/P (or per-rank weighted) scale into the SGD kernel.

Implementations
* :class:`NoSync` — world size 1.
* :class:`TorchDistSync` — ``torch.distributed`` (gloo on CPU, nccl = RCCL on GPU), async work
  handles per bucket.  ``mode="root"`` reproduces the reference's centralised pattern (reduce to
  rank 0 + broadcast) for comparison.
* :class:`NativeRcclSync` — the C++ runtime: ncclAllReduce per bucket on a dedicated HIP comm
  stream gated by per-bucket events (capturable in the step's hipGraph).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist


class GradSync:
    world = 1

    def __init__(self, arena):
        self.arena = arena
        self._pending_layers = set()
        self.seq = 0  # collective sequence number (for the sequence checker)

    def begin(self):
        self._done_buckets = set()

    def ready(self, layer: int):
        b = self.arena.bucket_of_layer(layer)
        if b.index in self._done_buckets:
            return
        if layer == min(b.layers):
            self._done_buckets.add(b.index)
            self._launch(b)

    def _launch(self, bucket):
        pass

    def launch_bucket(self, bucket, stream):
        """Launch the reduction of a complete bucket whose gradients were produced on ``stream``.
        Returns the stream on which the reduced bucket is ready (the engine runs that bucket's
        optimizer update there), or None when the update must wait for :meth:`finish`."""
        self._launch(bucket)
        return None

    def finish(self):
        pass


class NoSync(GradSync):
    world = 1

    def launch_bucket(self, bucket, stream):
        return stream   # single rank: the local gradient is final


class TorchDistSync(GradSync):
    """``grad_dtype="bf16"``: the payload is rounded to bf16 before and after the reduction
    (the gloo/CPU rendition of the compressed all-reduce; the native path reduces in bf16)."""

    def __init__(self, arena, group, world: int, mode: str = "allreduce", overlap: bool = True,
                 grad_dtype: str = "fp32"):
        super().__init__(arena)
        self.group = group
        self.world = world
        self.mode = mode
        self.overlap = overlap and grad_dtype == "fp32"
        self.bf16 = grad_dtype == "bf16"
        self._works: List = []
        self._rounded: List = []

    def _launch(self, bucket):
        view = self.arena.grad[bucket.offset:bucket.offset + bucket.numel]
        self.seq += 1
        if self.bf16:
            view.copy_(view.to(torch.bfloat16))
            self._rounded.append(view)
        if self.mode == "root":
            # reference pattern: everything through rank 0 (reduce to root, then fan out)
            dist.reduce(view, dst=0, group=self.group)
            dist.broadcast(view, src=0, group=self.group)
            return
        w = dist.all_reduce(view, group=self.group, async_op=self.overlap)
        if w is not None:
            self._works.append(w)

    def finish(self):
        for w in self._works:
            w.wait()
        self._works.clear()
        for v in self._rounded:
            v.copy_(v.to(torch.bfloat16))
        self._rounded.clear()


class NativeRcclSync(GradSync):
    """``inline=True``: the all-reduce is issued on the producing (compute) stream itself — no
    comm stream, no cross-queue events.  Measured on MI355X: every cross-HW-queue dependency
    costs ~8-10 us and a hipGraph with parallel branches spreads even a linear kernel chain over
    several queues, so for small (latency-bound) gradient volumes the serial inline form is
    faster than overlap; large volumes use the overlapped comm stream."""

    def __init__(self, arena, native_comm, world: int, priority: int = -1, inline: bool = False,
                 grad_dtype: str = "fp32"):
        super().__init__(arena)
        self.inline = bool(inline)
        # bf16 payload: half the bytes on xGMI (bandwidth-bound regime, e.g. the 8192-wide
        # model); the gradient is cast into a bf16 staging arena before and back after the
        # reduction, on the stream that owns that step.
        self.bf16 = grad_dtype == "bf16"
        if self.inline and len(arena.buckets) > 1:
            # serial all-reduce: one call over the whole arena amortises the collective latency
            arena.buckets = arena._plan_buckets(float(1 << 62), 4)
        from .. import native
        self.native = native
        self.comm = native_comm
        self.world = world
        self.gs = native.lib().GradSync(native_comm, len(arena.buckets), priority)
        self._launched = False
        self.gbuf = (torch.empty(arena.numel, dtype=torch.bfloat16, device=arena.grad.device)
                     if self.bf16 else None)
        self._comm_stream = torch.cuda.ExternalStream(self.gs.comm_stream)

    def _launch(self, bucket, stream=None):
        view = self.arena.grad[bucket.offset:bucket.offset + bucket.numel]
        self.seq += 1
        h = int(stream.cuda_stream) if stream is not None else self.native.stream_handle()
        lib = self.native.lib()
        ptr, dt = view.data_ptr(), 0
        if self.bf16:
            ptr, dt = self.gbuf[bucket.offset:].data_ptr(), 1
            lib.cast_f32_bf16(view.data_ptr(), ptr, bucket.numel, h)
        if self.inline:
            self.comm.allreduce(ptr, bucket.numel, dt, 0, h)
            if self.bf16:
                lib.cast_bf16_f32(ptr, view.data_ptr(), bucket.numel, h)
            return
        self.gs.bucket_ready(bucket.index, ptr, bucket.numel, dt, h)
        if self.bf16:   # back to fp32 on the comm stream, ahead of the bucket's update there
            lib.cast_bf16_f32(ptr, view.data_ptr(), bucket.numel, self.gs.comm_stream)
        self._launched = True

    def launch_bucket(self, bucket, stream):
        self._launch(bucket, stream)
        return None if self.inline else self._comm_stream

    def finish(self):
        if self._launched:
            self.gs.join(self.native.stream_handle())
        self._launched = False
