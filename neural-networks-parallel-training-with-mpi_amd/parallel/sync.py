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
  stream gated by per-bucket events (capturable in the step's hipGraph); ``mode="root"`` is the
  reference's centralised pattern over RCCL (ncclReduce to rank 0 + ncclBroadcast).
* :class:`ShardedSync` — sharded optimizer state (ZeRO-1): reduce-scatter of the gradient, SGD
  on the rank's own 1/P slice of the arena only, all-gather of the updated parameters.
* :class:`ShmSync` — CPU ranks on one machine: the all-reduce through a shared-memory segment
  (``csrc/host/shm_comm.cpp``), the transport MPI uses between ranks of a node.
"""
from __future__ import annotations

from typing import List, Optional

import torch
from ..utils.knobs import knob
import torch.distributed as dist


def _subtract(rng, cuts):
    """The parts of the half-open range ``rng`` not covered by any of the ranges ``cuts``."""
    lo, hi = rng
    out = []
    for a, b in sorted(cuts):
        if b <= lo or a >= hi:
            continue
        if a > lo:
            out.append((lo, a))
        lo = max(lo, b)
        if lo >= hi:
            break
    if lo < hi:
        out.append((lo, hi))
    return out


class GradSync:
    world = 1

    def __init__(self, arena):
        self.arena = arena
        self._pending_layers = set()
        self._done_buckets = set()
        self.seq = 0  # collective sequence number (for the sequence checker)
        self.sig = 0  # running signature of every collective issued (kind, bucket, offset, size)
        self._recording: Optional[list] = None

    # -- collective signature (utils/seqcheck.py) --------------------------------------------
    # kinds: 1 all-reduce, 2 root reduce+broadcast, 3 reduce-scatter/owner-update/all-gather;
    # dtype codes: 0 fp32, 1 bf16.  Python hashes tuples of ints identically in every process.
    def note(self, kind: int, index: int, offset: int, numel: int, dtype: int):
        rec = (kind, index, offset, numel, dtype)
        self.seq += 1
        self.sig = (self.sig * 1000003 ^ hash(rec)) & 0xFFFFFFFFFFFFFFFF
        if self._recording is not None:
            self._recording.append(rec)

    def record(self, on: bool):
        """Start (on) / stop (returns the notes) recording the collectives issued meanwhile: the
        engine records a graph capture's collectives and replays them into the signature at
        every launch of that graph.  A capture issues nothing: stopping restores the sequence
        number AND the signature to their values at the start (also when the capture failed),
        so only the launches count -- a rank that captures an extra graph (e.g. a partial last
        mini-batch of its own) keeps the same signature as its peers."""
        if on:
            self._recording = []
            self._rec_saved = (self.seq, self.sig)
            return None
        out, self._recording = self._recording or [], None
        saved, self._rec_saved = getattr(self, "_rec_saved", None), None
        if saved is not None:
            self.seq, self.sig = saved
        return out

    def replay(self, notes):
        for rec in notes:
            self.note(*rec)

    def plan(self):
        """What this rank will issue every step: sync kind, payload dtype, buckets."""
        return (type(self).__name__, getattr(self, "bf16", False),
                tuple((b.index, b.offset, b.numel) for b in self.arena.buckets))

    def begin(self):
        self._done_buckets = set()

    def ready(self, layer: int):
        for b in self.arena.buckets_completed_by(layer):
            if b.index not in self._done_buckets:
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

    def capture_origin(self):
        """The stream a hipGraph capture of a step must START on (None: the compute stream).
        RCCL (ROCm 7, RCCL 2.26) crashes in hipStreamEndCapture when the first collective of a
        capture is issued on a stream forked from the origin (scripts/rccl_capture_probe.py,
        variant "side": SIGSEGV at P=2; "comm_origin": fine), so a schedule that issues its
        collectives on a comm stream captures with that stream as the origin and forks the
        compute stream from it."""
        return None

    def comm_only(self):
        """Issue exactly the collectives of one step's gradient synchronisation on the current
        stream, with no compute around them (the bench's comm-only timing: achieved bus
        bandwidth and how much of the communication the overlapped step hides)."""


class NoSync(GradSync):
    world = 1

    def launch_bucket(self, bucket, stream):
        return stream   # single rank: the local gradient is final


class TorchDistSync(GradSync):
    """``grad_dtype="bf16"``: the payload is rounded to bf16 before and after an fp32 reduction
    -- the numeric contract of the native path's one-rounding bf16 all-reduce
    (NativeRcclSync ``bf16_reduce="acc32"``), up to gloo's summation order at P > 2."""

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
        self.note(2 if self.mode == "root" else 1, bucket.index, bucket.offset, bucket.numel,
                  int(self.bf16))
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

    def comm_only(self):
        for b in self.arena.buckets:
            view = self.arena.grad[b.offset:b.offset + b.numel]
            if self.bf16:   # the payload the step sends (the wire-byte count assumes it)
                view = view.to(torch.bfloat16)
            if self.mode == "root":
                dist.reduce(view, dst=0, group=self.group)
                dist.broadcast(view, src=0, group=self.group)
            else:
                dist.all_reduce(view, group=self.group)

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
                 grad_dtype: str = "fp32", mode: str = "allreduce", bf16_reduce: str = "",
                 f32_reduce: str = ""):
        """``bf16_reduce`` (bf16 payload): ``acc32`` (default) sums the P bf16 copies of every
        element in fp32 on its owner and rounds ONCE (all-to-all + owner sum + all-gather,
        RcclComm::allreduce_bf16_acc32) -- the result is bf16(sum_r bf16(g_r)) whatever P is,
        the same contract as the CPU path's round / fp32-sum / round; ``rccl`` is ncclAllReduce
        in bf16, whose ring rounds the partial sum at every one of its P-1 hops (the error
        grows with P: tests/test_multirank_gpu.py::test_rccl_bf16_reduction_error_vs_p).
        ``f32_reduce`` (fp32 payload): ``ordered`` is the same all-to-all / owner sum /
        all-gather in fp32 (RcclComm::allreduce_f32_ordered): every element is summed in rank
        order wherever it sits in a bucket, so two schedules that cut the gradient into
        different buckets (inline vs overlap_rowband) agree bit for bit at any P when their
        per-rank gradients agree (for the row-band schedules: under the same RowbandStep
        split-K plan, NNMPI_RB_PLAN) -- a ring's order depends on the element's chunk, which
        differs between bucketings at P >= 3; ``rccl`` is one ncclAllReduce per bucket.  Default
        (""): ``rccl`` when the gradient is ONE bucket (the inline schedule: nothing to be
        independent of, and one collective costs less than two grouped all-to-all rounds plus
        a sum kernel), ``ordered`` when it is cut into several."""
        super().__init__(arena)
        self.mode = mode
        # the root pattern is a serial reduce + broadcast: always on the compute stream
        self.inline = bool(inline) or mode == "root"
        # bf16 payload: half the bytes on xGMI (bandwidth-bound regime, e.g. the 8192-wide
        # model); the gradient is cast into a bf16 staging arena before and back after the
        # reduction, on the stream that owns that step.
        self.bf16 = grad_dtype == "bf16"
        if self.inline and len(arena.buckets) > 1:
            # serial all-reduce: one call over the whole arena amortises the collective latency
            arena.replan_single_bucket()
        from .. import native
        self.native = native
        self.comm = native_comm
        self.world = world
        self.gs = native.lib().GradSync(native_comm, len(arena.buckets), priority)
        self._launched = False
        # zeros: ranges the engine's bf16 weight-gradient epilogues write directly are never
        # cast into, so their alignment padding must start (and stay) zero
        self.gbuf = (torch.zeros(arena.numel, dtype=torch.bfloat16, device=arena.grad.device)
                     if self.bf16 else None)
        self._comm_stream = torch.cuda.ExternalStream(self.gs.comm_stream)
        import os
        self.bf16_reduce = bf16_reduce or knob("NNMPI_BF16_REDUCE", "acc32")
        if self.bf16_reduce not in ("acc32", "rccl"):
            raise ValueError(f"bf16_reduce must be acc32 or rccl, not {self.bf16_reduce!r}")
        self.f32_reduce = f32_reduce or knob(
            "NNMPI_F32_REDUCE", "rccl" if len(arena.buckets) == 1 else "ordered")
        if self.f32_reduce not in ("ordered", "rccl"):
            raise ValueError(f"f32_reduce must be ordered or rccl, not {self.f32_reduce!r}")
        # collective stand-in (measurement only): "k:gbps" holds k CUs on the comm stream after
        # each bucket's collective for its bytes at gbps (csrc/kernels/standin.hip)
        st = knob("NNMPI_COMM_STANDIN", "")
        if st:
            k, gbps = st.split(":")
            self.gs.set_standin(int(k), float(gbps))
        self.scratch = None
        if self.bf16 and self.bf16_reduce == "acc32" and mode != "root":
            # one bucket reduces at a time on its stream: scratch for the largest
            n = max(b.numel for b in arena.buckets)
            self.scratch = torch.empty(max(1, native_comm.acc32_scratch_elems(n)),
                                       dtype=torch.bfloat16, device=arena.grad.device)
            self.gs.set_acc32_scratch(self.scratch.data_ptr())
        self.scratch32 = None
        if not self.bf16 and self.f32_reduce == "ordered" and mode != "root" and world > 1:
            n = max(b.numel for b in arena.buckets)
            self.scratch32 = torch.empty(max(1, native_comm.acc32_scratch_elems(n)),
                                         dtype=torch.float32, device=arena.grad.device)
            self.gs.set_f32_scratch(self.scratch32.data_ptr())

    def _allreduce(self, ptr: int, n: int, dt: int, h: int):
        if dt == 1 and self.scratch is not None:
            self.comm.allreduce_bf16_acc32(ptr, self.scratch.data_ptr(), n, h)
        elif dt == 0 and self.scratch32 is not None:
            self.comm.allreduce_f32_ordered(ptr, self.scratch32.data_ptr(), n, h)
        else:
            self.comm.allreduce(ptr, n, dt, 0, h)

    def _launch(self, bucket, stream=None, cast_back: bool = True, written=()):
        view = self.arena.grad[bucket.offset:bucket.offset + bucket.numel]
        self.note(2 if self.mode == "root" else 1, bucket.index, bucket.offset, bucket.numel,
                  int(self.bf16))
        h = int(stream.cuda_stream) if stream is not None else self.native.stream_handle()
        lib = self.native.lib()
        ptr, dt = view.data_ptr(), 0
        if self.bf16:
            ptr, dt = self.gbuf[bucket.offset:].data_ptr(), 1
            # cast the fp32 gradient into the payload, except the `written` arena ranges whose
            # bf16 values the producing kernels stored there themselves
            for lo, hi in _subtract((bucket.offset, bucket.offset + bucket.numel), written):
                lib.cast_f32_bf16(self.arena.grad[lo:].data_ptr(), self.gbuf[lo:].data_ptr(),
                                  hi - lo, h)
        if self.inline:
            if self.mode == "root":
                # reference pattern (ref.py:185-203): everything through rank 0
                self.comm.reduce(ptr, bucket.numel, dt, 0, 0, h)
                self.comm.broadcast(ptr, bucket.numel, dt, 0, h)
            else:
                self._allreduce(ptr, bucket.numel, dt, h)
            if self.bf16:
                lib.cast_bf16_f32(ptr, view.data_ptr(), bucket.numel, h)
            return
        self.gs.bucket_ready(bucket.index, ptr, bucket.numel, dt, h)
        if self.bf16 and cast_back:   # back to fp32 on the comm stream, ahead of its update
            lib.cast_bf16_f32(ptr, view.data_ptr(), bucket.numel, self.gs.comm_stream)
        self._launched = True

    def update_grad(self):
        """The buffer the engine's per-bucket updates read after :meth:`launch_bucket` with
        ``cast_back=False``: the bf16 payload itself (None: the fp32 gradient arena)."""
        return self.gbuf if (self.bf16 and not self.inline) else None

    def launch_bucket(self, bucket, stream, cast_back: bool = True, written=()):
        """``written``: (lo, hi) arena ranges already holding their bf16 gradient in the payload
        buffer (bf16 payload only)."""
        # NB: every collective of one communicator stays on ONE stream -- a bucket issued on
        # the compute stream while earlier ones are still queued on the comm stream lets the two
        # run concurrently on the GPU, in different orders on different ranks: measured to hang
        # (and, inside a capture, to crash) at P = 2 / 3
        self._launch(bucket, stream, cast_back=cast_back, written=written)
        return None if self.inline else self._comm_stream

    def capture_origin(self):
        return None if self.inline else self._comm_stream

    def comm_only(self):
        h = self.native.stream_handle()
        lib = self.native.lib()
        for b in self.arena.buckets:
            view = self.arena.grad[b.offset:b.offset + b.numel]
            ptr, dt = view.data_ptr(), 0
            if self.bf16:
                ptr, dt = self.gbuf[b.offset:].data_ptr(), 1
                lib.cast_f32_bf16(view.data_ptr(), ptr, b.numel, h)
            if self.mode == "root":
                self.comm.reduce(ptr, b.numel, dt, 0, 0, h)
                self.comm.broadcast(ptr, b.numel, dt, 0, h)
            else:
                self._allreduce(ptr, b.numel, dt, h)
            if self.bf16:
                lib.cast_bf16_f32(ptr, view.data_ptr(), b.numel, h)

    def finish(self):
        if self._launched:
            self.gs.join(self.native.stream_handle())
        self._launched = False


class ShardedSync(GradSync):
    """Sharded optimizer state, ZeRO stage 1 ("optional stretch: reduce-scatter +
    sharded SGD + all-gather").

    The flat arena (padded to a multiple of ``world * 64`` elements) is cut into ``world`` equal
    contiguous slices; rank r owns slice r.  Per step, after the whole backward:

    1. the gradient is reduce-scattered: rank r receives the SUM over ranks of its slice only
       (RCCL ncclReduceScatter in place; gloo has no reduce-scatter, so the CPU path all-reduces
       and uses its slice -- the same sums);
    2. only the owner applies SGD-momentum to its slice (1/P folded in, as usual), so the
       momentum of the other slices is never read or written;
    3. the updated parameters are all-gathered: the bf16 compute shadow when there is one (half
       the bytes of fp32), else the fp32 master.  With a shadow, the fp32 master is still read
       by the kernels in a few places -- every bias (forward epilogue) and the whole output
       layer (head) -- so those regions are refreshed in fp32 as well: one grouped in-place
       ncclBroadcast of each region's pieces from their owners (:meth:`_master_pieces`; a few
       KB).  The rest of the master of foreign slices is never read until
       :meth:`gather_state`.

    Bytes on the wire per step: reduce-scatter fp32 + all-gather bf16 (+ the fp32 bias/head
    pieces) ~= 3/4 of an fp32 all-reduce.  :meth:`gather_state` re-assembles the full fp32 master and momentum (collective:
    every rank calls it) before checkpoints and the final state_dict.
    """
    sharded = True

    def __init__(self, arena, world: int, rank: int, native_comm=None, group=None):
        super().__init__(arena)
        if arena.numel % (world * 64):
            raise ValueError("ShardedSync needs an arena padded to a multiple of world*64 "
                             f"(numel={arena.numel}, world={world})")
        self.world, self.rank = world, rank
        self.shard = arena.numel // world
        self.off = rank * self.shard
        self.comm = native_comm
        self.group = group
        if native_comm is not None:
            from .. import native
            self.native = native
        self.pieces = self._master_pieces()

    def _master_pieces(self):
        """(offsets, counts, roots) of the fp32-master regions the kernels read besides the
        bf16 shadow -- the output layer's weight + bias and every hidden bias -- cut at the
        shard boundaries, each piece owned (and broadcast) by the rank whose slice holds it."""
        ar = self.arena
        last = ar.n_layers - 1
        regions = [ar.layer_range[last]]
        for li in range(last):
            sl = ar.by_name[f"layers.{2 * li}.bias"]
            regions.append((sl.offset, sl.offset + sl.numel))
        offs, cnts, roots = [], [], []
        for s, e in regions:
            while s < e:
                r = s // self.shard
                cut = min(e, (r + 1) * self.shard)
                offs.append(s)
                cnts.append(cut - s)
                roots.append(r)
                s = cut
        return offs, cnts, roots

    def ready(self, layer: int):
        pass   # nothing moves until the whole gradient exists

    def launch_bucket(self, bucket, stream):
        return None

    def _views(self, buf):
        return [buf[r * self.shard:(r + 1) * self.shard] for r in range(self.world)]

    def update(self, ops, hp, nesterov: bool, first: bool):
        """Reduce-scatter -> owner SGD -> all-gather, on the current (compute) stream."""
        ar = self.arena
        self.note(3, 0, 0, self.shard, 0)
        if self.comm is not None:
            h = self.native.stream_handle()
            g = ar.grad.data_ptr()
            self.comm.reduce_scatter(g, g + 4 * self.off, self.shard, 0, 0, h)
        else:
            dist.all_reduce(ar.grad, group=self.group)
        ops.sgd(ar, hp, nesterov, first, offset=self.off, numel=self.shard)
        if self.comm is not None:
            if ar.shadow is not None:
                s = ar.shadow.data_ptr()
                self.comm.allgather(s + 2 * self.off, s, self.shard, 1, h)
                offs, cnts, roots = self.pieces
                self.comm.broadcast_pieces(ar.master.data_ptr(), offs, cnts, roots, 0, h)
            else:
                m = ar.master.data_ptr()
                self.comm.allgather(m + 4 * self.off, m, self.shard, 0, h)
        else:
            dist.all_gather(self._views(ar.master),
                            ar.master[self.off:self.off + self.shard].clone(), group=self.group)
            if ar.shadow is not None:
                ar.shadow.copy_(ar.master)

    def comm_only(self):
        ar = self.arena
        if self.comm is None:
            dist.all_reduce(ar.grad, group=self.group)
            dist.all_gather(self._views(ar.master),
                            ar.master[self.off:self.off + self.shard].clone(), group=self.group)
            return
        h = self.native.stream_handle()
        g = ar.grad.data_ptr()
        self.comm.reduce_scatter(g, g + 4 * self.off, self.shard, 0, 0, h)
        if ar.shadow is not None:
            s = ar.shadow.data_ptr()
            self.comm.allgather(s + 2 * self.off, s, self.shard, 1, h)
            offs, cnts, roots = self.pieces
            self.comm.broadcast_pieces(ar.master.data_ptr(), offs, cnts, roots, 0, h)
        else:
            m = ar.master.data_ptr()
            self.comm.allgather(m + 4 * self.off, m, self.shard, 0, h)

    def gather_state(self):
        """Full fp32 master + momentum on every rank (checkpoint / final parameters)."""
        ar = self.arena
        for buf in (ar.master, ar.momentum):
            own = buf[self.off:self.off + self.shard]
            if self.comm is not None:
                import torch as _t
                s = _t.cuda.current_stream()
                p = buf.data_ptr()
                self.comm.allgather(p + 4 * self.off, p, self.shard, 0, int(s.cuda_stream))
                s.synchronize()
            else:
                dist.all_gather(self._views(buf), own.clone(), group=self.group)


def shm_sync_ok(device_type: str, world: int, local_world: int, grad_dtype: str = "fp32",
                mode: str = "allreduce") -> bool:
    """CPU ranks that all run on this machine, fp32 all-reduce: the shared-memory transport
    applies (NNMPI_SHM=0 keeps gloo)."""
    import os
    return (device_type == "cpu" and world > 1 and local_world == world and grad_dtype == "fp32"
            and mode == "allreduce" and knob("NNMPI_SHM", "1") != "0")


def make_shm_sync(arena, group, world: int, rank: int, timeout_s: float = 120.0):
    """A :class:`ShmSync` when EVERY rank can use it, else None (the caller keeps gloo).  Each
    rank first tries to load the native library and the ranks agree on the outcome (a MIN
    all-reduce of an ok flag over ``group``), so a rank that cannot load it never leaves the
    others waiting in the segment setup's barriers; the segment setup agrees the same way."""
    try:
        from .. import native
        native.lib()
        ok = 1
    except Exception:
        ok = 0
    if not _agree(ok, group):
        return None
    try:
        return ShmSync(arena, group, world, rank, timeout_s=timeout_s)
    except _ShmSetupFailed:
        return None


def _agree(ok: int, group) -> bool:
    t = torch.tensor([int(ok)], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


class _ShmSetupFailed(RuntimeError):
    pass


class ShmSync(GradSync):
    """Gradient all-reduce of CPU ranks on one machine through shared memory.

    The reference's mpiexec ranks exchange gradients through MPI, which moves intra-node
    messages through shared memory; gloo (``TorchDistSync``) goes through loopback TCP -- for the
    reference config's 13-parameter gradient ~0.3-0.4 ms per all-reduce, ten times the whole
    native step (ops/host_ops.py).  Here every call is a copy into this rank's slot of a mapped
    segment, one arrival counter and a rank-ordered sum (identical bits on every rank), inline in
    the step like the native RCCL path's inline form.  Set up over the job's gloo group: rank 0
    creates the segment under a random name, the others attach, then the name is unlinked (the
    mapping lives until the last rank exits, nothing is left in /dev/shm)."""

    def __init__(self, arena, group, world: int, rank: int, timeout_s: float = 120.0):
        super().__init__(arena)
        import os
        import secrets
        from .. import native
        self.world, self.rank, self.group, self.timeout_s = world, rank, group, float(timeout_s)
        if len(arena.buckets) > 1:
            arena.replan_single_bucket()   # one call per step amortises the arrival wait
        obj = [f"/nnmpi-{os.getpid()}-{secrets.token_hex(6)}" if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        self.name = obj[0]
        cap = max(b.numel for b in arena.buckets)
        lib = native.lib()
        # create on rank 0, then attach on the others; every step agreed over gloo, so a failure
        # on any rank fails the setup on all of them (make_shm_sync falls back to gloo)
        self.comm = None
        for creator in (True, False):
            ok = 1
            if (rank == 0) == creator:
                try:
                    self.comm = lib.ShmComm(self.name, rank, world, cap, creator)
                except Exception:
                    ok = 0
            if not _agree(ok, group):
                if rank == 0 and self.comm is not None:
                    self.comm.unlink()
                raise _ShmSetupFailed("shared-memory all-reduce setup failed on some rank")
        if rank == 0:
            self.comm.unlink()

    def _launch(self, bucket):
        view = self.arena.grad[bucket.offset:bucket.offset + bucket.numel]
        self.note(1, bucket.index, bucket.offset, bucket.numel, 0)
        self.comm.allreduce_sum(view.data_ptr(), bucket.numel, self.timeout_s)

    def comm_only(self):
        for b in self.arena.buckets:
            self._launch(b)

