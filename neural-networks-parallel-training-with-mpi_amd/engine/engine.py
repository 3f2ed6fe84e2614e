"""Explicit data-parallel MLP training engine.

One step (per rank), replacing the reference's hot loop ``ref.py:155-211`` (DataLoader ->
``.float()`` -> forward -> MSELoss -> autograd backward -> gather/average/send -> SGD):

    forward   h_i = act(h_{i-1} W_i^T + b_i)                  hidden layers (GEMM + epilogue)
    head      logits, loss, dlogits, dZ_{L-2}, dW_{L-1}, db   fused output layer + loss
              -> grad bucket(s) of layer L-1 ready -> all-reduce starts on the comm stream
    backward  for i = L-2 .. 0:
                 dW_i, db_i = dZ_i^T h_{i-1}, sum(dZ_i)       wgrad (+ fused bias grad)
                 -> bucket ready -> all-reduce overlaps the rest of backward
                 dZ_{i-1} = (dZ_i W_i) * act'(h_{i-1})        dgrad + activation backward
    join      compute stream waits for the comm stream
    update    fused SGD-momentum over the whole arena (1/P folded in, bf16 shadow refreshed,
              gradients zeroed for the next step)

All buffers are allocated once (rows capacity), so on the GPU the steady-state step is
allocation-free and is captured into ONE hipGraph (kernels + RCCL + cross-stream events) that
is replayed every step.  The same schedule runs with :class:`~nnmpi_amd.ops.torch_ops.TorchOps`
on the CPU (gloo) — that is the reference-semantics path and the test oracle.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Tuple

import torch
from ..utils.knobs import knob

from ..models.mlp import MLPSpec
from .arena import Arena

TINY_MAX_WIDTH = 16
TINY_MAX_LAYERS = 4


LOSS_HIST_MAX = 1024   # steps per loss-recording graph (run_steps(..., losses=...))


class MLPEngine:
    def __init__(self, spec: MLPSpec, arena: Arena, ops, sync, *, device, dtype: torch.dtype,
                 rows_capacity: int, lr: float, momentum: float, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, use_graph: bool = True,
                 use_tiny: Optional[bool] = None, overlap: bool = True, fuse_sgd: bool = True,
                 grouped: bool = True, rowband_overlap: bool = False,
                 rowband_plan: Optional[int] = None):
        self.spec = spec
        self.arena = arena
        self.ops = ops
        self.sync = sync
        self.device = torch.device(device)
        self.dtype = dtype
        self.R = max(1, int(rows_capacity))
        self.nesterov = bool(nesterov)
        self.is_cuda = self.device.type == "cuda"
        L = spec.n_layers
        w = spec.widths
        self.L = L
        self.act = spec.activation
        self.loss_kind = spec.loss
        if use_tiny is None:
            # GPU: tiny_mlp.hip; CPU: the host twin when the op set has it (ops/host_ops.py)
            use_tiny = ((self.is_cuda or hasattr(ops, "tiny_step")) and dtype == torch.float32
                        and L <= TINY_MAX_LAYERS and max(w) <= TINY_MAX_WIDTH)
        self.use_tiny = bool(use_tiny)
        # host-driven torch.distributed transports (gloo copies device tensors through the host;
        # torch's nccl runs on its own side stream) cannot live inside a replayed hipGraph
        from ..parallel.sync import TorchDistSync
        self.use_graph = (bool(use_graph) and self.is_cuda
                          and not (isinstance(sync, TorchDistSync) and sync.world > 1))
        self._validate()
        dev, R = self.device, self.R
        self.stream = torch.cuda.Stream(device=dev) if self.is_cuda else None
        # persistent buffers
        self.X = torch.zeros(R, w[0], dtype=dtype, device=dev)
        if spec.loss == "mse":
            self.Y = torch.zeros(R, w[-1], dtype=torch.float32, device=dev)
            self.labels = None
        else:
            self.Y = None
            self.labels = torch.zeros(R, dtype=torch.int64, device=dev)
        self.acts = [torch.zeros(R, w[i + 1], dtype=dtype, device=dev) for i in range(L - 1)]
        self.dzl = [torch.zeros(R, w[i + 1], dtype=dtype, device=dev) for i in range(L - 1)]
        self.dlogits = torch.zeros(R, w[-1], dtype=torch.float32, device=dev)
        self.loss_out = torch.zeros(4, dtype=torch.float32, device=dev)
        self.hp = torch.tensor([lr, momentum, dampening, weight_decay, 1.0, 0, 0, 0],
                               dtype=torch.float32, device=dev)
        self.overlap = bool(overlap) and self.is_cuda and not self.use_tiny
        from ..parallel.sync import NoSync
        self.fuse_sgd = (bool(fuse_sgd) and self.overlap and isinstance(sync, NoSync)
                         and dtype == torch.bfloat16 and hasattr(ops, "sgd_fusion"))
        # tiny single-rank model: the one-block kernel applies SGD itself (one launch per step)
        self.tiny_fused = (bool(fuse_sgd) and self.use_tiny and isinstance(sync, NoSync)
                           and hasattr(ops, "tiny_can_fuse_sgd") and ops.tiny_can_fuse_sgd(self.R))
        self._first = True
        self.ws = torch.zeros(max(1, self._workspace_bytes() // 4 + 64), dtype=torch.float32,
                              device=dev)
        # grouped backward (bf16 GPU): dgrad_i + wgrad_i + combine_{i+1} in one launch.  Layer
        # i's slabs live in ws_pair[(L-1-i) % 2] so they never alias the pending combine's.
        from ..parallel.sync import NativeRcclSync
        self.sharded = bool(getattr(sync, "sharded", False))
        inline_sync = (isinstance(sync, NoSync) or self.sharded or
                       (isinstance(sync, NativeRcclSync) and sync.inline))
        # per-bucket collectives on the native comm stream, each bucket's SGD on an update stream
        self.comm_overlap = isinstance(sync, NativeRcclSync) and not sync.inline
        # (shapes the grouped kernel does not cover -- e.g. the 256x256-tile 8192-wide layers --
        # take the sequential fused schedule, whose un-split wgrads apply SGD in their epilogue)
        # (layers cut into output-row chunk buckets are reduced chunk by chunk behind their own
        # weight-gradient launches: the sequential schedule, never the grouped one)
        self.grouped = (bool(grouped) and self.overlap and dtype == torch.bfloat16
                        and (inline_sync or self.comm_overlap)
                        and not any(getattr(b, "rows", None) is not None for b in arena.buckets)
                        and hasattr(ops, "bwd_group") and L > 1 and
                        all(ops.bwd_group_supported(self.R, *spec.layer_shape(i))
                            for i in range(L - 1)))
        self.ws_pair = [self.ws, torch.zeros_like(self.ws)] if self.grouped else [self.ws, self.ws]
        # Row-band step (narrow square MSE regressor, e.g. the 512-wide proxy): the forward, the
        # head and every activation gradient in ONE launch, all weight gradients in one more and
        # every combine (+ the fused update on one rank) in a third -- see rowband.hip.  Taken
        # whenever the gradient is reduced after the backward (one rank, the inline all-reduce,
        # ZeRO-1): it produces every layer's gradient at once, so there is nothing for a
        # per-bucket overlapped schedule to hide.  NNMPI_EXPERIMENTS=1 NNMPI_ROWBAND=0 keeps the grouped schedule
        # (proxy step 0.082 vs 0.094 ms, profiles/r3s2_rowband_*).
        # rowband_overlap: also with per-bucket collectives on the comm stream -- the band launch
        # and the last hidden layer's + the head's weight gradients first, their bucket's
        # all-reduce overlapping the other layers' weight gradients (_step_body_rowband_overlap)
        self.rb_overlap = bool(rowband_overlap) and self.comm_overlap
        self.rowband = (self.overlap and dtype == torch.bfloat16 and
                        (inline_sync or self.rb_overlap) and
                        hasattr(ops, "rowband_ok") and knob("NNMPI_ROWBAND", "1") != "0"
                        and ops.rowband_ok(self.R, w, self.act, spec.loss))
        # split-K plan of the weight gradients (RowbandStep::plan): the overlapped schedule's
        # phased plan, else one launch filling the chip with every layer
        if rowband_plan is None:
            rowband_plan = int(knob("NNMPI_RB_PLAN", "1" if self.rb_overlap else "0"))
        self.rb_plan = int(rowband_plan)
        self.ws_rb = (torch.zeros(ops.rowband_workspace_bytes(self.R, w[1], L - 1, in_=w[0]) // 4 + 64,
                                  dtype=torch.float32, device=dev) if self.rowband else None)
        # v2 row-band kernel: the weights also live in fragment-major images (one global load per
        # MFMA operand, no LDS staging -- rowband.hip).  The images must hold the CURRENT weights:
        # the single-rank fused combine rewrites them from the updated weights; every other
        # update path (the multi-rank SGD pass, ZeRO-1, other schedules, a reload of the arena
        # -- Arena.version) leaves them stale and the next row-band step rebuilds them first.
        self.rb_version = (ops.rowband_version(self.R, w, self.act, spec.loss) if self.rowband
                           and hasattr(ops, "rowband_version") else (1 if self.rowband else 0))
        self.rb_packed = None
        if self.rb_version == 2:
            self._rb_buf, self.rb_packed = ops.rowband_packed(w[1], w[0], L - 1, dev)
        self._rb_fresh = False
        self._rb_ver = -1
        # A band's passes cost the same whatever the number of bands (per-CU bound: 47 us at
        # 1,024 rows as at 8,192, profiles/r3s2_rowband_pmc.txt), so below this the band kernel
        # is not taken; small batches (strong-scaling shards: up to 4,096 rows of the 512-wide
        # proxy) run the column-split form instead (rowband.hip rowband_split_kernel: each band
        # over 2-8 CUs, activations exchanged per layer), everything else the grouped schedule.
        # 512-wide shards of 4,097-6,143 rows: the band kernel (the column-split form stops at
        # 4,096 rows) -- 0.0629 / 0.0641 / 0.0670 ms at 4,500 / 5,000 / 6,000 rows vs the grouped
        # schedule's 0.0811 / 0.0822 / 0.0868 (profiles/r6_rowband_threshold.txt); other widths
        # keep the measured 6,144
        self.rowband_min_rows = int(knob("NNMPI_ROWBAND_MIN_ROWS", "4097" if w[1] == 512 else "6144"))
        self._rb_split: Dict[int, bool] = {}
        # True: the row-band step also copies out the last hidden layer's activations (debug /
        # inspection; nothing downstream reads them)
        self.rb_keep_last = False
        if self.is_cuda:
            self.ev_wfree = [torch.cuda.Event(enable_timing=False) for _ in range(L)]
        # bf16-payload overlapped schedule: per-bucket updates read the bf16 payload
        self._upd_grad = (sync.update_grad() if (self.comm_overlap and hasattr(sync, "update_grad")
                                                 and hasattr(ops, "sgd")) else None)
        # ... and the chunked weight gradients store that bf16 payload themselves
        self._w16 = (self._upd_grad is not None and dtype == torch.bfloat16
                     and hasattr(ops, "wgrad_can_write_bf16"))
        self._written16: List[Tuple[int, int]] = []
        # Deferred updates (several ranks, bf16 payload written by the chunk weight gradients):
        # the SGD of chunk bucket (layer i+1, rows r0:r1) runs in the epilogue of the weight
        # gradient of chunk (layer i, rows r0:r1) -- same [rows, in] shape -- once its all-reduce
        # has completed (the compute stream waits for that collective's event), instead of as a
        # separate memory-bound pass next to compute-bound GEMMs.  _defer_plan: chunk bucket
        # index -> the partner bucket it updates.
        self._defer_plan: Dict[int, object] = {}
        # (not for the row-band schedules: they never launch the chunk weight gradients whose
        # epilogues would apply these updates, so every target bucket would fall to _join_comm)
        if (self._w16 and hasattr(ops, "linear_wgrad_defer") and not self.sharded
                and not self.rb_overlap and knob("NNMPI_DEFER", "1") != "0"):
            for i in range(L - 2):
                if spec.layer_shape(i) != spec.layer_shape(i + 1):
                    continue
                nxt = {b.rows: b for b in arena.chunk_buckets(i + 1)}
                for b in arena.chunk_buckets(i):
                    if b.rows in nxt:
                        self._defer_plan[b.index] = nxt[b.rows]
        self._defer_targets = {b.index for b in self._defer_plan.values()}
        # NNMPI_DEFER_WAIT=chunk: every deferred update waits on its own partner's collective
        # (default: one wait per partner layer, see _defer_update)
        self._defer_wait_layer = knob("NNMPI_DEFER_WAIT", "layer") != "chunk"
        self._waited = set()
        self.ev_ar = ({b.index: torch.cuda.Event(enable_timing=False)
                       for b in self._defer_plan.values()} if self._defer_plan else {})
        self.rows = 0
        self.steps_done = 0
        self._graphs: Dict[tuple, object] = {}
        self.inv_count = 1.0
        self.loss_scale = 1.0
        self.timer = None   # utils.metrics.EventTimer: per-phase breakdown (steps run eagerly)

    def _mark(self, name: str):
        if self.timer is not None:
            self.timer.mark(name, self.stream)

    # ------------------------------------------------------------------------------------
    def _validate(self):
        w = self.spec.widths
        if self.is_cuda and not self.use_tiny:
            if self.dtype == torch.bfloat16:
                for i in range(self.L - 1):
                    if w[i] % 8 or w[i + 1] % 8:
                        raise ValueError(f"bf16 GPU path needs hidden/input widths % 8 == 0: {w}")
            # (any output layer: heads beyond the skinny kernels run on the general path)

    def _workspace_bytes(self) -> int:
        ops, R, w = self.ops, self.R, self.spec.widths
        need = 0
        if self.use_tiny:
            return ops.tiny_workspace_bytes(R, self.arena.numel) if hasattr(ops, "tiny_workspace_bytes") else 0
        if hasattr(ops, "wgrad_workspace_bytes"):
            for i in range(self.L - 1):
                need = max(need, ops.wgrad_workspace_bytes(R, w[i + 1], w[i], self.dtype))
                # an output-row chunk is its own GEMM: fewer tiles than the whole layer, so it
                # may split K where the layer does not (1024 of 2048 rows at K = 1024: 2 splits)
                for b in self.arena.chunk_buckets(i):
                    need = max(need, ops.wgrad_workspace_bytes(R, b.rows[1] - b.rows[0], w[i],
                                                               self.dtype))
        if hasattr(ops, "head_workspace_bytes"):
            need = max(need, ops.head_workspace_bytes(R, w[-2], w[-1]))
        return need

    # ------------------------------------------------------------------------------------
    def set_hparams(self, lr=None, momentum=None, grad_scale=None):
        # written on the engine's stream: the kernels that read hp (SGD, fused combines) run
        # there, so the write is ordered before the next step and after the previous one
        ctx = torch.cuda.stream(self.stream) if self.is_cuda else _nullctx()
        with ctx, torch.no_grad():
            # fill_ with a scalar is a kernel launch (capturable inside a graph, e.g. the
            # per-step scales of run_epoch); item assignment would copy a host tensor
            if lr is not None:
                self.hp[0:1].fill_(float(lr))
            if momentum is not None:
                self.hp[1:2].fill_(float(momentum))
            if grad_scale is not None:
                self.hp[4:5].fill_(float(grad_scale))

    def set_scales(self, inv_count: float, loss_scale: float, grad_scale: float):
        """Loss-gradient scale (1/count), reported-loss scale, optimizer gradient scale (1/P)."""
        self.inv_count, self.loss_scale = float(inv_count), float(loss_scale)
        self.set_hparams(grad_scale=grad_scale)

    def load_batch(self, X: torch.Tensor, Y: Optional[torch.Tensor] = None,
                   labels: Optional[torch.Tensor] = None):
        """Copy a batch into the persistent (graph-stable) input buffers."""
        n = X.shape[0]
        if n > self.R:
            raise ValueError(f"batch of {n} rows exceeds capacity {self.R}")
        ctx = torch.cuda.stream(self.stream) if self.is_cuda else _nullctx()
        with ctx, torch.no_grad():
            self.X[:n].copy_(X, non_blocking=True)
            if self.Y is not None and Y is not None:
                self.Y[:n].copy_(Y.reshape(n, self.Y.shape[1]), non_blocking=True)
            if self.labels is not None and labels is not None:
                self.labels[:n].copy_(labels, non_blocking=True)
        self.rows = n

    def load_batch_indexed(self, X: torch.Tensor, Y: Optional[torch.Tensor],
                           labels: Optional[torch.Tensor], idx: torch.Tensor):
        """Mini-batch ``idx`` (int64, on the engine's device) of a resident shard, gathered
        straight into the persistent input buffers (HIP: one gather launch per tensor; the
        reference's DataLoader shuffle + per-row __getitem__ + collate, ref.py:146,155)."""
        n = idx.numel()
        if n > self.R:
            raise ValueError(f"batch of {n} rows exceeds capacity {self.R}")
        if n == 0:   # empty micro-batch of a short shard: zero gradient, still steps
            self.rows = 0
            return
        ctx = torch.cuda.stream(self.stream) if self.is_cuda else _nullctx()
        with ctx, torch.no_grad():
            self.ops.gather_rows(X, idx, self.X)
            if self.Y is not None and Y is not None:
                self.ops.gather_rows(Y.reshape(Y.shape[0], self.Y.shape[1]), idx, self.Y)
            if self.labels is not None and labels is not None:
                self.ops.gather_rows(labels, idx, self.labels)
        self.rows = n

    # ------------------------------------------------------------------------------------
    def _dz(self, k: int, rows: int, width: int) -> torch.Tensor:
        return self.dzbuf[k][: rows * width].view(rows, width)

    def _dzl(self, layer: int, rows: int) -> torch.Tensor:
        """Gradient w.r.t. the pre-activation of hidden layer ``layer`` (own buffer per layer,
        so a concurrent wgrad(layer) never races with the next dgrad's output)."""
        return self.dzl[layer][:rows]

    # ---------------- sequential schedule (CPU path, and the no-overlap debug mode) ----------
    def forward_backward(self):
        rows, ops, ar, L = self.rows, self.ops, self.arena, self.L
        if rows == 0:  # empty shard: contributes a zero gradient, still joins every collective
            self.loss_out.zero_()
            ar.grad.zero_()
            for i in reversed(range(L)):
                self.sync.ready(i)
            return
        if self.use_tiny:
            fz = (ops.sgd_fusion(ar, self.hp, self.nesterov, self._first)
                  if self.tiny_fused else None)
            ops.tiny_step(self.spec, ar, self.X[:rows], self.Y[:rows] if self.Y is not None else None,
                          self.labels[:rows] if self.labels is not None else None,
                          self.inv_count, self.loss_out, self.ws, sgd=fz,
                          loss_scale=self.loss_scale)
            for i in reversed(range(L)):
                self.sync.ready(i)
            return
        x = self.X[:rows]
        h = self._forward(x)
        self._mark("fwd")
        last = L - 1
        dz = self._dzl(last - 1, rows) if L > 1 else None
        self._head(h, dz)
        self._mark("head")
        self.sync.ready(last)
        for i in range(L - 2, -1, -1):
            x_in = self.acts[i - 1][:rows] if i > 0 else x
            for _ in self._wgrad_chunks(i, dz, x_in):
                pass
            self.sync.ready(i)
            if i > 0:
                dz_next = self._dzl(i - 1, rows)
                ops.linear_dgrad(dz, ar.compute_weight(i), self.acts[i - 1][:rows], self.act, dz_next)
                dz = dz_next
        self._mark("bwd")

    def _wgrad_chunks(self, i: int, dz, x_in, bf16_out: bool = False):
        """Weight gradient of layer i; a layer cut into output-row chunk buckets (Arena
        .layer_chunks) is computed chunk by chunk, yielding each chunk's bucket as soon as its
        launch is queued (so its all-reduce can start while the next chunk computes).  Every
        output tile is the same GEMM tile over the same K either way: the result is bitwise
        independent of the chunking.

        ``bf16_out`` (bf16-payload overlapped schedule): the chunks' GEMM epilogues store the
        gradient straight into the bf16 payload buffer -- no fp32 gradient write and no cast
        pass; the layer's arena range is recorded in ``self._written16`` so its buckets skip the
        cast.  Same rounding as the cast: bitwise identical payload."""
        ar = self.arena
        gW, gb = ar.grad_weight(i), ar.grad_bias(i)
        chunks = ar.chunk_buckets(i)
        if not chunks:
            self.ops.linear_wgrad(dz, x_in, gW, gb, ws=self.ws)
            return
        g16 = self._upd_grad if bf16_out else None
        if g16 is not None:
            out_f, in_f = self.spec.layer_shape(i)
            if all(self.ops.wgrad_can_write_bf16(dz.shape[0], b.rows[1] - b.rows[0], in_f)
                   for b in chunks):
                self._written16.append(ar.layer_range[i])
            else:
                g16 = None
        for b in chunks:
            r0, r1 = b.rows
            if g16 is not None:
                if not self._defer_update(b, i, dz[:, r0:r1], x_in, g16):
                    self.ops.linear_wgrad(dz[:, r0:r1], x_in, None, None, out_bf16=(
                        ar.weight(i, g16)[r0:r1], ar.bias(i, g16)[r0:r1]))
            else:
                self.ops.linear_wgrad(dz[:, r0:r1], x_in, gW[r0:r1], gb[r0:r1], ws=self.ws)
            yield b

    def _defer_update(self, b, i: int, dz, x_in, g16) -> bool:
        """Launch chunk bucket b's weight gradient (layer i, bf16 payload) with the pending SGD
        of its partner bucket fused into the epilogue; False when there is nothing to fuse."""
        part = self._defer_plan.get(b.index)
        if part is None:
            return False
        k = next((n for n, (pb, _) in enumerate(self._pending_sgd) if pb.index == part.index), None)
        out_f, in_f = self.spec.layer_shape(i)
        r0, r1 = b.rows
        if k is None or not self.ops.wgrad_defer_ok(dz.shape[0], r1 - r0, in_f):
            return False
        self._pending_sgd.pop(k)
        ar, main = self.arena, self.stream
        if self._defer_wait_layer:
            # ONE cross-queue wait per layer: on the collective of the partner layer's last
            # chunk (the comm stream runs its collectives in order, so all earlier chunks of that
            # layer are reduced too) -- issued a whole dgrad earlier, so already complete unless
            # the links are slower than a dgrad; every cross-queue edge in a replayed graph costs
            # 5-10 us whether or not its event has completed (docs/PERF.md)
            li = part.layers[0]
            if li not in self._waited:
                last = max(b.index for b in ar.chunk_buckets(li))
                main.wait_event(self.ev_ar[last])
                self._waited.add(li)
        else:
            main.wait_event(self.ev_ar[part.index])      # the partner's all-reduce has completed
        woff = ar.by_name[f"layers.{2 * (i + 1)}.weight"].offset + part.rows[0] * in_f
        self.ops.linear_wgrad_defer(dz, x_in, ar.weight(i, g16)[r0:r1], ar.bias(i, g16)[r0:r1],
                                    ar, self.hp, self.nesterov, self._first, woff, g16)
        # the rest of the partner bucket (its layer's bias and padding, in the last chunk)
        wend = woff + (r1 - r0) * in_f
        rest = part.offset + part.numel - wend
        if rest > 0:
            self.ops.sgd(ar, self.hp, self.nesterov, self._first, offset=wend, numel=rest,
                         **self._upd_kw())
        return True

    def _forward(self, x):
        h = x
        for i in range(self.L - 1):
            out = self.acts[i][:self.rows]
            self.ops.linear_act(h, self.arena.compute_weight(i), self.arena.bias(i), self.act, out)
            h = out
        return h

    def _head(self, h, dz, sgd=None):
        rows, ar, last = self.rows, self.arena, self.L - 1
        kw = {"sgd": sgd} if sgd is not None else {}
        self.ops.head(h, ar.weight(last), ar.bias(last),
                      self.Y[:rows] if self.Y is not None else None,
                      self.labels[:rows] if self.labels is not None else None,
                      self.loss_kind, self.inv_count, self.act if self.L > 1 else "none", dz,
                      ar.grad_weight(last), ar.grad_bias(last), self.dlogits[:rows], self.loss_out,
                      self.loss_scale, ws=self.ws, **kw)

    def _rb_current(self) -> bool:
        """The v2 row-band weight images hold the current weights."""
        return self._rb_fresh and self._rb_ver == self.arena.version

    def _rb_pack(self):
        """Rebuild the v2 weight images from the bf16 shadow (one launch, on the engine's stream)."""
        self.ops.rowband_pack([self.arena.compute_weight(i) for i in range(self.L - 1)],
                              self.rb_packed)
        self._rb_fresh, self._rb_ver = True, self.arena.version

    def _step_body(self, first: bool):
        self._mark("start")
        if not (self.overlap and self.rows > 0 and self.uses_rowband(self.rows)):
            self._rb_fresh = False        # this step updates the weights without the images
        if self.overlap and self.rows > 0:
            self._step_body_overlap(first)
        else:
            # sequential schedule; also every empty batch (a short shard's empty mini-batch, a
            # rank without rows): forward_backward zeroes the gradient and still issues every
            # bucket's collective in backward order, so this rank joins the same collective
            # sequence as its peers, whatever schedule they run
            self._first = first
            self.sync.begin()
            self.forward_backward()
            self.sync.finish()
            self._mark("comm")
            if not self.tiny_fused or self.rows == 0:
                self._update(first)
        self._mark("update")

    def _update(self, first: bool):
        """Optimizer update of the whole arena (or, sharded, of this rank's slice + gathers)."""
        if self.sharded:
            self.sync.update(self.ops, self.hp, self.nesterov, first)
        else:
            self.ops.sgd(self.arena, self.hp, self.nesterov, first)

    # ---------------- comm-overlapped schedule (GPU) -----------------------------------------
    # Compute stays on ONE stream (measured: splitting wgrad onto a side stream only adds
    # cross-stream waits — every GEMM already fills all 256 CUs, so nothing overlaps).  What runs
    # concurrently is communication: as soon as a bucket's last wgrad is done its all-reduce
    # starts on the comm stream, followed there by that bucket's SGD update (gated on the last
    # reader of its weights, ev_wfree), so only the final bucket's all-reduce + update remain
    # on the critical path.  With one rank the update of the whole arena runs once at the end.
    def _step_body_overlap(self, first: bool):
        rows, ops, ar, L = self.rows, self.ops, self.arena, self.L
        if self.uses_rowband(rows):
            return self._step_body_rowband(first)
        if self.grouped:
            return self._step_body_grouped(first)
        if self.fuse_sgd:
            return self._step_body_fused(first)
        main = self.stream
        self.sync.begin()
        self._sgd_done = set()
        self._reduced = {}
        self._pending_sgd = []
        self._written16 = []
        self._waited = set()
        self._first = first
        x = self.X[:rows]
        h = self._forward(x)
        self._mark("fwd")
        last = L - 1
        dz = self._dzl(last - 1, rows) if L > 1 else None
        self._head(h, dz)
        self._mark("head")
        main.record_event(self.ev_wfree[last])
        self._layer_done(last, main)
        for i in range(L - 2, -1, -1):
            x_in = self.acts[i - 1][:rows] if i > 0 else x
            for b in self._wgrad_chunks(i, dz, x_in, bf16_out=self._w16):
                self._bucket_reduce(b, main)      # chunk's all-reduce starts right away
            if i > 0:
                dz_next = self._dzl(i - 1, rows)
                ops.linear_dgrad(dz, ar.compute_weight(i), self.acts[i - 1][:rows], self.act, dz_next)
                dz = dz_next
            main.record_event(self.ev_wfree[i])
            self._layer_done(i, main)
        self._mark("bwd")
        self._join_comm()
        self._mark("comm")
        rest = [b for b in ar.buckets if b.index not in self._sgd_done]
        if len(rest) == len(ar.buckets):
            self._update(first)                             # one pass over the whole arena
        else:
            for b in rest:
                ops.sgd(ar, self.hp, self.nesterov, first, offset=b.offset, numel=b.numel,
                        **self._upd_kw())

    # Single rank: a layer's gradient is final as soon as its split-K partials are combined, so
    # the reducer applies the SGD update itself (no gradient round trip through HBM, no separate
    # optimizer pass).  dgrad_i runs BEFORE wgrad_i here: it is the last reader of W_i.
    def _step_body_fused(self, first: bool):
        rows, ops, ar, L = self.rows, self.ops, self.arena, self.L
        fz = ops.sgd_fusion(ar, self.hp, self.nesterov, first)
        x = self.X[:rows]
        h = self._forward(x)
        self._mark("fwd")
        last = L - 1
        dz = self._dzl(last - 1, rows) if L > 1 else None
        unfused = []
        if ops.head_can_fuse_sgd(self.spec.widths[-1], self.spec.widths[-2], self.loss_kind):
            self._head(h, dz, sgd=fz)
        else:
            self._head(h, dz)
            unfused.append(last)
        self._mark("head")
        # Wide layers (256x256-tile, un-split weight gradients): wgrad_i + its SGD epilogue runs
        # in ONE launch with dgrad_{i-1} (or, last, with wgrad_0) -- ops.wide_pair -- so the
        # memory-bound SGD epilogues overlap compute-bound main loops.  `pend` is the weight
        # gradient waiting for its partner; every hazard is as in the sequential order: W_i's
        # last reader dgrad_i ran in an earlier launch, dgrad_{i-1} reads only W_{i-1}.
        pairs = hasattr(ops, "wide_pair")
        pend = None

        def wg_of(i, dz_i, x_in):
            return (dz_i, x_in, ar.grad_weight(i), ar.grad_bias(i))

        def pair_wg_ok(i, dz_i):
            out_f, in_f = self.spec.layer_shape(i)
            return pairs and ops.wide_pair_wgrad_ok(dz_i.shape[0], out_f, in_f)

        def issue_wgrad(i, dz_i, x_in):
            out_f, in_f = self.spec.layer_shape(i)
            # dgrad_i was issued before: nothing reads W_i any more, so even an un-split wgrad
            # may update it in its epilogue
            if ops.wgrad_can_fuse_sgd(rows, out_f, in_f, self.dtype, epilogue=True):
                ops.linear_wgrad(dz_i, x_in, ar.grad_weight(i), ar.grad_bias(i), ws=self.ws, sgd=fz)
            else:
                ops.linear_wgrad(dz_i, x_in, ar.grad_weight(i), ar.grad_bias(i), ws=self.ws)
                unfused.append(i)

        for i in range(L - 2, -1, -1):
            x_in = self.acts[i - 1][:rows] if i > 0 else x
            dz_i = dz
            if i > 0:
                dz_next = self._dzl(i - 1, rows)
                dg = (dz_i, ar.compute_weight(i), self.acts[i - 1][:rows], self.act, dz_next)
                out_f, in_f = self.spec.layer_shape(i)
                if pend is not None and pair_wg_ok(pend[0], pend[1]) and \
                        ops.wide_pair_dgrad_ok(rows, out_f, in_f):
                    ops.wide_pair(wg_of(*pend), fz, dgrad=dg)
                else:
                    if pend is not None:
                        issue_wgrad(*pend)
                    ops.linear_dgrad(*dg)
                pend = None
                dz = dz_next
            if pend is not None:            # i == 0: the last two weight gradients
                if pair_wg_ok(pend[0], pend[1]) and pair_wg_ok(i, dz_i):
                    ops.wide_pair(wg_of(*pend), fz, wgrad2=wg_of(i, dz_i, x_in), sgd2=fz)
                    pend = None
                    continue
                issue_wgrad(*pend)
            pend = (i, dz_i, x_in)
        if pend is not None:
            issue_wgrad(*pend)
        self._mark("bwd")
        for i in unfused:
            s, e = ar.layer_range[i]
            ops.sgd(ar, self.hp, self.nesterov, first, offset=s, numel=e - s)

    def uses_rowband(self, rows: Optional[int] = None) -> bool:
        """True when a step of ``rows`` rows (default: the loaded batch) runs the row-band step."""
        rows = self.rows if rows is None else rows
        return bool(self.rowband and (rows >= max(1, self.rowband_min_rows) or self.uses_rowband_split(rows)))

    def uses_rowband_split(self, rows: Optional[int] = None) -> bool:
        """True when a step of ``rows`` rows runs the column-split row-band kernel (small batches
        below the band kernel's threshold)."""
        rows = self.rows if rows is None else rows
        if not self.rowband or rows <= 0 or rows >= max(1, self.rowband_min_rows):
            return False
        if rows not in self._rb_split:
            w = self.spec.widths
            self._rb_split[rows] = bool(hasattr(self.ops, "rowband_split_ok") and self.ops.rowband_split_ok(
                rows, w[1], w[0], self.L - 1, self.act))
        return self._rb_split[rows]

    def check_device_errors(self):
        """Raise if a column-split row-band step gave up a bounded wait (a band's blocks were not
        all resident within 2 ms: its results are invalid).  Reads one device word (host sync)."""
        if self.ws_rb is not None and any(self._rb_split.values()) and hasattr(self.ops, "rowband_error_word"):
            i = self.ops.rowband_error_word()
            word = self.ws_rb[i:i + 1].view(torch.int32)
            if int(word.item()) != 0:
                # sticky until read: clear it so one timed-out step is reported once
                with torch.no_grad():
                    word.zero_()
                torch.cuda.synchronize(self.device)
                raise RuntimeError("row-band split step: a band's hand-off wait timed out (results invalid)")

    def schedule_name(self) -> str:
        """The step schedule a batch of the loaded size runs (bench / result reports)."""
        if self.uses_rowband():
            return "rowband_overlap" if self.rb_overlap else "rowband"
        if self.grouped:
            return "grouped"
        return "overlap" if self.overlap else "sequential"

    # Row-band schedule (see rowband.hip): three launches per step.  One rank: the combine
    # applies the SGD update; several ranks: the combine writes the gradient, then the inline
    # all-reduce (or ZeRO-1's reduce-scatter / all-gather) and the update follow.
    def _rb_images(self):
        """{layer: (forward image, dgrad image)} for an optimizer pass of a row-band step (the
        pass refreshes the v2 images it covers), else None."""
        if self.rb_packed is None or not self.uses_rowband():
            return None
        return dict(enumerate(self.rb_packed))

    def _rb_layers(self):
        rows, ar = self.rows, self.arena
        # (the last hidden layer's activations are consumed inside the band -- head and its
        # weight-gradient partials -- so the hot path does not copy them out; evaluation and the
        # other schedules recompute or write their own)
        last = self.L - 2
        return [(ar.compute_weight(i), ar.bias(i),
                 self.acts[i][:rows] if (i < last or self.rb_keep_last) else None, self._dzl(i, rows),
                 ar.grad_weight(i), ar.grad_bias(i)) for i in range(self.L - 1)]

    def _rb_launch(self, sgd=None, phase: int = 0):
        rows, ar, last = self.rows, self.arena, self.L - 1
        kw = {}
        if self.rb_packed is not None:
            if phase <= 1 and not self._rb_current():
                self._rb_pack()
            kw["packed"] = self.rb_packed
        self.ops.rowband_step(self.X[:rows], self._rb_layers(), ar.weight(last), ar.bias(last),
                              self.Y[:rows], self.inv_count, ar.grad_weight(last),
                              ar.grad_bias(last), self.ws_rb, self.loss_scale, self.loss_out,
                              self.act, sgd=sgd, phase=phase, plan=self.rb_plan,
                              split=1 if self.uses_rowband_split(rows) else 0, **kw)

    # Row-band step with per-bucket collectives on the comm stream (several ranks): the band
    # launch and the last hidden layer's + the head's weight gradients first (phase 1); their
    # bucket's all-reduce -- and its SGD, which also refreshes that layer's v2 images -- run on
    # the comm stream while the other layers' weight gradients compute (phase 2); the buckets
    # those complete follow.  Every weight's last reader is the band launch.
    def _step_body_rowband_overlap(self, first: bool):
        ar, L, main = self.arena, self.L, self.stream
        self.sync.begin()
        self._sgd_done = set()
        self._reduced = {}
        self._pending_sgd = []
        self._written16 = []
        self._waited = set()
        self._first = first
        self._rb_launch(phase=1)
        for l in range(L):
            main.record_event(self.ev_wfree[l])
        self._mark("bwd_tail")
        self._layer_done(L - 1, main)
        self._layer_done(L - 2, main)
        if L > 2:
            self._rb_launch(phase=2)
            for i in range(L - 3, -1, -1):
                self._layer_done(i, main)
        self._mark("bwd")
        self._join_comm()
        self._mark("comm")
        for b in ar.buckets:
            if b.index not in self._sgd_done:
                self.ops.sgd(ar, self.hp, self.nesterov, first, offset=b.offset, numel=b.numel,
                             **self._upd_kw())
        self._rb_fresh = self.rb_packed is not None

    def _step_body_rowband(self, first: bool):
        rows, ops, ar, L = self.rows, self.ops, self.arena, self.L
        if self.rb_overlap:
            return self._step_body_rowband_overlap(first)
        fz = ops.sgd_fusion(ar, self.hp, self.nesterov, first) if self.fuse_sgd else None
        self._rb_launch(sgd=fz)
        # the fused combine rewrote the images from the updated weights; the multi-rank update
        # below does not
        self._rb_fresh = fz is not None
        self._mark("bwd")
        if fz is not None:
            return
        if self.sharded:
            self._update(first)
            return
        self.sync.begin()
        for b in ar.buckets:
            self.sync.launch_bucket(b, self.stream)
        self.sync.finish()
        self._mark("comm")
        # (every gradient element the pass reads is rewritten by the next step's launches -- the
        # combines store whole layer gradients, the arena's padding is never written and stays
        # zero -- so the pass does not zero the gradient behind itself: 3 MB less to write on the
        # 512-wide proxy)
        if self.rb_packed is not None:
            # the optimizer pass also rewrites the v2 weight images from the updated weights
            ops.sgd(ar, self.hp, self.nesterov, first, zero_grad=False,
                    images=dict(enumerate(self.rb_packed)))
            self._rb_fresh = True
        else:
            ops.sgd(ar, self.hp, self.nesterov, first, zero_grad=False)

    # Grouped schedule: the backward of layer i is ONE launch holding three independent jobs —
    # dgrad_i, wgrad_i (split-K partial slabs) and the slab combine of layer i+1 (with the SGD
    # update fused on a single rank) — so each job's tail is filled by the others' blocks and
    # the step has L+1 fewer launch gaps.  Hazards: combine_{i+1} updates W_{i+1}, which no job
    # of the group reads (dgrad_i reads W_i); the two slab workspaces alternate.
    def _step_body_grouped(self, first: bool):
        rows, ops, ar, L = self.rows, self.ops, self.arena, self.L
        fz = ops.sgd_fusion(ar, self.hp, self.nesterov, first) if self.fuse_sgd else None
        comm = self.comm_overlap
        main = self.stream
        if comm:
            # several ranks, per-bucket collectives: each combine's finished layer gradient goes
            # straight to its bucket's all-reduce on the comm stream (its SGD follows there)
            # while the next grouped launch computes
            self.sync.begin()
            self._sgd_done = set()
            self._reduced = {}
            self._pending_sgd = []
            self._written16 = []
            self._first = first
        x = self.X[:rows]
        h = self._forward(x)
        self._mark("fwd")
        last = L - 1
        dz = self._dzl(last - 1, rows)
        unfused = []
        pending_layer = last
        if ops.head_can_fuse_sgd(self.spec.widths[-1], self.spec.widths[-2], self.loss_kind):
            pending = ops.head_deferred(
                h, ar.weight(last), ar.bias(last), self.Y[:rows] if self.Y is not None else None,
                self.inv_count, self.act, dz, ar.grad_weight(last), ar.grad_bias(last),
                self.loss_out, self.loss_scale, self.ws_pair[0], sgd=fz,
                labels=self.labels[:rows] if self.labels is not None else None,
                loss=self.loss_kind, dlogits=self.dlogits[:rows])
        else:
            self._head(h, dz)
            pending = None
            pending_layer = None          # the head's gradient is already final
            unfused.append(last)
            if comm:
                main.record_event(self.ev_wfree[last])
                self._layer_done(last, main)
        self._mark("head")
        for i in range(L - 2, -1, -1):
            x_in = self.acts[i - 1][:rows] if i > 0 else x
            dgrad = None
            dz_i = dz
            if i > 0:
                dz = self._dzl(i - 1, rows)
                dgrad = (dz_i, ar.compute_weight(i), self.acts[i - 1][:rows], self.act, dz)
            out_f, in_f = self.spec.layer_shape(i)
            fuse = fz is not None and ops.wgrad_can_fuse_sgd(rows, out_f, in_f, self.dtype)
            if not fuse:
                unfused.append(i)
            pending = ops.bwd_group(dgrad, (dz_i, x_in, ar.grad_weight(i), ar.grad_bias(i),
                                            self.ws_pair[(last - i) % 2]),
                                    fz if fuse else None, pending)
            if comm and pending_layer == i + 1:
                # this launch held combine_{i+1}: layer i+1's gradient is final, and its
                # weights' last reader (dgrad_{i+1} / the head) ran in an earlier launch
                main.record_event(self.ev_wfree[i + 1])
                self._layer_done(i + 1, main)
            pending_layer = i
        ops.slab_reduce(pending)
        self._mark("bwd")
        if comm:
            main.record_event(self.ev_wfree[0])
            self._layer_done(0, main)
            self._join_comm()
            self._mark("comm")
            for b in ar.buckets:
                if b.index not in self._sgd_done:
                    ops.sgd(ar, self.hp, self.nesterov, first, offset=b.offset, numel=b.numel,
                            **self._upd_kw())
            return
        if fz is not None:
            for i in unfused:
                s, e = ar.layer_range[i]
                ops.sgd(ar, self.hp, self.nesterov, first, offset=s, numel=e - s)
            return
        if self.sharded:
            self._update(first)
            return
        self.sync.begin()
        for b in ar.buckets:
            self.sync.launch_bucket(b, self.stream)
        self.sync.finish()
        self._mark("comm")
        ops.sgd(ar, self.hp, self.nesterov, first)

    def _bucket_reduce(self, b, stream):
        """Launch bucket b's collective (once); returns the stream it completes on.  One queued
        bucket update is issued behind every new collective, so the comm stream alternates
        collectives and updates instead of parking a later collective behind an update that
        waits for its weights' last reader."""
        if b.index not in self._reduced:
            if self._upd_grad is not None:
                # bf16 payload: the bucket's update reads the reduced bf16 gradient directly
                self._reduced[b.index] = self.sync.launch_bucket(
                    b, stream, cast_back=False, written=self._written16)
            else:
                self._reduced[b.index] = self.sync.launch_bucket(b, stream)
            if b.index in self.ev_ar and self._reduced[b.index] is not None:
                self._reduced[b.index].record_event(self.ev_ar[b.index])
            self._flush_sgd(1)
        return self._reduced[b.index]

    def _layer_done(self, layer: int, stream):
        """Layer ``layer``'s gradient is final and ev_wfree[layer] is recorded: reduce every
        bucket it completes and queue each bucket's SGD (on the stream its collective completes
        on, behind the last reader of its weights).  Updates stay on the comm stream itself: a
        third stream in a step graph whose capture origin is the comm stream crashes hipGraph
        instantiation on ROCm 7 (measured at 1 and 2 ranks: docs/PERF.md §3)."""
        for b in self.arena.buckets_completed_by(layer):
            rs = self._bucket_reduce(b, stream)
            if rs is None or rs is stream:
                continue   # reduced on this stream already (single rank): update once at the end
            self._pending_sgd.append((b, rs))
            self._sgd_done.add(b.index)

    def _flush_sgd(self, n: Optional[int] = None):
        # (updates planned into a later weight-gradient epilogue stay queued for it;
        # _join_comm runs whatever is left)
        while n is None or n > 0:
            k = next((k for k, (pb, _) in enumerate(self._pending_sgd)
                      if pb.index not in self._defer_targets), None)
            if k is None:
                break
            b, rs = self._pending_sgd.pop(k)
            with torch.cuda.stream(rs):
                for l in b.layers:
                    rs.wait_event(self.ev_wfree[l])
                self.ops.sgd(self.arena, self.hp, self.nesterov, self._first, offset=b.offset,
                             numel=b.numel, **self._upd_kw())
            if n is not None:
                n -= 1

    def _upd_kw(self):
        kw = {} if self._upd_grad is None else {"grad_bf16": self._upd_grad}
        img = self._rb_images()
        if img is not None:
            kw["images"] = img
        return kw

    def _join_comm(self):
        """Join the comm stream into the compute stream.  Updates still queued at this point
        (the last buckets) run after the join on the compute stream, merged into one SGD launch
        per contiguous range, instead of as a serial tail of small launches on the comm stream
        in front of the join."""
        tail = self._pending_sgd
        self._pending_sgd = []
        self.sync.finish()   # joins the comm stream into the compute stream
        tail.sort(key=lambda br: br[0].offset)
        i = 0
        while i < len(tail):
            s0 = tail[i][0].offset
            e0 = s0 + tail[i][0].numel
            j = i + 1
            while j < len(tail) and tail[j][0].offset == e0:
                e0 += tail[j][0].numel
                j += 1
            self.ops.sgd(self.arena, self.hp, self.nesterov, self._first, offset=s0,
                         numel=e0 - s0, **self._upd_kw())
            i = j

    def step(self):
        """One optimizer step on the loaded batch.  Asynchronous on the GPU."""
        first = self.steps_done == 0
        if not self.is_cuda:
            self._step_body(first)
        else:
            with torch.cuda.stream(self.stream):
                if first or not self.use_graph or self.timer is not None:
                    self._step_body(first)
                else:
                    # scales are baked into the captured launches -> part of the key
                    key = (self.rows, self.inv_count, self.loss_scale)
                    g = self._graphs.get(key)
                    if g is None:
                        try:
                            g = self._capture()
                        except RuntimeError as e:   # e.g. a collective that cannot be captured
                            import sys
                            print(f"[nnmpi] hipGraph capture failed ({e}); running eagerly",
                                  file=sys.stderr, flush=True)
                            self.use_graph = False
                            self._step_body(False)
                            self.steps_done += 1
                            return
                        self._graphs[key] = g
                    g.launch(int(self.stream.cuda_stream))
        self.steps_done += 1

    # ---------------- multi-step graphs ------------------------------------------------------
    # A hipGraph replay has a fixed cost (~8 us measured between consecutive replays on MI355X,
    # MI355X_MICROARCH.md "graph-replay-floor"), which is ~8 % of a 512-wide step.  When the
    # host has nothing to do between steps (a timed loop, full-batch epochs without per-step
    # output) the engine can replay graphs holding `chunk` complete consecutive steps.
    def _chunks(self, n: int, chunk: int):
        out = []
        while n > 0:
            c = min(chunk, n)
            out.append(c)
            n -= c
        return out

    def prepare_steps(self, n: int, chunk: int = 16, losses: bool = False):
        """Capture (without running) every graph that run_steps(n, chunk) will replay
        (``losses``: the form that records every step's loss, see run_steps)."""
        if not (self.is_cuda and self.use_graph and self.timer is None and self.steps_done > 0):
            return
        with torch.cuda.stream(self.stream):
            for c in set(self._chunks(n, chunk)):
                key = (self.rows, self.inv_count, self.loss_scale, c, losses)
                if key not in self._graphs:
                    self._graphs[key] = self._capture(c, hist=losses)

    def run_steps(self, n: int, chunk: int = 16, losses: Optional[torch.Tensor] = None):
        """n optimizer steps (asynchronous on the GPU).  In graph mode the steps are replayed as
        graphs of up to `chunk` consecutive steps; results are identical to n step() calls.

        ``losses``: a device fp32 tensor of >= n entries; step k's loss (what loss() would
        return right after it) lands in losses[k] -- per-step losses without a host sync per
        step (the compat trainer's full-batch epochs).  Written on the engine's stream:
        synchronize() before reading them on the host."""
        k0 = 0

        def keep(k):
            if losses is not None:
                losses[k:k + 1].copy_(self.loss_out[:1])
        if not (self.is_cuda and self.use_graph and self.timer is None):
            ctx = torch.cuda.stream(self.stream) if self.is_cuda else _nullctx()
            for k in range(n):
                self.step()
                with ctx:
                    keep(k)
            return
        if n > 0 and self.steps_done == 0:
            self.step()          # eager first step (momentum initialisation semantics)
            with torch.cuda.stream(self.stream):
                keep(0)
            n -= 1
            k0 = 1
        hist = losses is not None
        try:
            self.prepare_steps(n, chunk, losses=hist)
        except RuntimeError:
            for k in range(n):   # capture unavailable: step() falls back to eager by itself
                self.step()
                with torch.cuda.stream(self.stream):
                    keep(k0 + k)
            return
        with torch.cuda.stream(self.stream):
            for c in self._chunks(n, chunk):
                self._graphs[(self.rows, self.inv_count, self.loss_scale, c, hist)].launch(
                    int(self.stream.cuda_stream))
                if hist:
                    losses[k0:k0 + c].copy_(self._loss_hist[:c])
                self.steps_done += c
                k0 += c

    def run_epoch(self, X: torch.Tensor, Y: Optional[torch.Tensor],
                  labels: Optional[torch.Tensor], perm: torch.Tensor, plan) -> None:
        """One mini-batch epoch as ONE graph replay: for every ``(lo, hi, inv_count, loss_scale,
        grad_scale)`` of ``plan`` the rows ``perm[lo:hi]`` of the resident shard are gathered
        into the input buffers and a step is taken with those scales -- exactly what
        load_batch_indexed + set_scales + step() do per step, with the per-step host work
        gone.  ``perm`` must be the same device buffer every epoch (rewrite its contents; the
        graph holds its address).  Falls back to those per-step calls when graphs are off or
        no step has run yet."""
        plan = [tuple(p) for p in plan]

        def body():
            for lo, hi, inv, lsc, gsc in plan:
                self.load_batch_indexed(X, Y, labels, perm[lo:hi])
                self.set_scales(inv, lsc, gsc)
                self._step_body(False)
        if not (self.is_cuda and self.use_graph and self.timer is None and self.steps_done > 0):
            for lo, hi, inv, lsc, gsc in plan:
                self.load_batch_indexed(X, Y, labels, perm[lo:hi])
                self.set_scales(inv, lsc, gsc)
                self.step()
            return
        key = ("epoch", tuple(plan), X.data_ptr(), perm.data_ptr(),
               None if Y is None else Y.data_ptr(), None if labels is None else labels.data_ptr())
        with torch.cuda.stream(self.stream):
            g = self._graphs.get(key)
            if g is None:
                g = self._capture_fn(body)
                self._graphs[key] = g
            else:
                # the host-side state the per-step calls would leave behind (rows, scales)
                lo, hi, inv, lsc, gsc = plan[-1]
                self.rows = hi - lo
                self.inv_count, self.loss_scale = float(inv), float(lsc)
            g.launch(int(self.stream.cuda_stream))
        self.steps_done += len(plan)

    def _capture(self, nsteps: int = 1, hist: bool = False):
        """One graph of ``nsteps`` consecutive steps; ``hist``: step k also copies its loss into
        self._loss_hist[k] (a node inside the graph)."""
        if hist:
            # allocated once: captured graphs keep writing to this address
            if getattr(self, "_loss_hist", None) is None:
                self._loss_hist = torch.zeros(LOSS_HIST_MAX, dtype=torch.float32, device=self.device)
            if nsteps > LOSS_HIST_MAX:
                raise ValueError(f"loss-recording graphs hold at most {LOSS_HIST_MAX} steps")

        def body():
            for k in range(nsteps):
                self._step_body(False)
                if hist:
                    self._loss_hist[k:k + 1].copy_(self.loss_out[:1])
        return self._capture_fn(body)

    def _capture_fn(self, body):
        """Capture ``body()`` (work on the engine's streams) as one replayable graph."""
        from .. import native
        g = native.lib().GraphRunner()
        # the row-band image state the captured body assumes at its start, and leaves behind
        rb_pre = (self._rb_fresh, self._rb_ver)
        origin = self.sync.capture_origin()
        if origin is None:
            origin = self.stream
        g.begin(int(origin.cuda_stream))
        self.sync.record(True)
        try:
            if origin is not self.stream:
                # collectives live on the comm stream: it is the capture origin, the compute
                # stream forks from it here and joins back below (see GradSync.capture_origin)
                self.stream.wait_stream(origin)
            body()
            if origin is not self.stream:
                origin.wait_stream(self.stream)
        except Exception:
            self.sync.record(False)
            g.cancel()    # leave the stream out of capture mode, drop the partial graph
            self._rb_fresh, self._rb_ver = rb_pre
            raise
        # (record(False) rolls the sequence number and the signature back: the capture issued
        # these collectives once, but every launch runs them, and the launch adds them to the
        # collective signature -- utils/seqcheck.py)
        notes = self.sync.record(False)
        g.end()
        rb_post = self._rb_fresh
        self._rb_fresh, self._rb_ver = rb_pre     # nothing ran yet
        return _Graph(g, self.sync, notes, self,
                      rb_pre[0] and rb_pre[1] == self.arena.version, rb_post)

    # ---------------- gradient accumulation ----------------------------------------------------
    # Not in the reference (one backward per step, SURVEY.md §2.3 "optional").  A step over more
    # rows than fit the activation buffers is cut into micro-batches: each runs the sequential
    # forward/backward kernels with communication and the optimizer switched off and its
    # gradient is added into an fp32 accumulation arena; the step's gradient synchronisation
    # and update then run ONCE on the sum.  set_scales() must carry the row count of the whole
    # step (inv_count = 1/rows_step), so the sum is the step's mean gradient and the summed
    # micro-batch losses are the step's mean loss.
    def accumulate(self):
        """Forward + backward of the loaded micro-batch; gradient and loss are added to the
        accumulators (asynchronous on the GPU)."""
        ar = self.arena
        if not hasattr(self, "_acc"):
            self._acc = torch.zeros_like(ar.grad)
            self._acc_loss = torch.zeros(1, dtype=torch.float32, device=self.device)
            self._n_acc = 0
        ctx = torch.cuda.stream(self.stream) if self.is_cuda else _nullctx()
        with ctx, torch.no_grad():
            sync, tiny_fused = self.sync, self.tiny_fused
            self.sync, self.tiny_fused = _SilentSync(), False
            try:
                self.forward_backward()
            finally:
                self.sync, self.tiny_fused = sync, tiny_fused
            if self._n_acc == 0:
                self._acc.copy_(ar.grad)
                self._acc_loss.copy_(self.loss_out[:1])
            else:
                self._acc.add_(ar.grad)
                self._acc_loss.add_(self.loss_out[:1])
        self._n_acc += 1

    def apply_accumulated(self):
        """Gradient synchronisation + optimizer update on the accumulated gradient: one optimizer
        step (steps_done += 1).  The accumulators restart empty."""
        if not getattr(self, "_n_acc", 0):
            raise RuntimeError("apply_accumulated() without a preceding accumulate()")
        first = self.steps_done == 0
        ar = self.arena
        ctx = torch.cuda.stream(self.stream) if self.is_cuda else _nullctx()
        with ctx, torch.no_grad():
            ar.grad.copy_(self._acc)
            self.loss_out[:1].copy_(self._acc_loss)
            self._first = first
            self.sync.begin()
            for i in reversed(range(self.L)):
                self.sync.ready(i)
            self.sync.finish()
            self._update(first)
        self._rb_fresh = False
        self._n_acc = 0
        self.steps_done += 1

    # ---------------- evaluation (forward only) ---------------------------------------------
    def evaluate(self, X: torch.Tensor, Y: Optional[torch.Tensor] = None,
                 labels: Optional[torch.Tensor] = None):
        """Forward-only loss over held-out rows, chunked by the row capacity.  Parameters and
        optimizer state are untouched (the head's gradient outputs go to scratch buffers and no
        optimizer fusion is requested).  The training batch in the input buffers is overwritten:
        reload it before the next step.  Returns (sum of per-row losses, rows); the reference's
        validation/test hooks are dead code (ref.py:213-236)."""
        n = X.shape[0]
        if n == 0:
            return 0.0, 0
        out_f = self.spec.widths[-1]
        per = out_f if self.loss_kind == "mse" else 1
        if not hasattr(self, "_eval_gw"):
            last = self.L - 1
            self._eval_gw = torch.zeros_like(self.arena.grad_weight(last))
            self._eval_gb = torch.zeros_like(self.arena.grad_bias(last))
        total = 0.0
        ctx = torch.cuda.stream(self.stream) if self.is_cuda else _nullctx()
        for lo in range(0, n, self.R):
            hi = min(n, lo + self.R)
            self.load_batch(X[lo:hi], Y[lo:hi] if Y is not None else None,
                            labels[lo:hi] if labels is not None else None)
            rows = self.rows
            with ctx, torch.no_grad():
                if self.use_tiny:
                    # the one-block kernel's mean loss (its gradient output is rewritten by the
                    # next training step; no optimizer fusion here)
                    self.ops.tiny_step(self.spec, self.arena, self.X[:rows],
                                       self.Y[:rows] if self.Y is not None else None,
                                       self.labels[:rows] if self.labels is not None else None,
                                       1.0 / (rows * per), self.loss_out, self.ws, sgd=None)
                    scale = rows * per
                else:
                    h = self._forward(self.X[:rows])
                    last = self.L - 1
                    self.ops.head(h, self.arena.weight(last), self.arena.bias(last),
                                  self.Y[:rows] if self.Y is not None else None,
                                  self.labels[:rows] if self.labels is not None else None,
                                  self.loss_kind, 0.0, self.act if self.L > 1 else "none", None,
                                  self._eval_gw, self._eval_gb, self.dlogits[:rows], self.loss_out,
                                  1.0, ws=self.ws)
                    scale = 1.0
            total += self.loss() * scale
        return total, n

    def loss(self) -> float:
        """Local (this rank's) mean loss of the last step (host sync)."""
        if self.is_cuda:
            self.stream.synchronize()
        self.check_device_errors()
        return float(self.loss_out[0].item())

    def synchronize(self, check: bool = True):
        """Wait for the engine's stream.  ``check``: then raise if a column-split row-band step
        gave up a hand-off wait since the last check (one device word read; only once a split
        step has run) -- every host sync of the training paths sees a timed-out step instead of
        training on.  A timed region passes check=False and calls check_device_errors() after
        its clock stops."""
        if self.is_cuda:
            self.stream.synchronize()
            if check:
                self.check_device_errors()

    @property
    def flops_per_step(self) -> float:
        return float(self.spec.flops_per_sample()) * self.rows


class _Graph:
    """A captured graph plus the collectives it issues per launch (for the signature) and the
    row-band weight-image state it was captured under: a body captured with current images
    skips their rebuild, so before it replays on stale images they are rebuilt eagerly."""

    def __init__(self, runner, sync, notes, engine=None, rb_pre: bool = False,
                 rb_post: bool = False):
        import weakref
        self.runner, self.sync, self.notes = runner, sync, notes
        # (a weak reference: engine -> _graphs -> graph -> engine would be a cycle, freed by the
        # garbage collector in arbitrary order at teardown -- a graph holding RCCL kernels then
        # outlives its communicator, and the teardown of the two hung a 2-rank RCCL job)
        self._eng = weakref.ref(engine) if engine is not None else (lambda: None)
        self.rb_pre, self.rb_post = rb_pre, rb_post

    def launch(self, stream_handle: int):
        eng = self._eng()
        if eng is not None and eng.rb_packed is not None and self.rb_pre and not eng._rb_current():
            with torch.cuda.stream(eng.stream):
                eng._rb_pack()
        self.runner.launch(stream_handle)
        self.sync.replay(self.notes)
        if eng is not None:
            eng._rb_fresh, eng._rb_ver = self.rb_post, eng.arena.version


class _SilentSync:
    """Stand-in for the gradient sync while a micro-batch's gradient is produced."""

    def ready(self, layer: int):
        pass


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
