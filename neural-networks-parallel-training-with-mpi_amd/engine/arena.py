"""Flat parameter / gradient / optimizer-state arena.

All parameters of the MLP live in ONE contiguous fp32 buffer (the master weights), with a
gradient buffer, a momentum buffer and (for bf16 compute) a bf16 shadow copy of identical
layout.  Tensors are laid out in **reverse layer order** — ``[W_{L-1}, b_{L-1}, ..., W_0,
b_0]`` — so the gradients that backward produces first are at the front and every
communication bucket is one contiguous range in backward order.  Each tensor
starts on a 64-element (256-byte) boundary so kernels can use 16-byte vector accesses.

Replaces the reference's per-parameter ``param.grad`` lists that are pickled to the root
(``ref.py:179-185``) and the per-tensor SGD loop (``ref.py:211``): the optimizer, the
all-reduce and checkpointing all operate on flat ranges.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
from ..utils.knobs import knob

ALIGN = 64  # elements


def _align(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


@dataclass(frozen=True)
class Slot:
    name: str
    layer: int
    kind: str          # "weight" | "bias"
    offset: int
    shape: Tuple[int, ...]

    @property
    def numel(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n


@dataclass(frozen=True)
class Bucket:
    index: int
    layers: Tuple[int, ...]   # layer ids in backward order (descending)
    offset: int
    numel: int
    rows: Optional[Tuple[int, int]] = None   # sub-layer bucket: output rows [r0, r1) of layers[0]


# A layer whose gradient is larger than one bucket is cut into output-row chunks, each its own
# bucket, so its all-reduce can start while the rest of that layer's weight gradient is still
# being computed (the last layer of backward is otherwise one fully exposed collective).  The
# chunk count keeps every chunk's weight-gradient GEMM a full wave of 256x256 tiles on the
# 256 CUs (rows per chunk a multiple of 256, >= 256 tiles per chunk).
CHUNK_TILE = 256
CHUNK_MIN_TILES = 256


def row_chunks(out_f: int, in_f: int, grad_bytes: int, bucket_bytes: float,
               min_tiles: int = 0) -> int:
    if grad_bytes <= bucket_bytes or out_f % CHUNK_TILE or in_f % CHUNK_TILE:
        return 1
    # min_tiles: tiles per chunk at least (0: NNMPI_CHUNK_MIN_TILES, else CHUNK_MIN_TILES; tests
    # exercise the chunked schedule on small layers, bench.py tunes 2 vs 4 chunks per layer)
    if min_tiles <= 0:
        min_tiles = int(knob("NNMPI_CHUNK_MIN_TILES", CHUNK_MIN_TILES))
    c = 1
    while (out_f % (2 * c * CHUNK_TILE) == 0 and
           (out_f // (2 * c * CHUNK_TILE)) * (in_f // CHUNK_TILE) >= min_tiles):
        c *= 2
    return c


class Arena:
    def __init__(self, layer_shapes: List[Tuple[int, int]], device, shadow_dtype=None,
                 bucket_bytes: float = 25 * 2 ** 20, grad_elem_bytes: int = 4, pad_to: int = ALIGN,
                 chunk_layers: bool = True, chunk_min_tiles: int = 0):
        """``pad_to``: the total length is rounded up to this multiple (a multiple of ALIGN) --
        the sharded optimizer uses ``world * ALIGN`` so every rank owns an equal, aligned shard.
        ``chunk_layers``: cut layers larger than a bucket into output-row chunk buckets."""
        self.layer_shapes = list(layer_shapes)
        self.n_layers = len(layer_shapes)
        self.version = 0
        self.device = torch.device(device)
        slots: List[Slot] = []
        off = 0
        self.layer_range: Dict[int, Tuple[int, int]] = {}
        for li in reversed(range(self.n_layers)):
            out_f, in_f = layer_shapes[li]
            start = off
            slots.append(Slot(f"layers.{2 * li}.weight", li, "weight", off, (out_f, in_f)))
            off = _align(off + out_f * in_f)
            slots.append(Slot(f"layers.{2 * li}.bias", li, "bias", off, (out_f,)))
            off = _align(off + out_f)
            self.layer_range[li] = (start, off)
        self.slots = slots
        self.by_name = {s.name: s for s in slots}
        self.numel = _align(off, max(ALIGN, int(pad_to)))
        z = lambda dt: torch.zeros(self.numel, dtype=dt, device=self.device)  # noqa: E731
        self.master = z(torch.float32)
        self.grad = z(torch.float32)
        self.momentum = z(torch.float32)
        self.shadow: Optional[torch.Tensor] = z(shadow_dtype) if shadow_dtype is not None else None
        self.layer_chunks: Dict[int, int] = {}
        if chunk_layers:
            for li, (out_f, in_f) in enumerate(layer_shapes):
                c = row_chunks(out_f, in_f, out_f * in_f * grad_elem_bytes, bucket_bytes,
                               chunk_min_tiles)
                if c > 1:
                    self.layer_chunks[li] = c
        self.buckets = self._plan_buckets(bucket_bytes, grad_elem_bytes)

    # ---- views -------------------------------------------------------------------------
    def _view(self, buf: torch.Tensor, slot: Slot) -> torch.Tensor:
        return buf[slot.offset:slot.offset + slot.numel].view(slot.shape)

    def weight(self, li: int, buf: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self._view(self.master if buf is None else buf,
                          self.by_name[f"layers.{2 * li}.weight"])

    def bias(self, li: int, buf: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self._view(self.master if buf is None else buf,
                          self.by_name[f"layers.{2 * li}.bias"])

    def compute_weight(self, li: int) -> torch.Tensor:
        return self.weight(li, self.shadow if self.shadow is not None else self.master)

    def compute_bias(self, li: int) -> torch.Tensor:
        return self.bias(li, self.shadow if self.shadow is not None else self.master)

    def grad_weight(self, li: int) -> torch.Tensor:
        return self.weight(li, self.grad)

    def grad_bias(self, li: int) -> torch.Tensor:
        return self.bias(li, self.grad)

    # ---- model binding / state ------------------------------------------------------
    def load_from_model(self, model) -> None:
        lins = model.linears()
        assert len(lins) == self.n_layers
        with torch.no_grad():
            for li, lin in enumerate(lins):
                self.weight(li).copy_(lin.weight.detach().to(self.device, torch.float32))
                self.bias(li).copy_(lin.bias.detach().to(self.device, torch.float32))
        self.sync_shadow()

    def bind_model(self, model) -> None:
        """Make the model's parameters views of the master arena (state_dict == arena)."""
        self.load_from_model(model)
        for li, lin in enumerate(model.linears()):
            lin.weight.data = self.weight(li)
            lin.bias.data = self.bias(li)

    def sync_shadow(self) -> None:
        """Refresh the bf16 shadow after the master weights were written outside an optimizer
        step (model binding, state_dict load, broadcast).  Bumps ``version``: derived weight
        copies (the row-band v2 images, engine.py) are rebuilt before their next use."""
        self.version += 1
        if self.shadow is not None:
            self.shadow.copy_(self.master)

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """Reference-format state_dict (keys ``layers.{i}.weight/bias``), forward order."""
        out = {}
        for li in range(self.n_layers):
            out[f"layers.{2 * li}.weight"] = self.weight(li).detach().clone()
            out[f"layers.{2 * li}.bias"] = self.bias(li).detach().clone()
        return out

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        with torch.no_grad():
            for li in range(self.n_layers):
                self.weight(li).copy_(sd[f"layers.{2 * li}.weight"].to(self.device))
                self.bias(li).copy_(sd[f"layers.{2 * li}.bias"].to(self.device))
        self.sync_shadow()

    def flat_params_forward_order(self) -> torch.Tensor:
        """Parameters flattened in ``model.parameters()`` order (golden-value layout)."""
        parts = []
        for li in range(self.n_layers):
            parts += [self.weight(li).reshape(-1), self.bias(li).reshape(-1)]
        return torch.cat(parts)

    # ---- buckets ----------------------------------------------------------------------
    def _plan_buckets(self, bucket_bytes: float, elem_bytes: int,
                      min_bytes: float = 64 * 2 ** 10, chunked: bool = True) -> List[Bucket]:
        """Greedy grouping of consecutive layers (backward order) into contiguous buckets.  A
        bucket below ``min_bytes`` (the output layer: a few KB) is never closed on its own --
        it rides with the next layer instead of paying a collective's latency by itself.
        Layers in ``layer_chunks`` become one bucket per output-row chunk (the last chunk also
        holds the bias)."""
        cap = max(1, int(bucket_bytes // elem_bytes))
        minc = int(min_bytes // elem_bytes)
        buckets: List[Bucket] = []
        cur: List[int] = []
        cur_start = 0

        def close():
            end = self.layer_range[cur[-1]][1]
            buckets.append(Bucket(len(buckets), tuple(cur), cur_start, end - cur_start))

        for li in reversed(range(self.n_layers)):
            s, e = self.layer_range[li]
            nch = self.layer_chunks.get(li, 1) if chunked else 1
            if nch > 1:
                if cur:
                    close()
                    cur = []
                out_f, in_f = self.layer_shapes[li]
                per = out_f // nch
                for c in range(nch):
                    r0, r1 = c * per, (c + 1) * per
                    o0 = s + r0 * in_f
                    o1 = e if c == nch - 1 else s + r1 * in_f
                    buckets.append(Bucket(len(buckets), (li,), o0, o1 - o0, rows=(r0, r1)))
                continue
            if cur and (e - cur_start) > cap and (s - cur_start) >= minc:
                close()
                cur = []
            if not cur:
                cur_start = s
            cur.append(li)
        if cur:
            close()
        return buckets

    def replan_single_bucket(self):
        """One bucket over the whole arena (a serial all-reduce amortises the latency)."""
        self.buckets = [Bucket(0, tuple(reversed(range(self.n_layers))), 0, self.numel)]

    def bucket_of_layer(self, li: int) -> Bucket:
        """The bucket that holds the END of layer ``li`` (its bias): the one that completes
        when the layer's gradient is final."""
        s, e = self.layer_range[li]
        for b in self.buckets:
            if li in b.layers and b.offset < e <= b.offset + b.numel:
                return b
        raise KeyError(li)

    def buckets_completed_by(self, li: int) -> List[Bucket]:
        """Buckets whose every gradient is final once layer ``li``'s is (backward order: the
        layer with the smallest index in the bucket is produced last)."""
        return [b for b in self.buckets if li in b.layers and li == min(b.layers)]

    def chunk_buckets(self, li: int) -> List[Bucket]:
        return [b for b in self.buckets if b.rows is not None and b.layers == (li,)]
