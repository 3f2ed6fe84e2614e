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

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

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


class Arena:
    def __init__(self, layer_shapes: List[Tuple[int, int]], device, shadow_dtype=None,
                 bucket_bytes: float = 25 * 2 ** 20, grad_elem_bytes: int = 4, pad_to: int = ALIGN):
        """``pad_to``: the total length is rounded up to this multiple (a multiple of ALIGN) --
        the sharded optimizer uses ``world * ALIGN`` so every rank owns an equal, aligned shard."""
        self.layer_shapes = list(layer_shapes)
        self.n_layers = len(layer_shapes)
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
    def _plan_buckets(self, bucket_bytes: float, elem_bytes: int) -> List[Bucket]:
        """Greedy grouping of consecutive layers (backward order) into contiguous buckets."""
        cap = max(1, int(bucket_bytes // elem_bytes))
        buckets: List[Bucket] = []
        cur: List[int] = []
        cur_start = 0
        for li in reversed(range(self.n_layers)):
            s, e = self.layer_range[li]
            if cur and (e - cur_start) > cap:
                buckets.append(Bucket(len(buckets), tuple(cur), cur_start,
                                      self.layer_range[cur[-1]][1] - cur_start))
                cur = []
            if not cur:
                cur_start = s
            cur.append(li)
        if cur:
            buckets.append(Bucket(len(buckets), tuple(cur), cur_start,
                                  self.layer_range[cur[-1]][1] - cur_start))
        return buckets

    def bucket_of_layer(self, li: int) -> Bucket:
        for b in self.buckets:
            if li in b.layers:
                return b
        raise KeyError(li)
