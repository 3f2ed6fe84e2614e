"""CPU op set with native steps for tiny models: :class:`TorchOps` plus the host twins of the
one-launch tiny-MLP step and the fused SGD pass (``csrc/host/tiny_host.cpp``).

BASELINE config 1 -- the reference's own 2 -> 3 -> 1 regressor, fp32, CPU ranks over gloo
(ref.py:41-45,72,155-211) -- is pure per-op overhead on the plain-PyTorch path: ~170 Python and
ATen calls per step for a few hundred flops.  Here the whole step (forward, loss, backward, and on
one rank the SGD-momentum update) is ONE native call.  With several ranks the update after the
all-reduce stays TorchOps' (ATen) pass, so the all-reduce and ZeRO-1 paths keep one update
formula and stay bitwise equal.  Every wider model keeps the TorchOps path, which stays the
numerics oracle (``NNMPI_EXPERIMENTS=1 NNMPI_CPU_NATIVE=0`` selects it for tiny models too).
"""
from __future__ import annotations

from ..utils.knobs import knob
import os

from .. import native
from .hip_ops import LOSS_CODES
from .torch_ops import ACT_CODES, TorchOps


def _p(t):
    return native.ptr(t)


def host_ops_enabled() -> bool:
    return knob("NNMPI_CPU_NATIVE", "1") != "0"


class HostOps(TorchOps):
    name = "host"

    def __init__(self, device="cpu"):
        super().__init__(device)
        self.lib = native.lib()

    # ---------------- whole tiny step ----------------
    def tiny_workspace_bytes(self, rows, numel) -> int:
        return 0

    def tiny_can_fuse_sgd(self, rows: int) -> bool:
        return True

    @staticmethod
    def sgd_fusion(arena, hp, nesterov: bool, first: bool):
        return (_p(arena.grad), _p(arena.master), _p(arena.momentum), 0, _p(hp), int(nesterov),
                int(first))

    def tiny_step(self, spec, arena, X, y, labels, inv_count, loss_out, ws, sgd=None,
                  loss_scale=None):
        L = spec.n_layers
        w_off = [arena.by_name[f"layers.{2 * i}.weight"].offset for i in range(L)]
        b_off = [arena.by_name[f"layers.{2 * i}.bias"].offset for i in range(L)]
        if loss_scale is None:
            rows = X.shape[0]
            loss_scale = 1.0 / rows if spec.loss == "xent" else 1.0 / (rows * spec.widths[-1])
        assert X.is_contiguous() and (y is None or y.is_contiguous())
        self.lib.tiny_mlp_step_host(list(spec.widths), w_off, b_off, ACT_CODES[spec.activation],
                                    LOSS_CODES[spec.loss], _p(arena.master), _p(X), _p(y),
                                    _p(labels), X.shape[0], float(inv_count), _p(arena.grad),
                                    arena.numel, _p(loss_out), float(loss_scale), sgd)
