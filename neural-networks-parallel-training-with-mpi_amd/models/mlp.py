"""MLP model definitions.

:class:`MLP` keeps the reference module surface (``ref.py:35-51``): an ``nn.Module`` with a
``layers`` ``nn.Sequential`` of ``Linear``/activation pairs, so its state_dict keys are
``layers.{2i}.weight`` / ``layers.{2i}.bias`` (the activation occupies the odd indices).
``MLP()`` with no arguments is exactly the reference 2→3→1 ReLU regressor with torch's
default init (kaiming-uniform weights, U(±1/√fan_in) biases).

The training engines never run this module's ``forward`` in the hot path; they bind its
parameters to views of a flat fp32 arena (:mod:`nnmpi_amd.engine.arena`) and run explicit
forward/backward schedules.  Because the parameters *are* the arena views, ``state_dict()``
and ``torch.save(model.state_dict())`` produce the reference-compatible format directly.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence

import torch
from torch import nn

ACTIVATIONS = {"relu": nn.ReLU, "tanh": nn.Tanh}


@dataclass(frozen=True)
class MLPSpec:
    widths: tuple
    activation: str = "relu"
    loss: str = "mse"

    @property
    def n_layers(self) -> int:
        return len(self.widths) - 1

    def layer_shape(self, i: int):
        """(out, in) of Linear layer i."""
        return (self.widths[i + 1], self.widths[i])

    def param_names(self, i: int):
        return (f"layers.{2 * i}.weight", f"layers.{2 * i}.bias")

    @property
    def n_params(self) -> int:
        return sum(o * k + o for o, k in (self.layer_shape(i) for i in range(self.n_layers)))

    def flops_per_sample(self) -> int:
        """fwd+bwd matmul FLOPs per sample (2 fwd + 4 bwd per MAC; no dgrad for layer 0)."""
        f = 0
        for i in range(self.n_layers):
            o, k = self.layer_shape(i)
            f += 2 * o * k * (3 if i > 0 else 2)
        return f


class MLP(nn.Module):
    """Multilayer Perceptron for regression (reference ref.py:35-51)."""

    def __init__(self, widths: Sequence[int] = (2, 3, 1), activation: str = "relu",
                 device=None):
        super().__init__()
        widths = list(widths)
        mods: List[nn.Module] = []
        for i in range(len(widths) - 1):
            mods.append(nn.Linear(widths[i], widths[i + 1], device=device))
            if i < len(widths) - 2:
                mods.append(ACTIVATIONS[activation]())
        self.widths = widths
        self.activation = activation
        self.layers = nn.Sequential(*mods)

    @property
    def spec(self) -> MLPSpec:
        return MLPSpec(tuple(self.widths), self.activation)

    def linears(self) -> List[nn.Linear]:
        return [m for m in self.layers if isinstance(m, nn.Linear)]

    def forward(self, x):
        """Forward pass."""
        return self.layers(x)


def reference_init(widths=(2, 3, 1), activation="relu", seed: int = 0, device=None) -> MLP:
    """Rank-0 init of the reference: ``torch.manual_seed(0)`` then ``MLP()`` (ref.py:69,84).

    With ``device=None`` the init runs on the CPU generator (bitwise the reference's values);
    large models may be initialised directly on the GPU (device generator, same seed on every
    rank, then broadcast from rank 0 as the reference does at ref.py:87).
    """
    dev = torch.device(device) if device is not None else torch.device("cpu")
    with torch.random.fork_rng(devices=[dev] if dev.type == "cuda" else []):
        torch.manual_seed(seed)
        m = MLP(widths, activation, device=dev)
    return m
