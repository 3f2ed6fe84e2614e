"""Checkpoint / resume.

The reference never saves anything; its only serialised model form is the
pickled ``state_dict`` it broadcasts at init (ref.py:87).  The framework writes:

* ``<path>`` — ``torch.save(state_dict)`` with the reference keys ``layers.{i}.weight/bias``
  (loadable by the reference ``MLP().load_state_dict`` and by ``torch.load(weights_only=True)``);
* ``<path>.train`` — resume state: momentum arena, epoch, step counter, config (all tensors /
  plain types, so it also loads with ``weights_only=True``).
Writes are atomic (tmp file + rename) and done by rank 0 only.
"""
from __future__ import annotations

import dataclasses
import os

import torch


def _atomic_save(obj, path: str):
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save(path: str, arena, epoch: int, steps: int, cfg=None):
    sd = {k: v.detach().cpu() for k, v in arena.state_dict().items()}
    _atomic_save(sd, path)
    train = {
        "momentum": arena.momentum.detach().cpu().clone(),
        "epoch": int(epoch),
        "steps": int(steps),
        "numel": int(arena.numel),
        "config": {k: (v if isinstance(v, (int, float, str, bool, type(None))) else str(v))
                   for k, v in (dataclasses.asdict(cfg).items() if cfg is not None else [])},
    }
    _atomic_save(train, path + ".train")


def load_state_dict(path: str):
    return torch.load(path, map_location="cpu", weights_only=True)


def load_training_state(path: str, arena):
    """Load weights (+ momentum/epoch if ``<path>.train`` exists).  Returns (epoch, steps)."""
    arena.load_state_dict(load_state_dict(path))
    tp = path + ".train"
    if not os.path.exists(tp):
        return 0, 0
    st = torch.load(tp, map_location="cpu", weights_only=True)
    if int(st.get("numel", -1)) == arena.numel:
        arena.momentum.copy_(st["momentum"].to(arena.momentum.device))
    return int(st.get("epoch", 0)), int(st.get("steps", 0))
