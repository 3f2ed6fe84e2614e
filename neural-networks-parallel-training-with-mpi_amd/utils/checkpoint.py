"""Checkpoint / resume.

The reference never saves anything; its only serialised model form is the
pickled ``state_dict`` it broadcasts at init (ref.py:87).  The framework writes:

* ``<path>`` — ``torch.save(state_dict)`` with the reference keys ``layers.{i}.weight/bias``
  (loadable by the reference ``MLP().load_state_dict`` and by ``torch.load(weights_only=True)``);
* ``<path>.train`` — resume state: the momentum of every parameter keyed by its reference name
  (unpadded, so it re-lays into ANY arena: another world size, with or without the sharded
  optimizer's padding), epoch, step counter, config (all tensors / plain types, so it also
  loads with ``weights_only=True``).
Writes are atomic (tmp file + rename) and done by rank 0 only.  A resume whose optimizer state
does not fit the model raises instead of silently restarting the momentum from zero.
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
        "momentum_by_name": {k: v.detach().cpu().clone()
                             for k, v in _momentum_views(arena).items()},
        "epoch": int(epoch),
        "steps": int(steps),
        "numel": int(arena.numel),
        "config": {k: (v if isinstance(v, (int, float, str, bool, type(None))) else str(v))
                   for k, v in (dataclasses.asdict(cfg).items() if cfg is not None else [])},
    }
    _atomic_save(train, path + ".train")


def load_state_dict(path: str):
    return torch.load(path, map_location="cpu", weights_only=True)


def _momentum_views(arena):
    """name -> the momentum of that parameter (a view of the arena's momentum buffer)."""
    out = {}
    for li in range(arena.n_layers):
        out[f"layers.{2 * li}.weight"] = arena.weight(li, arena.momentum)
        out[f"layers.{2 * li}.bias"] = arena.bias(li, arena.momentum)
    return out


def load_training_state(path: str, arena):
    """Load weights (+ momentum/epoch if ``<path>.train`` exists).  Returns (epoch, steps).
    Raises ValueError when the saved optimizer state does not match the model."""
    arena.load_state_dict(load_state_dict(path))
    tp = path + ".train"
    if not os.path.exists(tp):
        return 0, 0
    st = torch.load(tp, map_location="cpu", weights_only=True)
    views = _momentum_views(arena)
    with torch.no_grad():
        if "momentum_by_name" in st:
            saved = st["momentum_by_name"]
            if set(saved) != set(views):
                raise ValueError(f"{tp}: momentum for {sorted(saved)}, model has {sorted(views)}")
            for k, v in views.items():
                if tuple(saved[k].shape) != tuple(v.shape):
                    raise ValueError(f"{tp}: momentum of {k} has shape {tuple(saved[k].shape)}, "
                                     f"the model's is {tuple(v.shape)}")
                v.copy_(saved[k].to(v.device))
        elif "momentum" in st:   # flat arena image (older checkpoints): same layout only
            m = st["momentum"]
            if m.numel() != arena.numel:
                raise ValueError(f"{tp}: flat momentum of {m.numel()} elements does not fit an "
                                 f"arena of {arena.numel} (older checkpoint format)")
            arena.momentum.copy_(m.to(arena.momentum.device))
    return int(st.get("epoch", 0)), int(st.get("steps", 0))
