"""Datasets and feature scaling.

:class:`RegressionDataset` keeps the reference constructor and item protocol
(``ref.py:12-30``): ``RegressionDataset(X, y, scale_data=True)``, ``len``, ``ds[i] -> (X[i],
y[i])``, float64 storage and an optional ``StandardScaler`` fit on the data it is given (which,
in the reference, is one rank's shard: per-shard scaling, defect D4).  Fixed defect D11: tensor
inputs are accepted (the reference silently leaves ``self.X`` unset for them).

:func:`scale_features` implements the three scaling modes of the framework:
``per_shard`` (reference), ``global`` (mean/std of the whole dataset through an all-reduce of
shard moments) and ``none``.
"""
from __future__ import annotations

import numpy as np
import torch


def _standardize_np(X: np.ndarray) -> np.ndarray:
    """sklearn ``StandardScaler().fit_transform`` semantics (ddof=0, zero-variance -> 1)."""
    if X.shape[0] == 0:
        return X.copy()
    from sklearn.preprocessing import StandardScaler
    return StandardScaler().fit_transform(X)


class RegressionDataset(torch.utils.data.Dataset):
    """Prepare the dataset for regression (reference ref.py:12-30)."""

    def __init__(self, X, y, scale_data=True):
        if torch.is_tensor(X):
            X = X.detach().cpu().numpy()
        if torch.is_tensor(y):
            y = y.detach().cpu().numpy()
        X = np.asarray(X)
        y = np.asarray(y)
        if scale_data:
            X = _standardize_np(X)
        self.X = torch.from_numpy(np.ascontiguousarray(X))
        self.y = torch.from_numpy(np.ascontiguousarray(y))

    def __len__(self):
        return len(self.X)

    def __getitem__(self, i):
        return self.X[i], self.y[i]


def shard_moments(X: torch.Tensor):
    """(count, sum, sum of squares) in float64 — the all-reduce payload for global scaling."""
    Xd = X.to(torch.float64)
    return (torch.tensor([float(X.shape[0])], dtype=torch.float64, device=X.device),
            Xd.sum(0), (Xd * Xd).sum(0))


def scale_features(X: torch.Tensor, mode: str, allreduce=None) -> torch.Tensor:
    """Standardize features of one shard.

    ``allreduce(t)`` sums a float64 tensor over ranks in place (only used for ``global``).
    Returns a new tensor with X's dtype and device.
    """
    if mode == "none":
        return X.clone()
    if mode == "per_shard":
        if X.device.type == "cpu" and X.dtype == torch.float64:
            return torch.from_numpy(_standardize_np(X.numpy()))
        n, s, ss = shard_moments(X)
    elif mode == "global":
        n, s, ss = shard_moments(X)
        if allreduce is not None:
            packed = torch.cat([n, s, ss])
            allreduce(packed)
            d = s.numel()
            n, s, ss = packed[:1], packed[1:1 + d], packed[1 + d:]
    else:
        raise ValueError(f"unknown scaling mode {mode!r}")
    cnt = float(n.item())
    if cnt == 0:
        return X.clone()
    mean = s / cnt
    var = torch.clamp(ss / cnt - mean * mean, min=0.0)
    std = torch.sqrt(var)
    std = torch.where(std == 0, torch.ones_like(std), std)
    return ((X.to(torch.float64) - mean) / std).to(X.dtype)
