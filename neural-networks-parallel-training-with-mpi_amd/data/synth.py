"""Synthetic datasets.

* :func:`reference_regression` — exactly the reference data: ``make_regression(n_samples=16,
  n_features=2, noise=1, random_state=42)`` concatenated to ``XY = [X | y]`` float64
  (``ref.py:72-74``).  Used whenever the dataset is small enough for host generation.
* :func:`chunked_regression` — a deterministic, partition-independent generator with the same
  statistics as sklearn's ``make_regression`` (standard-normal features, ``n_informative``
  non-zero coefficients ``100*U[0,1)``, Gaussian noise).  Rows are produced in fixed chunks
  seeded by ``(seed, chunk)``, so any rank can generate exactly its own rows (on device for the
  8192-feature configs where host sklearn is too slow: SURVEY.md §7.4 item 7), and the
  concatenation over ranks does not depend on the world size.
* :func:`chunked_classification` — MNIST-shaped synthetic classification (784 features, 10
  classes): class centroids plus Gaussian noise, for the cross-entropy path (BASELINE config 5).
"""
from __future__ import annotations

import numpy as np
import torch

CHUNK_ROWS = 1024


def reference_regression(n_samples=16, n_features=2, noise=1.0, random_state=42):
    """Return ``(X, y)`` float64 numpy arrays from sklearn's make_regression (ref.py:72)."""
    from sklearn.datasets import make_regression
    X, y = make_regression(n_samples=n_samples, n_features=n_features, noise=noise,
                           random_state=random_state)
    return X, y


def _gen(seed: int, chunk: int, device) -> torch.Generator:
    g = torch.Generator(device=device)
    g.manual_seed((seed * 1000003 + chunk * 7919 + 17) & 0x7FFFFFFFFFFF)
    return g


def regression_coef(n_features: int, seed: int, n_informative: int = 10, out: int = 1,
                    device="cpu") -> torch.Tensor:
    g = _gen(seed, -1, "cpu")
    k = min(n_informative, n_features)
    coef = torch.zeros(n_features, out, dtype=torch.float64)
    idx = torch.randperm(n_features, generator=g)[:k]
    coef[idx] = 100.0 * torch.rand(k, out, generator=g, dtype=torch.float64)
    return coef.to(device)


def chunked_regression(row_start: int, n_rows: int, n_features: int, noise: float = 1.0,
                       seed: int = 42, out: int = 1, device="cpu", dtype=torch.float32):
    """Rows ``[row_start, row_start+n_rows)`` of a virtual regression dataset.

    Returns ``(X [n_rows, n_features], y [n_rows, out])`` in ``dtype`` on ``device``.
    """
    dev = torch.device(device)
    coef = regression_coef(n_features, seed, out=out, device=dev).to(torch.float32)
    X = torch.empty(n_rows, n_features, device=dev, dtype=torch.float32)
    y = torch.empty(n_rows, out, device=dev, dtype=torch.float32)
    if n_rows == 0:
        return X.to(dtype), y
    c0 = row_start // CHUNK_ROWS
    c1 = (row_start + n_rows - 1) // CHUNK_ROWS
    gen_dev = "cuda" if dev.type == "cuda" else "cpu"
    for c in range(c0, c1 + 1):
        g = _gen(seed, c, dev if dev.type == "cuda" else "cpu")
        xc = torch.randn(CHUNK_ROWS, n_features, generator=g, device=gen_dev)
        ec = torch.randn(CHUNK_ROWS, out, generator=g, device=gen_dev)
        lo = max(row_start, c * CHUNK_ROWS)
        hi = min(row_start + n_rows, (c + 1) * CHUNK_ROWS)
        a, b = lo - c * CHUNK_ROWS, hi - c * CHUNK_ROWS
        X[lo - row_start:hi - row_start] = xc[a:b].to(dev)
        y[lo - row_start:hi - row_start] = (xc[a:b].to(dev) @ coef) + noise * ec[a:b].to(dev)
    return X.to(dtype), y


def chunked_classification(row_start: int, n_rows: int, n_features: int, n_classes: int,
                           seed: int = 7, noise: float = 1.0, device="cpu",
                           dtype=torch.float32):
    """Rows of a virtual MNIST-shaped classification set: ``(X, labels int64)``."""
    dev = torch.device(device)
    gc = _gen(seed, -2, "cpu")
    centroids = torch.randn(n_classes, n_features, generator=gc).to(dev)
    X = torch.empty(n_rows, n_features, device=dev, dtype=torch.float32)
    lab = torch.empty(n_rows, device=dev, dtype=torch.int64)
    if n_rows == 0:
        return X.to(dtype), lab
    c0 = row_start // CHUNK_ROWS
    c1 = (row_start + n_rows - 1) // CHUNK_ROWS
    gen_dev = "cuda" if dev.type == "cuda" else "cpu"
    for c in range(c0, c1 + 1):
        g = _gen(seed, c, dev if dev.type == "cuda" else "cpu")
        lc = torch.randint(0, n_classes, (CHUNK_ROWS,), generator=g, device=gen_dev)
        nc = torch.randn(CHUNK_ROWS, n_features, generator=g, device=gen_dev)
        lo = max(row_start, c * CHUNK_ROWS)
        hi = min(row_start + n_rows, (c + 1) * CHUNK_ROWS)
        a, b = lo - c * CHUNK_ROWS, hi - c * CHUNK_ROWS
        lab[lo - row_start:hi - row_start] = lc[a:b].to(dev)
        X[lo - row_start:hi - row_start] = centroids[lc[a:b].to(dev)] + noise * nc[a:b].to(dev)
    return X.to(dtype), lab


def as_xy_matrix(X: np.ndarray, y: np.ndarray) -> np.ndarray:
    """``XY = concat([X, y])`` as the reference builds it (ref.py:73)."""
    return np.concatenate((X, y.reshape(len(y), -1)), axis=1)
