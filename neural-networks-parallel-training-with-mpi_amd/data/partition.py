"""Row partitioning of a dataset across ranks.

Reference semantics (``ref.py:99-143``): ``result, residue = divmod(h, nprocs)``; with an
uneven split the first ``residue`` ranks receive ``result + 1`` rows and the rest ``result``,
as contiguous row blocks in rank order.  The reference computes element counts in ``int8``
and broadcasts them as ``MPI.INT`` (defects D1/D2: overflow past 42 rows/rank and a crash for
P in {3,5,6,7}); ranks with zero rows crash in ``StandardScaler`` (D3).  Here counts are int64,
computed identically on every rank (no broadcast needed), and empty shards are allowed.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List


@dataclass(frozen=True)
class Partition:
    n_rows: int
    world: int
    counts: tuple  # rows per rank
    displs: tuple  # first row of each rank

    def rows(self, rank: int) -> int:
        return self.counts[rank]

    def start(self, rank: int) -> int:
        return self.displs[rank]

    def slice(self, rank: int) -> slice:
        return slice(self.displs[rank], self.displs[rank] + self.counts[rank])

    @property
    def even(self) -> bool:
        return self.n_rows % self.world == 0

    @property
    def max_rows(self) -> int:
        return max(self.counts) if self.counts else 0

    def element_counts(self, row_width: int) -> List[int]:
        """Element counts as the reference's Scatterv would use (fixed D1: int64)."""
        return [c * row_width for c in self.counts]


def partition_rows(n_rows: int, world: int) -> Partition:
    if world <= 0:
        raise ValueError(f"world size must be positive, got {world}")
    if n_rows < 0:
        raise ValueError(f"n_rows must be >= 0, got {n_rows}")
    result, residue = divmod(n_rows, world)
    counts = tuple(result + 1 if p < residue else result for p in range(world))
    displs = []
    acc = 0
    for c in counts:
        displs.append(acc)
        acc += c
    return Partition(n_rows, world, counts, tuple(displs))
