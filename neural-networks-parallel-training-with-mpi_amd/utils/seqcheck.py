"""Collective-sequence checker (race / mismatch detection).

Every rank must issue the same collectives in the same order (the reference relies on this
implicitly: ref.py:87,97,108|133/138,185,199/203).  In debug mode each rank contributes
``(epoch, number of gradient collectives issued so far)`` and the checker verifies over the gloo
control plane that all ranks agree, raising with the per-rank table if they do not.
"""
from __future__ import annotations


class CollectiveMismatch(RuntimeError):
    pass


class SequenceChecker:
    def __init__(self, pg):
        self.pg = pg

    def check(self, epoch: int, seq: int):
        rows = self.pg.allgather_object((int(epoch), int(seq)))
        if len(set(rows)) != 1:
            raise CollectiveMismatch(f"collective sequence diverged at epoch {epoch}: {rows}")
        return rows
