"""Collective-sequence checker (race / mismatch detection).

Every rank must issue the same collectives in the same order, with the same sizes (the
reference relies on this implicitly: ref.py:87,97,108|133/138,185,199/203).  Two ranks whose
bucket layouts differ (e.g. a per-rank environment changing how layers are chunked) issue the
same NUMBER of collectives with different sizes -- over RCCL that hangs or corrupts rather than
raising.  In ``--seqcheck`` mode:

* before the first collective, :meth:`SequenceChecker.check_plan` compares every rank's plan --
  sync kind, payload dtype and the (index, offset, numel) of every bucket -- over the gloo
  control plane and raises on any difference, so a layout mismatch never reaches RCCL;
* after every epoch, :meth:`SequenceChecker.check` compares ``(epoch, collectives issued,
  running signature)``, the signature hashing (kind, bucket index, offset, numel, dtype) of
  every collective issued so far (``GradSync.note``; graph replays replay the notes their
  capture recorded).
"""
from __future__ import annotations


class CollectiveMismatch(RuntimeError):
    pass


class SequenceChecker:
    def __init__(self, pg):
        self.pg = pg

    def check_plan(self, sync):
        plans = self.pg.allgather_object(sync.plan())
        if any(p != plans[0] for p in plans):
            diff = [r for r, p in enumerate(plans) if p != plans[0]]
            raise CollectiveMismatch(
                f"gradient-sync plans differ between ranks (ranks {diff} vs rank 0): "
                + "; ".join(f"rank {r}: {p}" for r, p in enumerate(plans)))
        return plans[0]

    def check(self, epoch: int, seq: int, sig: int = 0):
        rows = self.pg.allgather_object((int(epoch), int(seq), int(sig)))
        if len(set(rows)) != 1:
            raise CollectiveMismatch(f"collective sequence diverged at epoch {epoch}: {rows}")
        return rows
