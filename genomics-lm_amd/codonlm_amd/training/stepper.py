"""Rank-consistent control of the microbatch loop (src/codonlm/training/loop.py:1054-1261).

The reference loop is single-process: after each forward it checks ``torch.isfinite(loss)``
and aborts the accumulation group on a nonfinite value (loop.py:1197-1219), and at the end of
each iteration it checks the wall-time limit (``wall_timer.check()``, :1258).  With one
process per GPU these two decisions must be identical on every rank -- otherwise one rank
skips an optimizer step (or leaves the loop) while the others block in the next gradient
all-reduce.  ``GroupController.agree`` turns both into one collective: a MAX all-reduce of
(nonfinite, wall time exceeded) over a CPU (gloo) process group, so the flags never queue
behind the gradient buckets on the RCCL stream.  Token counts of committed groups are summed
over the same group.

``GroupController.completes_group`` says before a microbatch's backward whether that
microbatch will close its group if it is finite -- the point where the trainer hands the
bucketed RCCL all-reduce to the backward (overlap).  Health counters are identical on every
rank (the aborts are collective), so this decision is too.
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist


class GroupController:
    def __init__(self, *, gacc: int, health, world: int = 1, group=None, wall_limit_s: float | None = None,
                 clock=time.perf_counter, t0: float | None = None):
        self.gacc = max(1, int(gacc))
        self.health = health
        self.world = max(1, int(world))
        self.group = group
        self.wall_limit_s = None if wall_limit_s is None else float(wall_limit_s)
        self.clock = clock
        self.t0 = clock() if t0 is None else t0

    def completes_group(self, is_last_batch: bool) -> bool:
        """A finite microbatch now commits its group (gacc reached, or the epoch's last batch)."""
        return self.health.active_microbatches + 1 >= self.gacc or bool(is_last_batch)

    def time_exceeded(self) -> bool:
        return self.wall_limit_s is not None and (self.clock() - self.t0) > self.wall_limit_s

    def agree(self, nonfinite: bool) -> tuple[bool, bool]:
        """(abort, stop) identical on every rank: abort if any rank's loss is nonfinite, stop
        if any rank is past the wall-time limit."""
        stop = self.time_exceeded()
        if self.world == 1:
            return bool(nonfinite), stop
        t = torch.tensor([1.0 if nonfinite else 0.0, 1.0 if stop else 0.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return bool(t[0] > 0), bool(t[1] > 0)

    def sum(self, values):
        """Sum of host scalars over the ranks (token counts, val-loss sums)."""
        if self.world == 1:
            return [float(v) for v in values]
        t = torch.tensor([float(v) for v in values], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t.tolist()


def control_group(world: int):
    """CPU (gloo) process group for the loop's control collectives; None when single-process."""
    if world <= 1 or not (dist.is_available() and dist.is_initialized()):
        return None
    if dist.get_backend() == "gloo":
        return dist.group.WORLD
    return dist.new_group(backend="gloo")


__all__ = ["GroupController", "control_group"]
