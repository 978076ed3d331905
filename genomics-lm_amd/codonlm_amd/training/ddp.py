"""Data-parallel training step: one process per GPU, RCCL gradient all-reduce over xGMI
overlapped with the native backward.

The reference trains single-process (no torch.distributed anywhere); this
adds the DP exchange the north star asks for.  Gradients live in ONE flat buffer whose
layout puts each transformer block in its own contiguous range, so each backward phase
(head/ln_f, block L-1 ... block 0, embeddings) completes exactly one bucket.  Right after
the engine has *enqueued* a phase's kernels we issue ``all_reduce(bucket, async_op=True)``
on the RCCL process group: RCCL's stream waits on the compute stream at that point and
then runs concurrently with the next phase's kernels.  The 1/world average is folded
into the AdamW launch (``grad_scale``), as is the accumulation-group average
(loop.py:145-150).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import _lib as L
from ..model_tiny_gpt import mix_seed_rank


def bucket_ranges(model):
    """{phase_name: (begin, end)} flat-buffer ranges completed by each backward phase."""
    lay = model._layout
    total = model._flat.numel()
    layer_start = {}
    lnf = None
    for kind, layer, off, rows, cols, ld in lay:
        if kind == L.P_LN1_W:
            layer_start[layer] = off
        if kind == L.P_LNF_W:
            lnf = off
    L_ = model.n_layer
    ranges = {"head": (lnf, total)}
    for l in range(L_):
        end = layer_start[l + 1] if l + 1 < L_ else lnf
        ranges[l] = (layer_start[l], end)
    ranges["embed"] = (0, layer_start[0] if L_ > 0 else lnf)
    return ranges


class DataParallelStep:
    """fwd + CE + bwd (+ bucketed all-reduce) + AdamW for one microbatch group."""

    def __init__(self, model, optimizer, group=None, always_reduce: bool = False):
        """``always_reduce``: issue the bucket all-reduces even at world size 1 (an identity
        over one rank) -- the single-GPU smoke of the RCCL path (tests/test_gpu_rccl.py)."""
        self.model = model
        self.opt = optimizer
        self.group = group
        self.always_reduce = always_reduce
        on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if on else 1
        self.rank = dist.get_rank(group) if on else 0
        self.ranges = bucket_ranges(model)

    def _hook(self, handles):
        grads = self.model.flat_grads()

        def hook(name):
            if self.world <= 1 and not self.always_reduce:
                return
            b, e = self.ranges[name]
            if e > b:
                handles.append(dist.all_reduce(grads[b:e], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        return hook

    def bucket_hook(self, handles):
        """engine.backward / TinyGPT._bucket_hook callback that launches the async all-reduces."""
        return self._hook(handles)

    def microbatch(self, idx, targets, *, seed: int, accumulate: bool, sync: bool):
        """Forward + backward of one microbatch; all-reduce only when ``sync`` (last of a group).
        The rank is mixed into the dropout seed (independent masks per rank)."""
        eng = self.model.engine
        _, loss = eng.forward(idx, targets, training=True, seed=mix_seed_rank(seed, self.rank))
        handles = []
        eng.backward(accumulate=accumulate, bucket_hook=self._hook(handles) if sync else None)
        return loss, handles

    def step(self, idx, targets, *, seed: int):
        """One optimizer step on one microbatch per rank (grad_accum_steps = 1): gradients are
        averaged over the ranks (1/world folded into AdamW)."""
        loss, handles = self.microbatch(idx, targets, seed=seed, accumulate=False, sync=True)
        for h in handles:
            h.wait()
        self.opt.step(grad_scale=1.0 / self.world)
        return loss
