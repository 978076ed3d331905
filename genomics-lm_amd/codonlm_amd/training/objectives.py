"""Auxiliary training objectives on the MI355X path (mirrors src/codonlm/training/objectives.py).

Same functions, arguments and results as the reference module; the label construction
runs as integer kernels (cg_offset_targets, cg_termination_labels) and every cross-entropy
is the native fused CE (cg_cross_entropy), so the aux logits' gradients flow through
``_NativeCrossEntropy`` into TinyGPT's aux-head backward without a torch CE anywhere.

Row selection differs only in form: the reference gathers ``pred[valid]`` before its CE;
here invalid rows get the PAD target, which the PAD-ignoring CE drops -- the same rows, the
same weighted mean (label smoothing and class weights included).
"""
from __future__ import annotations

import torch

from .. import _lib as L
from .. import ops

PAD_ID = 0
DEFAULT_BOUNDARY_IDS = (2, 3)  # <EOS_CDS>, <SEP>


class _NativeCrossEntropy(torch.autograd.Function):
    """F.cross_entropy(logits2d, targets, ignore_index, label_smoothing, weight) -- forward
    and d(loss)/d(logits) in one native pass; backward scales the saved gradient."""

    @staticmethod
    def forward(ctx, logits2d, targets, eps, weight, ignore_index):
        loss, dl = ops.cross_entropy(logits2d, targets, eps=eps, weight=weight, ignore_index=ignore_index)
        ctx.save_for_backward(dl)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return dl * g, None, None, None, None


def cross_entropy(logits2d, targets, *, ignore_index=PAD_ID, label_smoothing=0.0, weight=None):
    L.require_device(logits2d, "cross_entropy")
    logits2d = logits2d.float()
    if logits2d.stride(-1) != 1:
        logits2d = logits2d.contiguous()
    w = None if weight is None else weight.to(device=logits2d.device, dtype=torch.float32).contiguous()
    return _NativeCrossEntropy.apply(logits2d, targets.to(torch.int64).contiguous(), float(label_smoothing), w,
                                     int(ignore_index))


def offset_target_mask(yb: torch.Tensor, offset: int, boundary_ids=DEFAULT_BOUNDARY_IDS) -> torch.Tensor:
    """Valid positions for predicting seq[t + offset] from logits at t (objectives.py:6-23)."""
    if offset < 1:
        raise ValueError("offset must be >= 1")
    if offset > yb.shape[1]:
        return torch.zeros((yb.shape[0], 0), dtype=torch.bool, device=yb.device)
    tk, _ = ops.offset_targets(yb, offset, boundary_ids, count=False)
    return tk[:, : yb.shape[1] - offset + 1] != PAD_ID


def multi_offset_lm_loss(
    logits,
    yb: torch.Tensor,
    offset_weights: dict,
    label_smoothing: float = 0.0,
    loss_weights: torch.Tensor | None = None,
    boundary_ids=DEFAULT_BOUNDARY_IDS,
    return_counts: bool = False,
):
    """sum_k w_k CE(logits_k at t, y[t+k-1]) over the valid targets (objectives.py:26-60).

    The reference skips an offset with no valid target (a host-side ``valid.any()``).
    ``return_counts=True`` keeps that decision on the device: an empty offset adds 0 to the
    total (its CE is 0/0; the gradient it passes is 0) and its entry in ``losses`` must be
    ignored by the caller when ``counts[k] == 0`` -- (total, losses, counts), no host sync."""
    losses = {}
    counts = {}
    total = torch.zeros((), dtype=torch.float32, device=yb.device)
    T = yb.shape[1]
    for offset, weight in offset_weights.items():
        if weight == 0.0 or offset <= 1 or offset > T:
            continue
        if isinstance(logits, dict):
            if offset not in logits:
                continue
            pred = logits[offset]
        else:
            pred = logits
        tk, n_valid = ops.offset_targets(yb, offset, boundary_ids)
        if not return_counts and int(n_valid.item()) == 0:  # the reference's bool(valid.any())
            continue
        V = pred.shape[-1]
        offset_loss = cross_entropy(pred[:, :T].reshape(-1, V), tk.view(-1), ignore_index=PAD_ID,
                                    label_smoothing=label_smoothing, weight=loss_weights)
        losses[offset] = offset_loss
        if return_counts:
            counts[offset] = n_valid
            offset_loss = torch.where(n_valid.reshape(()) > 0, offset_loss, 0.0)
        # total + weight * loss as one launch (the trainer's objective runs per microbatch: its small
        # elementwise launches were ~1 % of the C5 step)
        total = torch.add(total, offset_loss, alpha=float(weight))
    if return_counts:
        return total, losses, counts
    return total, losses


def termination_distance_bucket_labels(
    yb: torch.Tensor,
    stop_ids: tuple,
    bucket_edges: tuple = (0, 3, 10, 30),
    ignore_index: int = -100,
) -> torch.Tensor:
    """Bucket each valid position's distance to the next stop token (objectives.py:63-91)."""
    if not stop_ids:
        raise ValueError("stop_ids must not be empty")
    if tuple(bucket_edges) != tuple(sorted(bucket_edges)):
        raise ValueError("bucket_edges must be sorted")
    if len(stop_ids) > 8 or len(bucket_edges) > 8:
        raise ValueError("at most 8 stop ids and 8 bucket edges")
    return ops.termination_labels(yb, stop_ids, bucket_edges, ignore_index)


def termination_aux_loss(
    termination_logits: torch.Tensor,
    labels: torch.Tensor,
    class_weights: torch.Tensor | None = None,
    ignore_index: int = -100,
) -> torch.Tensor:
    """CE over the termination buckets (objectives.py:94-105)."""
    nc = termination_logits.size(-1)
    return cross_entropy(termination_logits.reshape(-1, nc), labels.reshape(-1), ignore_index=ignore_index,
                         weight=class_weights)


__all__ = ["PAD_ID", "DEFAULT_BOUNDARY_IDS", "cross_entropy", "offset_target_mask", "multi_offset_lm_loss",
           "termination_distance_bucket_labels", "termination_aux_loss"]
