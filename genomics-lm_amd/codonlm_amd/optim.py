"""Fused AdamW over TinyGPT's flat parameter buffer (one cg_adamw launch per step).

Semantics follow torch.optim.AdamW as the codon trainer builds it (loop.py:681-731):
decoupled weight decay, bias-corrected moments, beta=(0.9, 0.999), eps=1e-8, and the
reference's two param groups -- the "fast" group (offset_projs / termination_head,
lr_embedding, wd 0) and the backbone group (everything else incl. embeddings, LN and
biases, lr / weight_decay; the name match at loop.py:689 never hits tok_emb).
It subclasses torch.optim.Optimizer so torch's LambdaLR / ReduceLROnPlateau drive the
per-group ``lr`` exactly as in the reference.  ``grad_scale`` folds the
accumulation-group average (loop.py:145-150) and the DDP 1/world into the same launch.
"""
from __future__ import annotations

import torch

from . import _lib as L
from . import ops


def _is_fast(name: str) -> bool:
    return ("transformer.wte" in name or "shape_proj" in name or "offset_projs" in name
            or "termination_head" in name)


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, model, lr=3e-4, weight_decay=0.05, lr_embedding=None, betas=(0.9, 0.999), eps=1e-8):
        self.model = model
        flat = model.flat_parameters()
        fast, backbone = [], []
        for name, p in model.named_parameters():
            (fast if _is_fast(name) else backbone).append((name, p))
        groups = []
        if fast:
            groups.append({"params": [p for _, p in fast], "lr": lr if lr_embedding is None else lr_embedding,
                           "weight_decay": 0.0})
        if backbone:
            groups.append({"params": [p for _, p in backbone], "lr": lr, "weight_decay": weight_decay})
        super().__init__(groups, dict(lr=lr, weight_decay=weight_decay, betas=betas, eps=eps))
        self.betas, self.eps = betas, eps
        # the groups run as contiguous ranges of the flat buffer: the fast params (aux heads) are
        # laid out last by cg_model_param_layout, so they form its tail
        base = flat.data_ptr()
        total = flat.numel()
        fast_begin = min((p.data_ptr() - base) // 4 for _, p in fast) if fast else total
        if any((p.data_ptr() - base) // 4 >= fast_begin for _, p in backbone):
            raise RuntimeError("FusedAdamW: the fast parameter group is not the tail of the flat buffer")
        self._ranges = [(fast_begin, total), (0, fast_begin)] if fast else [(0, total)]
        self.exp_avg = torch.zeros_like(flat)
        self.exp_avg_sq = torch.zeros_like(flat)
        self.step_count = 0

    def zero_grad(self, set_to_none: bool = True):
        self.model.zero_grad(set_to_none)

    def _moment_view(self, buf, p):
        off = (p.data_ptr() - self.model.flat_parameters().data_ptr()) // 4
        return buf.as_strided(p.shape, p.stride(), buf.storage_offset() + off)

    def state_dict(self):
        """torch.optim.AdamW's format -- param_groups (the lr / wd the schedulers drive) and a
        per-parameter 'state' {step, exp_avg, exp_avg_sq} whose moments are views of the flat
        moment buffers -- plus 'flat_state' (the flat buffers themselves).  The reference trainer
        (torch.optim.AdamW.load_state_dict) resumes from the per-parameter state; this
        optimizer from either."""
        self.state.clear()
        if self.step_count > 0:
            for g in self.param_groups:
                for p in g["params"]:
                    self.state[p] = {"step": torch.tensor(float(self.step_count)),
                                     "exp_avg": self._moment_view(self.exp_avg, p),
                                     "exp_avg_sq": self._moment_view(self.exp_avg_sq, p)}
        sd = super().state_dict()
        self.state.clear()
        sd["flat_state"] = {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "step": int(self.step_count)}
        return sd

    def load_state_dict(self, state_dict):
        flat = state_dict.get("flat_state")
        per_param = state_dict.get("state") or {}
        super().load_state_dict({"state": {}, "param_groups": state_dict["param_groups"]})
        with torch.no_grad():
            if flat is not None:
                self.exp_avg.copy_(flat["exp_avg"])
                self.exp_avg_sq.copy_(flat["exp_avg_sq"])
                self.step_count = int(flat["step"])
            elif per_param:
                # a torch.optim.AdamW state (the reference trainer's checkpoints): moments per
                # parameter index, in param_groups order
                params = [p for g in self.param_groups for p in g["params"]]
                steps = set()
                self.exp_avg.zero_()
                self.exp_avg_sq.zero_()
                for idx, st in per_param.items():
                    p = params[int(idx)]
                    self._moment_view(self.exp_avg, p).copy_(st["exp_avg"])
                    self._moment_view(self.exp_avg_sq, p).copy_(st["exp_avg_sq"])
                    steps.add(int(float(st["step"])))
                if len(steps) > 1:
                    raise ValueError(f"FusedAdamW keeps one step count; the state has {sorted(steps)}")
                self.step_count = steps.pop() if steps else 0

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        loss = closure() if closure is not None else None
        self.step_count += 1
        segs = []
        for g, (b, e) in zip(self.param_groups, self._ranges):
            if e > b:
                segs.append((b, e, g["lr"], g["weight_decay"]))
        eng = self.model.engine
        shadow = eng.shadow if eng.cfg.dtype == "bf16" else None
        ops.adamw_(self.model.flat_parameters(), self.model.flat_grads(), self.exp_avg, self.exp_avg_sq,
                   self.step_count, segs, shadow=shadow, beta1=self.betas[0], beta2=self.betas[1], eps=self.eps,
                   grad_scale=grad_scale)
        if shadow is not None:
            eng._shadow_stale = False
        return loss
