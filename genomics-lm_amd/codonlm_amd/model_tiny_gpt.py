"""Drop-in TinyGPT for MI355X (replaces src/codonlm/model_tiny_gpt.py of genomics-lm).

Same constructor (model_tiny_gpt.py:156-177), same state_dict keys/shapes (:197-251,
including the persistent ``blocks.{i}.attn.mask`` and ``loss_weights`` buffers), same
forward/forward_hidden/iter_hidden_states/build_attention_mask/to_dict surface
(:253-389) and the same hook-visible sub-module names (``blocks[i].attn.query`` ...).

What differs is where the math runs: every parameter is a view into one flat fp32
buffer whose layout the native library owns, and forward/backward are issued by the
native engine (engine.cpp) as hand-written gfx950 kernels.  ``loss.backward()`` works:
the loss returned in training mode carries an autograd node whose backward runs the
engine's backward and leaves the gradients in the flat grad buffer, which every
``param.grad`` views.

Extra keyword arguments (not in the reference): ``compute_dtype`` ("fp32" parity mode,
"bf16" throughput mode with fp32 master weights), ``device`` and ``engine_opts`` (a dict of
cg_model_opts fields selecting measured engine alternatives for tests / A/B runs; empty = the
defaults).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import _lib as L
from .engine import Engine, EngineConfig, param_layout

_KIND_NAMES = {
    L.P_LN1_W: "ln1.weight", L.P_LN1_B: "ln1.bias",
    L.P_Q_W: "attn.query.weight", L.P_K_W: "attn.key.weight", L.P_V_W: "attn.value.weight",
    L.P_Q_B: "attn.query.bias", L.P_K_B: "attn.key.bias", L.P_V_B: "attn.value.bias",
    L.P_PROJ_W: "attn.proj.weight", L.P_PROJ_B: "attn.proj.bias",
    L.P_LN2_W: "ln2.weight", L.P_LN2_B: "ln2.bias",
    L.P_FC1_W: "mlp.0.weight", L.P_FC1_B: "mlp.0.bias", L.P_FC2_W: "mlp.2.weight", L.P_FC2_B: "mlp.2.bias",
    L.P_GATE_W: "mlp.w_gate.weight", L.P_UP_W: "mlp.w_up.weight", L.P_DOWN_W: "mlp.w_down.weight",
}


def _entry_name(kind, layer, offsets):
    if kind == L.P_TOK_EMB:
        return "tok_emb.weight"
    if kind == L.P_POS_EMB:
        return "pos_emb.weight"
    if kind == L.P_LNF_W:
        return "ln_f.weight"
    if kind == L.P_LNF_B:
        return "ln_f.bias"
    if kind == L.P_HEAD_W:
        return "head.weight"
    if kind == L.P_TERM_W:
        return "termination_head.weight"
    if kind == L.P_TERM_B:
        return "termination_head.bias"
    if kind in (L.P_OFF1_W, L.P_OFF1_B, L.P_OFF2_W, L.P_OFF2_B):
        k = offsets[layer]
        sub = {L.P_OFF1_W: "0.weight", L.P_OFF1_B: "0.bias", L.P_OFF2_W: "2.weight", L.P_OFF2_B: "2.bias"}[kind]
        return f"offset_projs.{k}.{sub}"
    return f"blocks.{layer}.{_KIND_NAMES[kind]}"


class _Linear(nn.Module):
    """Hook-visible stand-in for nn.Linear whose parameters are flat-buffer views."""

    def __init__(self, in_features, out_features, bias=True):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(0))
        if bias:
            self.bias = nn.Parameter(torch.empty(0))
        else:
            self.register_parameter("bias", None)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, bias={self.bias is not None}"


class _LayerNorm(nn.Module):
    def __init__(self, n):
        super().__init__()
        self.normalized_shape = (n,)
        self.eps = 1e-5
        self.weight = nn.Parameter(torch.empty(0))
        self.bias = nn.Parameter(torch.empty(0))


class _Embedding(nn.Module):
    def __init__(self, num, dim):
        super().__init__()
        self.num_embeddings, self.embedding_dim = num, dim
        self.weight = nn.Parameter(torch.empty(0))


class RotaryEmbedding(nn.Module):
    """Mirror of model_tiny_gpt.py:9-33 (non-persistent cos/sin caches, hd-wide)."""

    def __init__(self, dim, max_position_embeddings=512, base=10000):
        super().__init__()
        self.dim, self.max_position_embeddings, self.base = dim, max_position_embeddings, base
        inv_freq = 1.0 / (base ** (torch.arange(0, dim, 2, dtype=torch.float32) / dim))
        self.register_buffer("inv_freq", inv_freq, persistent=False)


class SwiGLU(nn.Module):
    def __init__(self, n_embd, dropout):
        super().__init__()
        hidden = int(8 * n_embd // 3)
        self.w_gate = _Linear(n_embd, hidden, bias=False)
        self.w_up = _Linear(n_embd, hidden, bias=False)
        self.w_down = _Linear(hidden, n_embd, bias=False)
        self.dropout = nn.Dropout(dropout)


class CausalSelfAttention(nn.Module):
    def __init__(self, n_embd, n_head, dropout, block_size, n_kv_head=None, use_sdpa=False, use_rope=False):
        super().__init__()
        assert n_embd % n_head == 0
        self.n_head = n_head
        self.n_kv_head = n_kv_head if (n_kv_head is not None and 0 < n_kv_head <= n_head) else None
        self.use_sdpa = bool(use_sdpa)
        hd = n_embd // n_head
        kvd = (self.n_kv_head * hd) if self.n_kv_head is not None else n_embd
        self.key = _Linear(n_embd, kvd)
        self.query = _Linear(n_embd, n_embd)
        self.value = _Linear(n_embd, kvd)
        self.proj = _Linear(n_embd, n_embd)
        self.dropout = nn.Dropout(dropout)
        self.register_buffer("mask", torch.tril(torch.ones(block_size, block_size)).unsqueeze(0).unsqueeze(0))
        self.rotary_emb = RotaryEmbedding(hd, max_position_embeddings=block_size) if use_rope else None


class Block(nn.Module):
    def __init__(self, n_embd, n_head, dropout, block_size, n_kv_head=None, use_sdpa=False, use_swiglu=False,
                 use_rope=False):
        super().__init__()
        self.ln1 = _LayerNorm(n_embd)
        self.attn = CausalSelfAttention(n_embd, n_head, dropout, block_size, n_kv_head=n_kv_head,
                                        use_sdpa=use_sdpa, use_rope=use_rope)
        self.ln2 = _LayerNorm(n_embd)
        if use_swiglu:
            self.mlp = SwiGLU(n_embd, dropout)
        else:
            self.mlp = nn.Sequential(_Linear(n_embd, 4 * n_embd), nn.GELU(), _Linear(4 * n_embd, n_embd),
                                     nn.Dropout(dropout))


def mix_seed_rank(seed: int, rank: int) -> int:
    """Dropout seed of a data-parallel rank: the shared step counter with the rank mixed in
    (identity for rank 0)."""
    if not rank:
        return int(seed) & 0xFFFFFFFF
    x = (int(seed) ^ (int(rank) * 0x85EBCA6B)) & 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    return x ^ (x >> 15)


class _EngineBackward(torch.autograd.Function):
    """Autograd node tying ``loss`` to the native backward (loop.py:1233 loss.backward())."""

    @staticmethod
    def forward(ctx, loss, anchor, model):
        ctx.model = model
        return loss.clone()

    @staticmethod
    def backward(ctx, gout):
        ctx.model._native_backward(gout)
        return None, None, None


class _AuxEngineBackward(torch.autograd.Function):
    """Autograd node over (loss, termination logits, offset logits...) of a return_aux forward:
    whatever objective the caller builds from them (objectives.py), its gradients w.r.t. these
    outputs are handed to the native phase-0 backward in one call."""

    @staticmethod
    def forward(ctx, model, anchor, has_loss, has_term, *outs):
        ctx.model, ctx.has_loss, ctx.has_term = model, has_loss, has_term
        ctx.set_materialize_grads(False)  # unused heads arrive as None (their grads are zeroed)
        if has_loss:
            return (outs[0].clone(),) + tuple(outs[1:])
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        i = 0
        g_loss = g_term = None
        if ctx.has_loss:
            g_loss, i = grads[0], 1
        if ctx.has_term:
            g_term, i = grads[i], i + 1
        ctx.model._native_backward(g_loss, d_term=g_term, d_offsets=list(grads[i:]))
        return (None, None, None, None) + (None,) * len(grads)


class TinyGPT(nn.Module):
    def __init__(self, vocab_size, block_size, n_layer=3, n_head=4, n_embd=256, dropout=0.1, use_checkpoint=False,
                 label_smoothing: float = 0.0, sep_id: int | None = 3, tie_embeddings: bool = True,
                 n_kv_head: int | None = None, use_sdpa: bool = False, loss_weights=None,
                 termination_aux: bool = False, termination_n_classes: int = 5, multi_offset_targets=None,
                 use_swiglu: bool = False, use_rope: bool = False, use_shape_guidance: bool = False, *,
                 compute_dtype: str = "fp32", device=None, engine_opts: dict | None = None):
        super().__init__()
        if use_shape_guidance:
            raise ValueError("use_shape_guidance is outside the MI355X hot path (SURVEY §2: biophysics encoder)")
        if compute_dtype not in ("fp32", "bf16"):
            raise ValueError("compute_dtype must be 'fp32' or 'bf16'")
        if n_kv_head is not None and n_kv_head > 0 and n_kv_head <= n_head and n_head % n_kv_head != 0:
            raise ValueError("n_head must be divisible by n_kv_head for GQA")
        self.block_size = block_size
        self.vocab_size = vocab_size
        self.n_layer = n_layer
        self.n_head = n_head
        self.n_embd = n_embd
        self.dropout_p = float(dropout)
        self.use_checkpoint = use_checkpoint
        self.label_smoothing = float(label_smoothing)
        self.sep_id = sep_id
        self.tie_embeddings = bool(tie_embeddings)
        self.n_kv_head = n_kv_head if (n_kv_head is not None and n_kv_head > 0) else None
        self.use_sdpa = bool(use_sdpa)
        self.termination_aux = bool(termination_aux)
        self.termination_n_classes = int(termination_n_classes)
        self.use_swiglu = bool(use_swiglu)
        self.use_rope = bool(use_rope)
        self.use_shape_guidance = False
        self.compute_dtype = compute_dtype
        self.multi_offset_targets = sorted(set(int(t) for t in multi_offset_targets)) if multi_offset_targets else []
        if len(self.multi_offset_targets) > 8:
            raise ValueError("at most 8 multi_offset_targets")

        # ---- module tree with reference names (registration order == reference order)
        self.tok_emb = _Embedding(vocab_size, n_embd)
        self.pos_emb = None if self.use_rope else _Embedding(block_size, n_embd)
        self.drop = nn.Dropout(dropout)
        self.blocks = nn.ModuleList([
            Block(n_embd, n_head, dropout, block_size, n_kv_head=self.n_kv_head, use_sdpa=self.use_sdpa,
                  use_swiglu=self.use_swiglu, use_rope=self.use_rope) for _ in range(n_layer)])
        self.ln_f = _LayerNorm(n_embd)
        self.head = _Linear(n_embd, vocab_size, bias=False)
        if self.tie_embeddings:
            self.head.weight = self.tok_emb.weight
        self.termination_head = _Linear(n_embd, self.termination_n_classes) if self.termination_aux else None
        self.offset_projs = nn.ModuleDict()
        for k in self.multi_offset_targets:
            self.offset_projs[str(k)] = nn.Sequential(_Linear(n_embd, n_embd), nn.GELU(), _Linear(n_embd, n_embd))
        lw = torch.tensor(loss_weights, dtype=torch.float32) if loss_weights is not None else \
            torch.ones(vocab_size, dtype=torch.float32)
        self.register_buffer("loss_weights", lw)

        # ---- flat buffers + views
        self._ecfg = EngineConfig(vocab_size=vocab_size, block_size=block_size, n_layer=n_layer, n_head=n_head,
                                  n_embd=n_embd, n_kv_head=self.n_kv_head, use_swiglu=self.use_swiglu,
                                  use_rope=self.use_rope, sep_id=sep_id, tie_embeddings=self.tie_embeddings,
                                  termination_aux=self.termination_aux,
                                  termination_n_classes=self.termination_n_classes,
                                  multi_offset_targets=tuple(self.multi_offset_targets), dropout=self.dropout_p,
                                  label_smoothing=self.label_smoothing, dtype=compute_dtype,
                                  opts=tuple(sorted((engine_opts or {}).items())))
        self._layout, total = param_layout(self._ecfg)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        device = torch.device(device)
        self.register_buffer("_flat", torch.zeros(total, dtype=torch.float32, device=device), persistent=False)
        self.register_buffer("_flat_grad", torch.zeros(total, dtype=torch.float32, device=device), persistent=False)
        self._specs = {}
        for kind, layer, off, rows, cols, ld in self._layout:
            self._specs[_entry_name(kind, layer, self.multi_offset_targets)] = (off, rows, cols, ld)
        self._bind_views()
        self._reference_init()
        self._engine = None
        self._grads_fresh = True
        self._accum_next = False
        self._dropout_seed = 0
        # data-parallel rank mixed into the dropout seeds (ranks draw independent masks for the
        # same step; rank 0 keeps the single-process sequence) and the per-backward bucket hook
        # a data-parallel caller sets before loss.backward() (engine.backward's overlap point)
        self._seed_rank = 0
        self._bucket_hook = None

    # ------------------------------------------------------------------ layout/views
    def _view(self, buf, spec):
        off, rows, cols, ld = spec
        if cols == 0:
            return buf[off: off + rows]
        return buf[off: off + rows * ld].view(rows, ld)[:, :cols]

    def _param_by_name(self, name):
        mod = self
        parts = name.split(".")
        for p in parts[:-1]:
            if isinstance(mod, nn.ModuleDict):
                mod = mod[p]
            elif p.isdigit():
                mod = mod[int(p)]
            else:
                mod = getattr(mod, p)
        return mod, parts[-1]

    def _bind_views(self):
        pairs = []
        for name, spec in self._specs.items():
            mod, attr = self._param_by_name(name)
            p = getattr(mod, attr)
            p.data = self._view(self._flat, spec)
            g = self._view(self._flat_grad, spec)
            p.grad = g
            pairs.append((p, g))
        # (parameter, its view of the flat grad buffer): re-attached by _bind_grad_views
        self._grad_pairs = pairs

    @torch.no_grad()
    def _reference_init(self):
        """PyTorch-default init drawn in the reference's module order (model_tiny_gpt.py:197-246),
        so torch.manual_seed(s) gives the same initial weights as the reference TinyGPT."""
        d, V = self.n_embd, self.vocab_size

        def put(name, t):
            mod, attr = self._param_by_name(name)
            getattr(mod, attr).copy_(t)

        put("tok_emb.weight", nn.Embedding(V, d).weight)
        if not self.use_rope:
            put("pos_emb.weight", nn.Embedding(self.block_size, d).weight)
        hd = d // self.n_head
        kvd = (self.n_kv_head * hd) if self.n_kv_head is not None and self.n_kv_head <= self.n_head else d
        for i in range(self.n_layer):
            p = f"blocks.{i}."
            ln = nn.LayerNorm(d)
            put(p + "ln1.weight", ln.weight); put(p + "ln1.bias", ln.bias)
            for nm, out in (("key", kvd), ("query", d), ("value", kvd), ("proj", d)):
                lin = nn.Linear(d, out)
                put(p + f"attn.{nm}.weight", lin.weight); put(p + f"attn.{nm}.bias", lin.bias)
            ln = nn.LayerNorm(d)
            put(p + "ln2.weight", ln.weight); put(p + "ln2.bias", ln.bias)
            if self.use_swiglu:
                h = int(8 * d // 3)
                put(p + "mlp.w_gate.weight", nn.Linear(d, h, bias=False).weight)
                put(p + "mlp.w_up.weight", nn.Linear(d, h, bias=False).weight)
                put(p + "mlp.w_down.weight", nn.Linear(h, d, bias=False).weight)
            else:
                l0, l2 = nn.Linear(d, 4 * d), nn.Linear(4 * d, d)
                put(p + "mlp.0.weight", l0.weight); put(p + "mlp.0.bias", l0.bias)
                put(p + "mlp.2.weight", l2.weight); put(p + "mlp.2.bias", l2.bias)
        ln = nn.LayerNorm(d)
        put("ln_f.weight", ln.weight); put("ln_f.bias", ln.bias)
        head = nn.Linear(d, V, bias=False)  # consumes RNG like the reference, then tied
        if not self.tie_embeddings:
            put("head.weight", head.weight)
        if self.termination_aux:
            th = nn.Linear(d, self.termination_n_classes)
            put("termination_head.weight", th.weight); put("termination_head.bias", th.bias)
        for k in self.multi_offset_targets:
            a, b = nn.Linear(d, d), nn.Linear(d, d)
            put(f"offset_projs.{k}.0.weight", torch.eye(d)); put(f"offset_projs.{k}.0.bias", torch.zeros(d))
            put(f"offset_projs.{k}.2.weight", torch.eye(d)); put(f"offset_projs.{k}.2.bias", torch.zeros(d))
            del a, b
        if getattr(self, "_engine", None) is not None:
            self._engine.mark_params_changed()

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        if self._flat.dtype != torch.float32:
            raise TypeError("TinyGPT master parameters are fp32; use compute_dtype='bf16' for bf16 compute")
        self._bind_views()
        if getattr(self, "_engine", None) is not None:
            lw = self._loss_weight_arg()
            self._engine.set_buffers(self._flat, self._flat_grad, lw)
        return self

    def _load_from_state_dict(self, *args, **kwargs):
        super()._load_from_state_dict(*args, **kwargs)
        if getattr(self, "_engine", None) is not None:
            self._engine.mark_params_changed()

    # ------------------------------------------------------------------ engine
    def _loss_weight_arg(self):
        lw = self.loss_weights
        if bool(torch.all(lw == 1.0)):
            return None
        return lw.to(self._flat.device, torch.float32).contiguous()

    @property
    def engine(self) -> Engine:
        if self._engine is None:
            L.require_device(self._flat, "TinyGPT")
            self._engine = Engine(self._ecfg, self._flat, self._flat_grad, self._loss_weight_arg())
        return self._engine

    def flat_parameters(self):
        return self._flat

    def flat_grads(self):
        return self._flat_grad

    def zero_grad(self, set_to_none: bool = True):
        # grads live in one flat buffer that param.grad views; "set_to_none" only resets it
        self._grads_fresh = True
        self._bind_grad_views()

    def _bind_grad_views(self):
        # runs twice per microbatch (zero_grad, after the backward): only grads that something
        # replaced or set to None are re-attached -- re-creating and re-assigning every view took
        # milliseconds of host time per step and left the GPU idle between optimizer step and
        # the next forward
        for p, g in self._grad_pairs:
            if p.grad is not g:
                p.grad = g

    def _native_backward(self, gout, d_term=None, d_offsets=None):
        """Native backward of the last forward: ``gout`` = d(objective)/d(loss) (None when the
        next-codon loss is unused), ``d_term`` / ``d_offsets`` = gradients of the aux logits."""
        # an optimizer that set grads to None means "fresh group"
        if self.tok_emb.weight.grad is None:
            self._grads_fresh = True
        eng = self.engine
        # d(objective)/d(loss) stays on the device: the engine scales the head gradient in-kernel
        eng.set_head_grads(0.0 if gout is None else 1.0, d_term, d_offsets,
                           scale_dev=None if gout is None else gout)
        hook, self._bucket_hook = self._bucket_hook, None
        eng.backward(accumulate=not self._grads_fresh, bucket_hook=hook)
        self._grads_fresh = False
        self._bind_grad_views()

    # ------------------------------------------------------------------ reference API
    def to_dict(self) -> dict:
        return {
            "vocab_size": int(self.vocab_size), "block_size": int(self.block_size), "n_layer": int(self.n_layer),
            "n_head": int(self.n_head), "n_embd": int(self.n_embd), "dropout": float(self.dropout_p),
            "sep_mask_enabled": self.sep_id is not None, "tie_embeddings": bool(self.tie_embeddings),
            "n_kv_head": self.n_kv_head, "use_sdpa": bool(self.use_sdpa), "termination_aux": bool(self.termination_aux),
            "termination_n_classes": int(self.termination_n_classes),
            "multi_offset_targets": self.multi_offset_targets, "use_swiglu": bool(self.use_swiglu),
            "use_rope": bool(self.use_rope), "use_shape_guidance": False,
        }

    def build_attention_mask(self, idx: torch.Tensor, attention_window: int | None = None):
        """Materialised mask (model_tiny_gpt.py:273-295) -- for inspection only; the kernels
        evaluate the same predicate on the fly from per-token segment starts."""
        _, length = idx.shape
        if attention_window is not None and int(attention_window) < 1:
            raise ValueError("attention_window must be at least 1")
        if self.sep_id is None and attention_window is None:
            return None
        pos = torch.arange(length, device=idx.device)
        dist = pos.unsqueeze(1) - pos.unsqueeze(0)
        m = dist >= 0
        if attention_window is not None:
            m = m & (dist < int(attention_window))
        m = m.unsqueeze(0).unsqueeze(0)
        if self.sep_id is not None:
            seg = torch.cumsum(idx == int(self.sep_id), dim=1)
            m = m & (seg.unsqueeze(-1) == seg.unsqueeze(-2)).unsqueeze(1)
        return m

    def _capture_attention(self):
        """`blocks[i].attn.last_attn` (B, H, T, T): the softmax probabilities before dropout, as the
        reference's manual attention path records them (model_tiny_gpt.py:128).  Opt-in here
        (`model.capture_attn = True`, any attention path): materialising B*H*T^2 floats per block
        is an inspection cost the training path does not pay."""
        if not getattr(self, "capture_attn", False):
            return
        for i, blk in enumerate(self.blocks):
            blk.attn.last_attn = self.engine.attn_probs(i)

    def next_dropout_seed(self) -> int:
        self._dropout_seed = (self._dropout_seed + 0x9E3779B9) & 0xFFFFFFFF
        return mix_seed_rank(self._dropout_seed, self._seed_rank)

    def forward(self, idx, targets=None, return_aux: bool = False, shape_embeddings=None,
                attention_window: int | None = None):
        if shape_embeddings is not None:
            raise ValueError("shape guidance is not supported on the MI355X path")
        if return_aux and (self.termination_aux or self.multi_offset_targets):
            return self._forward_aux(idx, targets, attention_window)
        eng = self.engine
        training = self.training and self.dropout_p > 0
        seed = self.next_dropout_seed() if training else 0
        logits, loss = eng.forward(idx, targets, training=training, seed=seed, window=attention_window)
        self._capture_attention()
        if loss is not None and self.training and torch.is_grad_enabled():
            loss = _EngineBackward.apply(loss, self.tok_emb.weight, self)
        if return_aux:
            return logits, loss, {}
        return logits, loss

    def _forward_aux(self, idx, targets, attention_window):
        """forward(..., return_aux=True) with aux heads: (logits, loss, {termination_logits,
        offset_logits: {k: (B,T,V)}}) as model_tiny_gpt.py:326-351, all on the native engine."""
        eng = self.engine
        training = self.training and self.dropout_p > 0
        seed = self.next_dropout_seed() if training else 0
        logits, loss = eng.forward(idx, targets, training=training, seed=seed, window=attention_window)
        term, offs = eng.aux_forward()
        B, T = idx.shape
        outs = ([loss] if loss is not None else []) + ([term.view(B, T, -1)] if term is not None else []) + \
            [o.view(B, T, -1) for o in offs]
        if self.training and torch.is_grad_enabled():
            outs = list(_AuxEngineBackward.apply(self, self.tok_emb.weight, loss is not None, term is not None,
                                                 *outs))
        if loss is not None:
            loss = outs.pop(0)
        aux = {}
        if term is not None:
            aux["termination_logits"] = outs.pop(0)
        if self.multi_offset_targets:
            aux["offset_logits"] = {k: outs[i] for i, k in enumerate(self.multi_offset_targets)}
        return logits, loss, aux

    @torch.no_grad()
    def iter_hidden_states(self, idx, shape_embeddings=None, attention_window: int | None = None):
        """(0, embedding), (1..L, block outputs), ("final", ln_f) -- model_tiny_gpt.py:368-389."""
        if shape_embeddings is not None:
            raise ValueError("shape guidance is not supported on the MI355X path")
        eng = self.engine
        training = self.training and self.dropout_p > 0
        eng.forward(idx, None, training=training, seed=self.next_dropout_seed() if training else 0,
                    window=attention_window)
        for layer in range(self.n_layer + 1):
            yield layer, eng.hidden(layer).clone()
        yield "final", eng.hidden(self.n_layer + 1).float().clone()

    def forward_hidden(self, idx, shape_embeddings=None, attention_window: int | None = None):
        final = None
        for _, h in self.iter_hidden_states(idx, shape_embeddings=shape_embeddings,
                                            attention_window=attention_window):
            final = h
        if final is None:
            raise RuntimeError("hidden-state iterator produced no states")
        return final


def num_params(model: TinyGPT) -> int:
    return sum(p.numel() for p in model.parameters())


__all__ = ["TinyGPT", "num_params", "mix_seed_rank"]
