"""CPU restatement of the reference TinyGPT hot path -- TEST INFRASTRUCTURE ONLY.

This module is the parity ORACLE for the MI355X path.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it, and only as the checker / the timed CPU baseline.  The product path
(``genomics-lm_amd/codonlm_amd``) never imports, calls or falls back to it.

It restates, in plain fp32 PyTorch-CPU functional code (no nn.Module), the
algorithm of the reference files below.  Every function cites the lines it
follows (paths relative to the upstream repo AvishaiBarnoy/genomics-lm):

* ``forward``            src/codonlm/model_tiny_gpt.py:297-352 (+ Block :150-153,
                         CausalSelfAttention manual path :82-132, SwiGLU :47-57,
                         RotaryEmbedding :9-45, build_attention_mask :273-295)
* ``iter_hidden_states`` src/codonlm/model_tiny_gpt.py:368-389
* ``cross_entropy``      F.cross_entropy(ignore_index=0, label_smoothing, weight)
                         as called at model_tiny_gpt.py:343-349 (formula in
                         SURVEY.md §8a row a13)
* ``adamw_step``         torch.optim.AdamW defaults as used at
                         src/codonlm/training/loop.py:681-731
* ``lr_lambda``          src/codonlm/training/loop.py:770-779
* ``offset_target_mask`` / ``termination_labels``
                         src/codonlm/training/objectives.py:6-23, 63-91
* ``multi_offset_loss`` / ``termination_loss`` / ``objective_backward``
                         objectives.py:26-60, 94-105; loop.py:1075-1112
* ``pool_state``         scripts/extract_embeddings.py:94-114

Parity pinning: the restatement is checked against golden vectors produced by
running the real reference in the build container (tests/golden/make_golden.py,
fixtures tests/golden/*.npz) -- see tests/test_oracle_golden.py.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field, asdict

import numpy as np
import torch
import torch.nn.functional as F

PAD_ID = 0
BOS_ID = 1
EOS_ID = 2
SEP_ID = 3


@dataclass
class OracleConfig:
    vocab_size: int = 68
    block_size: int = 64
    n_layer: int = 2
    n_head: int = 4
    n_embd: int = 64
    n_kv_head: int | None = None
    dropout: float = 0.0
    label_smoothing: float = 0.0
    sep_id: int | None = 3
    tie_embeddings: bool = True
    use_swiglu: bool = False
    use_rope: bool = False
    loss_weights: list | None = None
    termination_aux: bool = False
    termination_n_classes: int = 5
    multi_offset_targets: list = field(default_factory=list)

    @property
    def head_dim(self) -> int:
        return self.n_embd // self.n_head

    @property
    def kv_heads(self) -> int:
        # model_tiny_gpt.py:64 -- n_kv_head only honoured when 0 < kv <= H
        kv = self.n_kv_head
        if kv is not None and 0 < kv <= self.n_head:
            return kv
        return self.n_head

    @property
    def mlp_hidden(self) -> int:
        # SwiGLU width int(8*d//3) (model_tiny_gpt.py:50); GELU MLP 4d (:144)
        return int(8 * self.n_embd // 3) if self.use_swiglu else 4 * self.n_embd

    def to_dict(self) -> dict:
        return asdict(self)


def param_shapes(cfg: OracleConfig) -> dict[str, tuple]:
    """state_dict parameter names/shapes of the reference TinyGPT (model_tiny_gpt.py:197-251)."""
    d, V, T = cfg.n_embd, cfg.vocab_size, cfg.block_size
    kvd = cfg.kv_heads * cfg.head_dim
    out: dict[str, tuple] = {"tok_emb.weight": (V, d)}
    if not cfg.use_rope:
        out["pos_emb.weight"] = (T, d)
    for i in range(cfg.n_layer):
        p = f"blocks.{i}."
        out[p + "ln1.weight"] = (d,)
        out[p + "ln1.bias"] = (d,)
        out[p + "attn.key.weight"] = (kvd, d)
        out[p + "attn.key.bias"] = (kvd,)
        out[p + "attn.query.weight"] = (d, d)
        out[p + "attn.query.bias"] = (d,)
        out[p + "attn.value.weight"] = (kvd, d)
        out[p + "attn.value.bias"] = (kvd,)
        out[p + "attn.proj.weight"] = (d, d)
        out[p + "attn.proj.bias"] = (d,)
        out[p + "ln2.weight"] = (d,)
        out[p + "ln2.bias"] = (d,)
        if cfg.use_swiglu:
            h = cfg.mlp_hidden
            out[p + "mlp.w_gate.weight"] = (h, d)
            out[p + "mlp.w_up.weight"] = (h, d)
            out[p + "mlp.w_down.weight"] = (d, h)
        else:
            out[p + "mlp.0.weight"] = (4 * d, d)
            out[p + "mlp.0.bias"] = (4 * d,)
            out[p + "mlp.2.weight"] = (d, 4 * d)
            out[p + "mlp.2.bias"] = (d,)
    out["ln_f.weight"] = (d,)
    out["ln_f.bias"] = (d,)
    if not cfg.tie_embeddings:
        out["head.weight"] = (V, d)
    if cfg.termination_aux:
        out["termination_head.weight"] = (cfg.termination_n_classes, d)
        out["termination_head.bias"] = (cfg.termination_n_classes,)
    for k in sorted(set(int(t) for t in cfg.multi_offset_targets)):
        out[f"offset_projs.{k}.0.weight"] = (d, d)
        out[f"offset_projs.{k}.0.bias"] = (d,)
        out[f"offset_projs.{k}.2.weight"] = (d, d)
        out[f"offset_projs.{k}.2.bias"] = (d,)
    return out


def synthetic_params(cfg: OracleConfig, seed: int = 1234) -> dict[str, np.ndarray]:
    """Deterministic fp32 weights (numpy default_rng) with reference-like scales.

    Embeddings ~N(0,1) (nn.Embedding default), Linear weights ~U(-1/sqrt(in), 1/sqrt(in)),
    LayerNorm gamma around 1 / beta around 0 (perturbed so the affine path is exercised).
    """
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in param_shapes(cfg).items():
        if name.endswith("emb.weight"):
            a = rng.standard_normal(shape)
        elif ".ln" in name or name.startswith("ln_f"):
            if name.endswith("weight"):
                a = 1.0 + 0.1 * rng.standard_normal(shape)
            else:
                a = 0.1 * rng.standard_normal(shape)
        elif name.endswith("weight"):
            bound = 1.0 / math.sqrt(shape[1])
            a = rng.uniform(-bound, bound, size=shape)
        else:  # bias
            a = rng.uniform(-0.05, 0.05, size=shape)
        out[name] = a.astype(np.float32)
    return out


# ---------------------------------------------------------------------------
# dropout hash (restates genomics-lm_amd/csrc/common.h cg_hash / cg_keep)
# ---------------------------------------------------------------------------

def _fmix32(h: np.ndarray) -> np.ndarray:
    h = h.astype(np.uint32)
    h ^= h >> np.uint32(16)
    h = (h * np.uint32(0x85EBCA6B)).astype(np.uint32)
    h ^= h >> np.uint32(13)
    h = (h * np.uint32(0xC2B2AE35)).astype(np.uint32)
    h ^= h >> np.uint32(16)
    return h


def dropout_keep(seed: int, row: np.ndarray, col: np.ndarray, p: float) -> np.ndarray:
    """Bernoulli(1-p) keep mask identical to the device hash (common.h cg_keep)."""
    with np.errstate(over="ignore"):
        r = np.asarray(row, dtype=np.uint64).astype(np.uint32)
        c = np.asarray(col, dtype=np.uint64).astype(np.uint32)
        r, c = np.broadcast_arrays(r, c)
        # row hash: fmix32(seed ^ row*0x9E3779B1); pair mix: x = rowhash + (col>>1)*0x85EBCA77,
        # x ^= x>>15; x = (x & 0xFFFFFF) * 0x2C1B3D (24-bit multiply); x ^= x>>12
        # (common.h cg_row_hash / cg_pair_mix)
        hr = _fmix32(np.uint32(seed & 0xFFFFFFFF) ^ (r * np.uint32(0x9E3779B1)).astype(np.uint32))
        h = (hr + ((c >> np.uint32(1)) * np.uint32(0x85EBCA77)).astype(np.uint32)).astype(np.uint32)
        h ^= h >> np.uint32(15)
        h = ((h & np.uint32(0xFFFFFF)) * np.uint32(0x2C1B3D)).astype(np.uint32)
        h ^= h >> np.uint32(12)
        bits = np.where((c & np.uint32(1)) == 0, h & np.uint32(0xFFFF), h >> np.uint32(16))
    thr = np.uint32(min(65536, int(round(p * 65536.0))))
    return bits >= thr


def dropout_mask(seed: int, rows: int, cols: int, p: float) -> torch.Tensor:
    r = np.arange(rows, dtype=np.uint64)[:, None]
    c = np.arange(cols, dtype=np.uint64)[None, :]
    keep = dropout_keep(seed, r, c, p)
    return torch.from_numpy(keep.astype(np.float32) / (1.0 - p))


# seed derivation per dropout site (restates engine.cpp cg_site_seed)
SITE_EMB, SITE_ATTN, SITE_MLP = 0, 1, 2


def site_seed(seed: int, layer: int, site: int) -> int:
    x = np.array([(seed * 0x01000193 + layer * 0x9E37 + site * 0x7F4A7C15 + 0x3C6EF372) & 0xFFFFFFFF],
                 dtype=np.uint32)
    return int(_fmix32(x)[0])


# ---------------------------------------------------------------------------
# building blocks
# ---------------------------------------------------------------------------

def attention_mask(idx: torch.Tensor, sep_id: int | None, window: int | None = None) -> torch.Tensor:
    """causal & [dist<window] & same-SEP-segment (model_tiny_gpt.py:273-295)."""
    B, T = idx.shape
    pos = torch.arange(T)
    dist = pos[:, None] - pos[None, :]
    m = (dist >= 0)
    if window is not None:
        if int(window) < 1:
            raise ValueError("attention_window must be at least 1")
        m = m & (dist < int(window))
    m = m[None].expand(B, T, T)
    if sep_id is not None:
        seg = torch.cumsum((idx == int(sep_id)).long(), dim=1)
        m = m & (seg[:, :, None] == seg[:, None, :])
    return m  # (B, T, T) bool


def rope_cos_sin(T: int, hd: int) -> tuple[torch.Tensor, torch.Tensor]:
    """RotaryEmbedding cache (model_tiny_gpt.py:9-33): half-split, base 10000."""
    inv_freq = 1.0 / (10000 ** (torch.arange(0, hd, 2, dtype=torch.float32) / hd))
    t = torch.arange(T, dtype=torch.float32)
    freqs = torch.outer(t, inv_freq)
    emb = torch.cat((freqs, freqs), dim=-1)
    return emb.cos(), emb.sin()


def _rotate_half(x):
    h = x.shape[-1] // 2
    return torch.cat((-x[..., h:], x[..., :h]), dim=-1)


def layer_norm(x, w, b, eps=1e-5):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b


def gelu(x):
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def cross_entropy(logits2d: torch.Tensor, targets1d: torch.Tensor, eps: float,
                  weight: torch.Tensor | None, ignore_index: int = PAD_ID) -> torch.Tensor:
    """F.cross_entropy(ignore_index, label_smoothing, weight) restated.

    L = sum_{i valid}[(1-eps) w_{y_i} (-log p_{i,y_i}) + (eps/V) sum_c w_c (-log p_{i,c})]
        / sum_{i valid} w_{y_i}                          
    All-ignored input gives 0/0 = NaN like the reference.
    """
    V = logits2d.shape[-1]
    logp = torch.log_softmax(logits2d.float(), dim=-1)
    valid = targets1d != ignore_index
    w = weight if weight is not None else torch.ones(V, dtype=torch.float32)
    safe_t = torch.where(valid, targets1d, torch.zeros_like(targets1d))
    nll = -logp.gather(1, safe_t[:, None])[:, 0]
    wy = w[safe_t]
    smooth = -(logp * w[None, :]).sum(-1)
    per_row = (1.0 - eps) * wy * nll + (eps / V) * smooth
    num = torch.where(valid, per_row, torch.zeros_like(per_row)).sum()
    den = torch.where(valid, wy, torch.zeros_like(wy)).sum()
    return num / den


# ---------------------------------------------------------------------------
# forward
# ---------------------------------------------------------------------------

def _to_t(params: dict, requires_grad: bool) -> dict:
    out = {}
    for k, v in params.items():
        t = torch.as_tensor(np.asarray(v), dtype=torch.float32).clone()
        t.requires_grad_(requires_grad)
        out[k] = t
    return out


def _block(cfg, P, i, x, mask, cos_sin, drop, training, attn_out=None):
    p = f"blocks.{i}."
    B, T, d = x.shape
    H, KV, hd = cfg.n_head, cfg.kv_heads, cfg.head_dim
    h = layer_norm(x, P[p + "ln1.weight"], P[p + "ln1.bias"])
    q = (h @ P[p + "attn.query.weight"].T + P[p + "attn.query.bias"]).view(B, T, H, hd).transpose(1, 2)
    k = (h @ P[p + "attn.key.weight"].T + P[p + "attn.key.bias"]).view(B, T, KV, hd).transpose(1, 2)
    v = (h @ P[p + "attn.value.weight"].T + P[p + "attn.value.bias"]).view(B, T, KV, hd).transpose(1, 2)
    if KV != H:
        if H % KV != 0:
            raise ValueError("n_head must be divisible by n_kv_head for GQA")
        k = k.repeat_interleave(H // KV, dim=1)
        v = v.repeat_interleave(H // KV, dim=1)
    if cos_sin is not None:
        cos, sin = cos_sin
        q = q * cos + _rotate_half(q) * sin
        k = k * cos + _rotate_half(k) * sin
    att = (q @ k.transpose(-2, -1)) / math.sqrt(hd)
    att = att.masked_fill(~mask[:, None], float("-inf"))
    att = torch.softmax(att, dim=-1)
    if attn_out is not None:  # the manual path's `last_attn` (model_tiny_gpt.py:128), before dropout
        attn_out.append(att.detach().clone())
    if training and cfg.dropout > 0 and drop is not None:
        att = att * drop(i, SITE_ATTN, att.shape)
    y = (att @ v).transpose(1, 2).reshape(B, T, d)
    x = x + (y @ P[p + "attn.proj.weight"].T + P[p + "attn.proj.bias"])
    h2 = layer_norm(x, P[p + "ln2.weight"], P[p + "ln2.bias"])
    if cfg.use_swiglu:
        g = h2 @ P[p + "mlp.w_gate.weight"].T
        u = h2 @ P[p + "mlp.w_up.weight"].T
        m = (F.silu(g) * u) @ P[p + "mlp.w_down.weight"].T
    else:
        a = h2 @ P[p + "mlp.0.weight"].T + P[p + "mlp.0.bias"]
        m = gelu(a) @ P[p + "mlp.2.weight"].T + P[p + "mlp.2.bias"]
    if training and cfg.dropout > 0 and drop is not None:
        m = m * drop(i, SITE_MLP, m.shape)
    return x + m


def _make_dropper(cfg, seed, B, T):
    """Dropout masks keyed exactly like the device kernels (row/col counters)."""
    H = cfg.n_head
    d = cfg.n_embd

    def drop(layer, site, shape):
        s = site_seed(seed, layer, site)
        if site == SITE_ATTN:
            # row = (b*H + h)*T + q, col = key
            m = dropout_mask(s, B * H * T, T, cfg.dropout)
            return m.view(B, H, T, T)
        # rows = b*T + t, col = feature
        m = dropout_mask(s, B * T, d, cfg.dropout)
        return m.view(B, T, d)
    return drop


def embed(cfg, P, idx, drop, training):
    B, T = idx.shape
    x = P["tok_emb.weight"][idx]
    if not cfg.use_rope:
        x = x + P["pos_emb.weight"][:T][None]
    if training and cfg.dropout > 0 and drop is not None:
        x = x * drop(-1, SITE_EMB, x.shape)
    return x


def forward(cfg: OracleConfig, params: dict, idx, targets=None, *, training=False,
            dropout_seed: int = 0, attention_window=None, requires_grad=False,
            return_aux=False):
    """TinyGPT.forward restated (model_tiny_gpt.py:297-352). Returns dict."""
    P = params if isinstance(next(iter(params.values())), torch.Tensor) and \
        all(isinstance(v, torch.Tensor) for v in params.values()) else _to_t(params, requires_grad)
    idx = torch.as_tensor(np.asarray(idx), dtype=torch.long)
    B, T = idx.shape
    drop = _make_dropper(cfg, dropout_seed, B, T) if (training and cfg.dropout > 0) else None
    x = embed(cfg, P, idx, drop, training)
    mask = attention_mask(idx, cfg.sep_id, attention_window)
    cos_sin = rope_cos_sin(T, cfg.head_dim) if cfg.use_rope else None
    hidden = [x]
    for i in range(cfg.n_layer):
        x = _block(cfg, P, i, x, mask, cos_sin, drop, training)
        hidden.append(x)
    xf = layer_norm(x, P["ln_f.weight"], P["ln_f.bias"])
    W_head = P["tok_emb.weight"] if cfg.tie_embeddings else P["head.weight"]
    logits = xf @ W_head.T
    out = {"params": P, "logits": logits, "hidden": hidden, "final": xf}
    aux = {}
    if cfg.termination_aux:
        aux["termination_logits"] = xf @ P["termination_head.weight"].T + P["termination_head.bias"]
    if cfg.multi_offset_targets:
        off = {}
        for k in sorted(set(int(t) for t in cfg.multi_offset_targets)):
            pp = f"offset_projs.{k}."
            z = gelu(xf @ P[pp + "0.weight"].T + P[pp + "0.bias"])
            z = z @ P[pp + "2.weight"].T + P[pp + "2.bias"]
            off[k] = z @ W_head.T
        aux["offset_logits"] = off
    out["aux"] = aux
    if targets is not None:
        tg = torch.as_tensor(np.asarray(targets), dtype=torch.long)
        w = None
        if cfg.loss_weights is not None:
            w = torch.tensor(cfg.loss_weights, dtype=torch.float32)
            if bool(torch.all(w == 1.0)):
                w = None
        out["loss"] = cross_entropy(logits.reshape(-1, cfg.vocab_size), tg.reshape(-1),
                                    cfg.label_smoothing, w)
    return out


def attention_probs(cfg: OracleConfig, params: dict, idx, attention_window=None) -> list:
    """Per-block softmax probabilities (B, H, T, T) of an eval forward -- the reference's
    `last_attn` (model_tiny_gpt.py:117-128)."""
    P = _to_t(params, False)
    idx = torch.as_tensor(np.asarray(idx), dtype=torch.long)
    B, T = idx.shape
    with torch.no_grad():
        x = embed(cfg, P, idx, None, False)
        mask = attention_mask(idx, cfg.sep_id, attention_window)
        cos_sin = rope_cos_sin(T, cfg.head_dim) if cfg.use_rope else None
        out = []
        for i in range(cfg.n_layer):
            x = _block(cfg, P, i, x, mask, cos_sin, None, False, attn_out=out)
    return out


def iter_hidden_states(cfg, params, idx, attention_window=None):
    """(0, emb), (1..L, block outputs), ("final", ln_f) -- model_tiny_gpt.py:368-389."""
    with torch.no_grad():
        o = forward(cfg, params, idx, attention_window=attention_window)
    for i, h in enumerate(o["hidden"]):
        yield i, h.detach()
    yield "final", o["final"].detach()


def forward_backward(cfg, params, idx, targets, *, training=False, dropout_seed=0):
    """loss + d(loss)/d(param) for every parameter (autograd of the restatement)."""
    P = _to_t(params, True)
    o = forward(cfg, P, idx, targets, training=training, dropout_seed=dropout_seed)
    o["loss"].backward()
    grads = {k: (v.grad.detach().clone() if v.grad is not None else torch.zeros_like(v))
             for k, v in P.items()}
    return o, grads


# ---------------------------------------------------------------------------
# optimizer / schedule
# ---------------------------------------------------------------------------

def adamw_step(p, g, m, v, step, lr, wd, beta1=0.9, beta2=0.999, eps=1e-8):
    """torch.optim.AdamW single-tensor update (defaults used at loop.py:731). In-place."""
    p.mul_(1.0 - lr * wd)
    m.mul_(beta1).add_(g, alpha=1.0 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    step_size = lr / bc1
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-step_size)
    return p


def lr_lambda(step_idx: int, warmup_steps: int, total_steps: int, lr: float, min_lr: float) -> float:
    """Cosine-with-warmup LambdaLR factor (loop.py:770-779)."""
    w = max(1, warmup_steps)
    r = (min_lr / lr) if lr > 0 else 0.0
    if step_idx < w:
        return float(step_idx + 1) / w
    progress = (step_idx - w) / max(1, total_steps - w)
    return r + (1 - r) * 0.5 * (1.0 + math.cos(math.pi * progress))


# ---------------------------------------------------------------------------
# objectives (objectives.py) and pooling (extract_embeddings.py)
# ---------------------------------------------------------------------------

def offset_target_mask(yb, offset, boundary_ids=(2, 3)):
    yb = torch.as_tensor(yb)
    if offset < 1:
        raise ValueError("offset must be >= 1")
    if offset > yb.shape[1]:
        return torch.zeros((yb.shape[0], 0), dtype=torch.bool)
    target = yb[:, offset - 1:]
    valid = target != PAD_ID
    boundary = torch.zeros_like(yb, dtype=torch.bool)
    for b in boundary_ids:
        boundary |= yb == int(b)
    for s in range(offset - 1):
        valid &= ~boundary[:, s: s + target.shape[1]]
    return valid


def termination_labels(yb, stop_ids, bucket_edges=(0, 3, 10, 30), ignore_index=-100):
    """Pure-loop restatement of termination_distance_bucket_labels (objectives.py:63-91)."""
    y = np.asarray(yb)
    B, T = y.shape
    out = np.zeros((B, T), dtype=np.int64)
    for b in range(B):
        nxt = T
        for t in range(T - 1, -1, -1):
            if int(y[b, t]) in stop_ids:
                nxt = t
            if y[b, t] == PAD_ID:
                out[b, t] = ignore_index
            elif nxt == T:
                out[b, t] = len(bucket_edges)
            else:
                dist = nxt - t
                out[b, t] = sum(1 for e in bucket_edges if dist > e)
    return out


def multi_offset_loss(offset_logits: dict, yb, offset_weights: dict, eps=0.0, loss_weights=None,
                      boundary_ids=(2, 3)):
    """multi_offset_lm_loss restated (objectives.py:26-60): CE on the gathered valid rows."""
    yb = torch.as_tensor(np.asarray(yb), dtype=torch.long)
    T = yb.shape[1]
    total = torch.zeros(())
    losses = {}
    for k, w in offset_weights.items():
        if w == 0.0 or k <= 1 or k > T or k not in offset_logits:
            continue
        valid = offset_target_mask(yb, k, boundary_ids)
        if not bool(valid.any()):
            continue
        pred = offset_logits[k][:, : T - k + 1][valid]
        tgt = yb[:, k - 1:][valid]
        lk = cross_entropy(pred, tgt, eps, loss_weights)
        losses[k] = lk
        total = total + float(w) * lk
    return total, losses


def termination_loss(term_logits, labels, class_weights=None, ignore_index=-100):
    """termination_aux_loss restated (objectives.py:94-105)."""
    nc = term_logits.shape[-1]
    lab = torch.as_tensor(np.asarray(labels), dtype=torch.long).reshape(-1)
    return cross_entropy(term_logits.reshape(-1, nc), lab, 0.0, class_weights, ignore_index)


def objective_backward(cfg, params, idx, targets, offset_weights, term_weight, stop_ids,
                       bucket_edges=(0, 3, 10, 30), term_class_weights=None):
    """The trainer's objective with aux heads (loop.py:1075-1112) and its parameter grads."""
    P = _to_t(params, True)
    o = forward(cfg, P, idx, targets)
    total = o["loss"]
    lw = None
    if cfg.loss_weights is not None and not all(float(v) == 1.0 for v in cfg.loss_weights):
        lw = torch.tensor(cfg.loss_weights, dtype=torch.float32)
    parts = {"loss": o["loss"], "aux": o["aux"]}
    if cfg.multi_offset_targets:
        off_total, off_losses = multi_offset_loss(o["aux"]["offset_logits"], targets, offset_weights,
                                                  cfg.label_smoothing, lw)
        total = total + off_total
        parts.update({f"offset_loss_{k}": v for k, v in off_losses.items()})
    if cfg.termination_aux:
        labels = termination_labels(targets, tuple(stop_ids), tuple(bucket_edges))
        cw = None if term_class_weights is None else torch.tensor(term_class_weights, dtype=torch.float32)
        tl = termination_loss(o["aux"]["termination_logits"], labels, cw)
        total = total + term_weight * tl
        parts["term_loss"] = tl
        parts["term_labels"] = labels
    total.backward()
    grads = {k: (v.grad.detach().clone() if v.grad is not None else torch.zeros_like(v)) for k, v in P.items()}
    parts["total"] = total
    return parts, grads


def pool_state(hidden, idx, mode, content_ids, pad=PAD_ID):
    hidden = torch.as_tensor(hidden)
    idx = torch.as_tensor(np.asarray(idx))
    nonpad = idx.ne(pad)
    if mode == "mean_nonpad":
        mask = nonpad
    elif mode == "mean_content":
        mask = torch.zeros_like(nonpad)
        for t in content_ids:
            mask |= idx.eq(t)
    elif mode == "eos":
        pos = nonpad.long().sum(1).sub(1).clamp_min(0)
        return hidden[torch.arange(hidden.size(0)), pos]
    else:
        raise ValueError(mode)
    w = mask.to(hidden.dtype).unsqueeze(-1)
    return (hidden * w).sum(1) / w.sum(1).clamp_min(1.0)


# ---------------------------------------------------------------------------
# CPU baseline trainer (bench.py cpu_baseline leg)
# ---------------------------------------------------------------------------

class CpuTrainer:
    """fp32 CPU restatement of one training step: fwd + CE + bwd + AdamW (loop.py:1054-1182)."""

    def __init__(self, cfg: OracleConfig, params: dict, lr=3e-4, wd=0.05):
        self.cfg = cfg
        self.P = _to_t(params, True)
        self.m = {k: torch.zeros_like(v) for k, v in self.P.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.P.items()}
        self.step_n = 0
        self.lr, self.wd = lr, wd

    def step(self, idx, targets, dropout_seed=0):
        for t in self.P.values():
            t.grad = None
        o = forward(self.cfg, self.P, idx, targets, training=True, dropout_seed=dropout_seed)
        o["loss"].backward()
        self.step_n += 1
        with torch.no_grad():
            for k, p in self.P.items():
                adamw_step(p, p.grad, self.m[k], self.v[k], self.step_n, self.lr, self.wd)
        return float(o["loss"].detach())
