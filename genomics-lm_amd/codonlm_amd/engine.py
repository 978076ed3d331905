"""Host side of the whole-model engine (cg_model_* in include/codonlm_hip.h).

Owns the device buffers of one TinyGPT instance:
  * ``flat``   -- fp32 master parameters in the library's flat layout
                  (cg_model_param_layout); nn.Parameters are views into it,
  * ``grads``  -- fp32 gradients, same layout (param.grad views),
  * ``shadow`` -- bf16 copy of ``flat`` read by the bf16 MFMA GEMMs,
  * ``workspace`` -- activations saved for backward + backward scratch, sized per (B, T).
The per-step sequence of kernels is issued by the native engine (engine.cpp); Python
only makes one call per phase.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch

from . import _lib as L


@dataclass(frozen=True)
class EngineConfig:
    vocab_size: int
    block_size: int
    n_layer: int
    n_head: int
    n_embd: int
    n_kv_head: int | None = None
    use_swiglu: bool = False
    use_rope: bool = False
    sep_id: int | None = 3
    tie_embeddings: bool = True
    termination_aux: bool = False
    termination_n_classes: int = 5
    multi_offset_targets: tuple = ()
    dropout: float = 0.0
    label_smoothing: float = 0.0
    ln_eps: float = 1e-5
    dtype: str = "fp32"  # "fp32" (parity) | "bf16" (throughput)
    # cg_model_opts fields as ((name, value), ...): measured engine alternatives (tests, A/B runs)
    opts: tuple = ()

    @property
    def head_dim(self) -> int:
        return self.n_embd // self.n_head

    def to_c(self) -> L.ModelCfg:
        c = L.ModelCfg()
        c.vocab_size = self.vocab_size
        c.block_size = self.block_size
        c.n_layer = self.n_layer
        c.n_head = self.n_head
        kv = self.n_kv_head
        c.n_kv_head = kv if (kv is not None and 0 < kv <= self.n_head) else 0
        c.n_embd = self.n_embd
        c.use_swiglu = int(self.use_swiglu)
        c.use_rope = int(self.use_rope)
        c.sep_id = -1 if self.sep_id is None else int(self.sep_id)
        c.tie_embeddings = int(self.tie_embeddings)
        c.termination_aux = int(self.termination_aux)
        c.termination_n_classes = int(self.termination_n_classes)
        offs = list(self.multi_offset_targets)[:8]
        c.n_offsets = len(offs)
        for i, o in enumerate(offs):
            c.offsets[i] = int(o)
        c.dropout = float(self.dropout)
        c.label_smoothing = float(self.label_smoothing)
        c.ln_eps = float(self.ln_eps)
        c.dtype = L.CG_BF16 if self.dtype == "bf16" else L.CG_F32
        known = {f for f, _ in L.ModelOpts._fields_}
        for k, v in self.opts:
            if k not in known:
                raise ValueError(f"unknown engine option {k!r} (cg_model_opts: {sorted(known)})")
            setattr(c.opts, k, int(v))
        return c


def param_layout(cfg: EngineConfig):
    """[(kind, layer, offset, rows, cols, ld)], total elements -- from the native layout."""
    ccfg = cfg.to_c()
    total = C.c_longlong(0)
    n = L.lib.cg_model_param_layout(C.byref(ccfg), None, 0, C.byref(total))
    if n < 0:
        L.check(n, "cg_model_param_layout")
    arr = (L.ParamEntry * n)()
    L.lib.cg_model_param_layout(C.byref(ccfg), arr, n, C.byref(total))
    return [(e.kind, e.layer, e.offset, e.rows, e.cols, e.ld) for e in arr], int(total.value)


def rope_tables(block_size: int, head_dim: int):
    """cos/sin [T][hd/2] built like RotaryEmbedding._set_cos_sin_cache (model_tiny_gpt.py:15-25)."""
    inv_freq = 1.0 / (10000 ** (torch.arange(0, head_dim, 2, dtype=torch.float32) / head_dim))
    t = torch.arange(block_size, dtype=inv_freq.dtype)
    freqs = torch.outer(t, inv_freq)
    return freqs.cos().contiguous(), freqs.sin().contiguous()


class Engine:
    def __init__(self, cfg: EngineConfig, flat: torch.Tensor, grads: torch.Tensor,
                 loss_weights: torch.Tensor | None = None):
        self.cfg = cfg
        self.flat = flat
        self.grads = grads
        self.shadow = None
        self.loss_weights = loss_weights
        self.model = L.Model()
        self.model.cfg = cfg.to_c()
        self.workspace = None
        self._ws_key = None
        self.rope_cos = self.rope_sin = None
        self._shadow_stale = True
        self._rebind()

    # -- buffers --------------------------------------------------------------------
    def _rebind(self):
        dev = self.flat.device
        if self.cfg.use_rope:
            c, s = rope_tables(self.cfg.block_size, self.cfg.head_dim)
            self.rope_cos, self.rope_sin = c.to(dev), s.to(dev)
            self.model.rope_cos = self.rope_cos.data_ptr()
            self.model.rope_sin = self.rope_sin.data_ptr()
        self.model.params = self.flat.data_ptr()
        self.model.grads = self.grads.data_ptr()
        if self.cfg.dtype == "bf16":
            if self.shadow is None or self.shadow.device != dev or self.shadow.numel() != self.flat.numel():
                self.shadow = torch.empty(self.flat.numel(), dtype=torch.bfloat16, device=dev)
            self.model.shadow = self.shadow.data_ptr()
            self._shadow_stale = True
        lw = self.loss_weights
        self.model.loss_weights = lw.data_ptr() if lw is not None else None

    def set_buffers(self, flat, grads, loss_weights=None):
        self.flat, self.grads, self.loss_weights = flat, grads, loss_weights
        self.workspace = None
        self._ws_key = None
        self._rebind()

    def mark_params_changed(self):
        """Call after writing master params outside cg_adamw (load_state_dict, init)."""
        self._shadow_stale = True

    def sync_shadow(self, stream=None):
        if self.cfg.dtype != "bf16" or not self._shadow_stale:
            return
        s = stream if stream is not None else L.stream_ptr(self.flat.device)
        L.check(L.lib.cg_cast_f32_to_bf16(self.flat.data_ptr(), self.shadow.data_ptr(), self.flat.numel(), s),
                "cg_cast_f32_to_bf16")
        self._shadow_stale = False

    def _ensure_workspace(self, B: int, T: int):
        need = int(L.lib.cg_model_workspace_bytes(C.byref(self.model.cfg), B, T))
        if need <= 0:
            raise ValueError("invalid model configuration for workspace sizing")
        if self.workspace is None or self.workspace.numel() < need or self._ws_key != (B, T):
            if self.workspace is None or self.workspace.numel() < need:
                self.workspace = torch.empty(need, dtype=torch.uint8, device=self.flat.device)
            self._ws_key = (B, T)
        self.model.workspace = self.workspace.data_ptr()
        self.model.workspace_bytes = self.workspace.numel()

    # -- compute ----------------------------------------------------------------------
    def forward(self, idx: torch.Tensor, targets: torch.Tensor | None, *, training: bool, seed: int = 0,
                window: int | None = None, logits: torch.Tensor | None = None,
                loss: torch.Tensor | None = None):
        L.require_device(idx, "TinyGPT.forward")
        if idx.dim() != 2:
            raise ValueError("idx must be (B, T)")
        B, T = idx.shape
        if T > self.cfg.block_size:
            raise ValueError(f"sequence length {T} exceeds block_size {self.cfg.block_size}")
        if window is not None and int(window) < 1:
            raise ValueError("attention_window must be at least 1")
        dev = self.flat.device
        idx = idx.to(device=dev, dtype=torch.int64).contiguous()
        if targets is not None:
            targets = targets.to(device=dev, dtype=torch.int64).contiguous()
            if targets.shape != idx.shape:
                raise ValueError("targets must have the same shape as idx")
        self._ensure_workspace(B, T)
        self.sync_shadow()
        if logits is None:
            logits = torch.empty(B, T, self.cfg.vocab_size, dtype=torch.float32, device=dev)
        if targets is not None and loss is None:
            loss = torch.empty((), dtype=torch.float32, device=dev)
        self._idx, self._targets = idx, targets  # keep alive for backward
        st = L.stream_ptr(dev)
        L.check(L.lib.cg_model_forward(C.byref(self.model), idx.data_ptr(),
                                       targets.data_ptr() if targets is not None else None,
                                       B, T, int(bool(training)), int(seed) & 0xFFFFFFFF,
                                       int(window) if window is not None else 0,
                                       logits.data_ptr(), loss.data_ptr() if loss is not None else None, st),
                "cg_model_forward")
        return logits, loss

    def aux_forward(self):
        """Aux heads of the last forward (model_tiny_gpt.py:329-337): termination logits
        fp32 (M, n_classes) or None, and [offset logits fp32 (M, V)] in offset order."""
        cfg = self.cfg
        dev = self.flat.device
        M = self.model.B * self.model.T
        term = None
        if cfg.termination_aux:
            term = torch.empty(M, cfg.termination_n_classes, dtype=torch.float32, device=dev)
        # rows padded to a multiple of 16 columns (the GEMM then takes the vector tiles); the
        # callers see [:, :V] views
        Vp = (cfg.vocab_size + 15) // 16 * 16
        offs = [torch.empty(M, Vp, dtype=torch.float32, device=dev) for _ in cfg.multi_offset_targets]
        arr = (C.c_void_p * len(offs))(*[o.data_ptr() for o in offs]) if offs else None
        L.check(L.lib.cg_model_aux_forward(C.byref(self.model), term.data_ptr() if term is not None else None,
                                           term.stride(0) if term is not None else 0, arr, Vp, L.stream_ptr(dev)),
                "cg_model_aux_forward")
        return term, [o[:, :cfg.vocab_size] for o in offs]

    def set_head_grads(self, scale: float, d_term=None, d_offsets=None, scale_dev=None):
        """Gradients phase 0 consumes: the next-codon loss scale (host float, times the device
        float ``scale_dev`` when given -- the autograd output gradient, read in-kernel so the
        backward needs no host sync) and the aux-head logit gradients (fp32, flattened to
        (M, cols)); None = that head is unused."""
        m = self.model
        m.head_grad_scale = float(scale)
        keep = []
        m.head_grad_scale_dev = None
        if scale_dev is not None:
            sd = scale_dev.detach().reshape(1).to(torch.float32).contiguous()
            keep.append(sd)
            m.head_grad_scale_dev = sd.data_ptr()
        m.d_term_logits, m.ld_d_term = None, 0
        if d_term is not None:
            t = d_term.reshape(-1, d_term.shape[-1]).to(torch.float32).contiguous()
            keep.append(t)
            m.d_term_logits, m.ld_d_term = t.data_ptr(), t.stride(0)
        for i in range(8):
            m.d_offset_logits[i] = None
        for i, g in enumerate(d_offsets or []):
            if g is None:
                continue
            t = g.reshape(-1, g.shape[-1]).to(torch.float32).contiguous()
            keep.append(t)
            m.d_offset_logits[i] = t.data_ptr()
        self._grad_keep = keep  # alive until the backward kernels are enqueued

    # -- incremental decoding (KV cache) -------------------------------------------------
    def new_kv_cache(self, B: int, Tmax: int | None = None) -> "KVCache":
        return KVCache(self, B, Tmax or self.cfg.block_size)

    def backward_phase(self, phase: int, layer: int = 0, accumulate: bool = False):
        st = L.stream_ptr(self.flat.device)
        L.check(L.lib.cg_model_backward(C.byref(self.model), phase, layer, int(bool(accumulate)), st),
                f"cg_model_backward(phase={phase}, layer={layer})")

    def backward(self, accumulate: bool = False, bucket_hook=None):
        """Full backward; ``bucket_hook(name)`` runs as soon as a bucket's gradients are final
        (the DDP overlap point): "head" after phase 0, block l once its dW group has been
        issued (cg_model.dw_done_layer), "embed" after phase 2."""
        self.backward_phase(0, 0, accumulate)
        if bucket_hook:
            bucket_hook("head")
        done = self.cfg.n_layer
        for layer in range(self.cfg.n_layer - 1, -1, -1):
            self.backward_phase(1, layer, accumulate)
            if bucket_hook:
                for b in range(done - 1, self.model.dw_done_layer - 1, -1):
                    bucket_hook(b)
            done = min(done, self.model.dw_done_layer)
        self.backward_phase(2, 0, accumulate)
        if bucket_hook:
            bucket_hook("embed")

    def attn_probs(self, layer: int) -> torch.Tensor:
        """Attention probabilities of block `layer` of the last forward: fp32 (B, H, T, T)."""
        B, T, H = self.model.B, self.model.T, self.cfg.n_head
        dev = self.flat.device
        out = torch.empty(B, H, T, T, dtype=torch.float32, device=dev)
        L.check(L.lib.cg_model_attn_probs(C.byref(self.model), int(layer), out.data_ptr(), L.stream_ptr(dev)),
                "cg_model_attn_probs")
        return out

    def hidden(self, which: int) -> torch.Tensor:
        dt = C.c_int(0)
        ld = C.c_longlong(0)
        ptr = L.lib.cg_model_hidden(C.byref(self.model), which, C.byref(dt), C.byref(ld))
        if not ptr:
            raise ValueError(f"no hidden state {which}")
        B, T, d = self.model.B, self.model.T, self.cfg.n_embd
        base = self.workspace.data_ptr()
        off = ptr - base
        if dt.value == L.CG_F32:
            t = self.workspace[off: off + B * T * d * 4].view(torch.float32)
        else:
            t = self.workspace[off: off + B * T * d * 2].view(torch.bfloat16)
        return t.view(B, T, d)


class KVCache:
    """Per-sequence K/V rows of every layer for incremental decoding (cg_model_prefill /
    cg_model_decode): one prefill of the prompt, then one native call per generated token
    instead of the reference's full re-forward of the prefix (query_model.py:160-214).
    Valid while the sequence fits ``Tmax`` <= block_size."""

    def __init__(self, engine: Engine, B: int, Tmax: int):
        cfg = engine.cfg
        if Tmax > cfg.block_size:
            raise ValueError("Tmax exceeds block_size")
        self.eng, self.B, self.Tmax = engine, int(B), int(Tmax)
        dev = engine.flat.device
        nbytes = int(L.lib.cg_kv_cache_bytes(C.byref(engine.model.cfg), self.B, self.Tmax))
        self.cache = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
        self.seg = torch.zeros(self.B, dtype=torch.int32, device=dev)
        wsb = int(L.lib.cg_decode_workspace_bytes(C.byref(engine.model.cfg), self.B))
        self.ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        self.pos = 0

    @torch.no_grad()
    def prefill(self, idx: torch.Tensor, window: int | None = None) -> torch.Tensor:
        """Eval forward of the prompt (B, T); returns fp32 logits (B, T, V)."""
        eng = self.eng
        L.require_device(idx, "KVCache.prefill")
        B, T = idx.shape
        if B != self.B or T > self.Tmax:
            raise ValueError(f"prompt {tuple(idx.shape)} does not fit the cache (B={self.B}, Tmax={self.Tmax})")
        idx = idx.to(torch.int64).contiguous()
        eng._ensure_workspace(B, T)
        eng.sync_shadow()
        logits = torch.empty(B, T, eng.cfg.vocab_size, dtype=torch.float32, device=idx.device)
        eng._idx, eng._targets = idx, None
        L.check(L.lib.cg_model_prefill(C.byref(eng.model), idx.data_ptr(), B, T, int(window or 0),
                                       self.cache.data_ptr(), self.Tmax, self.seg.data_ptr(), logits.data_ptr(),
                                       L.stream_ptr(idx.device)), "cg_model_prefill")
        self.pos = T
        return logits

    @torch.no_grad()
    def decode(self, tok: torch.Tensor) -> torch.Tensor:
        """Append one token per sequence (B,) at the current position; returns logits (B, V)."""
        eng = self.eng
        if self.pos >= self.Tmax:
            raise ValueError("KV cache is full (the context reached Tmax)")
        tok = tok.reshape(self.B).to(device=self.cache.device, dtype=torch.int64).contiguous()
        eng.sync_shadow()
        logits = torch.empty(self.B, eng.cfg.vocab_size, dtype=torch.float32, device=tok.device)
        L.check(L.lib.cg_model_decode(C.byref(eng.model), tok.data_ptr(), self.B, self.pos, self.cache.data_ptr(),
                                      self.Tmax, self.seg.data_ptr(), self.ws.data_ptr(), self.ws.numel(),
                                      logits.data_ptr(), L.stream_ptr(tok.device)), "cg_model_decode")
        self._tok = tok
        self.pos += 1
        return logits
