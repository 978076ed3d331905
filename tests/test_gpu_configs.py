"""The BASELINE geometries on both engines vs the pinned oracle.

The bf16 engine is the path behind every throughput number (persistent / LDS-DMA MFMA
GEMMs, the dW tiles, the 32x32x16 MFMA attention kernels), so it is pinned here at the
real kernel shapes -- d512 hd64 T1024, d384 hd48 KV4 T512 with RoPE + SwiGLU, d256 T512,
d384 hd48 with the five offset heads + termination head -- against the CPU oracle
(oracle/tinygpt_oracle.py, itself pinned to the reference's golden vectors).  Each config
runs at its REAL depth (C1 4L, C2 6L, C3 10L, C4 12L, C5 10L) at B=2, and the bf16 engine is
told to plan its grouped weight gradients as for the benchmark's token count (engine_opts
dw_plan_tokens = bench B x T; the plan depends on B*T through the token-range split): C4's groups
of 5/5/2 blocks with the 256x256 dW tile, C2's one 6-block group split 3 ways over the tokens,
C5's 4/4/2 with the split remainder, slot reuse across groups, the per-group deferred
reductions.  The oracle's fp32 autograd of a 12-layer T1024 B=2 step takes a few seconds.  Three more legs pin what the throughput runs do beyond the plain step:
  * dropout 0.1 in training mode (the bench's setting): the engine's keep masks are the
    counter hash the oracle restates bit-for-bit, so the bf16 step with dropout is compared
    against O.forward_backward(training=True) at the same bounds;
  * ragged token counts: the dynamic-length loader pads each batch only to its own longest
    sequence (data_loading.py:380-393), so B*T is arbitrary -- B=3, T=T_cfg/3 - 1 gives
    B*T % 64 != 0 through every kernel, the grouped dW's zero-filled last k-step included.

Bounds.  fp32 engine: logits within an absolute bound ~5x the error measured at each geometry
(FP32_LOGIT_ABS, 3e-4 .. 2.5e-3 against logit scales of 116-391), the loss within the north-star
1e-4, every parameter gradient within 2e-4 of its largest entry.  bf16 engine: bf16 storage of
weights and activations (8 significant bits, rounding 2^-9 relative per value) with fp32
accumulation everywhere; through 4-12 residual blocks, the head and the loss that gives
relative L2 errors of a few 1e-3 (measured at full depth on the MI355X: 1.2-1.9e-3 logits,
<= 6.5e-3 for every gradient but the RoPE configs' key biases at <= 1.43e-2, identical with
dropout and at ragged B*T), so the bounds are
rel-L2 <= 5e-3 for logits and
<= 1.5e-2 for every parameter gradient (without RoPE the key biases are exactly zero in exact
arithmetic -- softmax shift invariance -- and are only checked to be at noise level).
ln_f.bias's gradient is the column sum over all tokens of d(loss)/d(xf) = dlogits . E, which
cancels to a small value; the engine therefore keeps dlogits as split bf16 (hi + lo,
CG_BF16X2) for that product, and it is held to the same bound as every other gradient.
"""
import numpy as np
import pytest
import torch

from oracle import tinygpt_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"

LOGIT_REL_L2_BF16 = 5e-3
GRAD_REL_L2_BF16 = 1.5e-2
TOL_FP32 = 1e-4
# fp32 logits, absolute: ~5x the max |dlogit| measured on the MI355X at these full-depth geometries
# (round 5: C1 5.3e-5, C2 1.7e-4, C3 4.6e-4, C4 4.0e-4, C5 2.4e-4 over plain + ragged), against
# logit scales of 116-391 (the N(0,1) embeddings) -- i.e. 1.3e-6 relative at worst, where the
# north star's "1e-4" relative reading would allow 3.9e-2.  The trained-scale (std 0.02) leg with
# the literal absolute 1e-4 is tests/test_gpu_greedy_neartie.py, at these same depths.
FP32_LOGIT_ABS = {"C1": 3e-4, "C2": 8e-4, "C3": 2.5e-3, "C4": 2e-3, "C5": 1.2e-3}

# per-GPU microbatch of each config's bench line (bench.py CONFIGS): the dW plan the parity runs take
BENCH_B = {"C2": 256, "C3": 256, "C4": 32, "C5": 128}
# (oracle config kwargs, microbatch B); C5 = stage2.6_large_scaling + its aux heads
CONFIGS = {
    "C1": (dict(n_layer=4, n_head=2, n_embd=128, block_size=512), 2),
    "C2": (dict(n_layer=6, n_head=4, n_embd=256, block_size=512), 2),
    "C3": (dict(n_layer=10, n_head=8, n_kv_head=4, n_embd=384, block_size=512, use_swiglu=True, use_rope=True,
                loss_weights=None), 2),
    "C4": (dict(n_layer=12, n_head=8, n_embd=512, block_size=1024), 2),
    "C5": (dict(n_layer=10, n_head=8, n_embd=384, block_size=512, termination_aux=True,
                multi_offset_targets=[2, 4, 8, 16, 32]), 2),
}
OFFSET_W = {2: 0.2, 4: 0.2, 8: 0.2, 16: 0.2, 32: 0.2}
TERM_W = 0.1


def _eos_weights(V=68, w=3.0):
    lw = [1.0] * V
    for t in (2, 52, 54, 60):  # <EOS_CDS>, TAA, TAG, TGA (loop.py:396-405)
        lw[t] = w
    return lw


def packed_batch(B, T, seed):
    """Packed CDS windows: BOS .. codons .. EOS, SEP between CDSs, a PAD tail on the last row."""
    rng = np.random.default_rng(seed)
    tok = rng.integers(4, 68, size=(B, T + 1))
    for b in range(B):
        p = 0
        while p < T + 1:
            n = int(rng.integers(40, 400))
            tok[b, p] = 1
            e = min(T, p + n)
            tok[b, e] = 2
            if e + 1 <= T:
                tok[b, e + 1] = 3
            p = e + 2
    tok[-1, -(T // 7):] = 0
    return tok[:, :-1].copy(), tok[:, 1:].copy()


def _cfg(name, label_smoothing=0.05):
    kw, B = CONFIGS[name]
    kw = dict(kw)
    if name == "C3":
        kw["loss_weights"] = _eos_weights()
    return O.OracleConfig(vocab_size=68, label_smoothing=label_smoothing, **kw), B


def _model(cfg, params, dtype, dropout=0.0, name=None):
    from codonlm_amd import TinyGPT
    opts = {}
    if dtype == "bf16" and name in BENCH_B:
        opts["dw_plan_tokens"] = BENCH_B[name] * cfg.block_size
    m = TinyGPT(cfg.vocab_size, cfg.block_size, n_layer=cfg.n_layer, n_head=cfg.n_head, n_embd=cfg.n_embd,
                dropout=dropout, label_smoothing=cfg.label_smoothing, sep_id=cfg.sep_id, n_kv_head=cfg.n_kv_head,
                loss_weights=cfg.loss_weights, termination_aux=cfg.termination_aux,
                multi_offset_targets=cfg.multi_offset_targets or None, use_swiglu=cfg.use_swiglu,
                use_rope=cfg.use_rope, compute_dtype=dtype, device=DEV, engine_opts=opts)
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    assert not unexpected
    m.train()
    return m


def _gpu_objective(m, cfg, x, y):
    from codonlm_amd.training import objectives as obj
    if not (cfg.termination_aux or cfg.multi_offset_targets):
        logits, loss = m(x, y)
        return logits, loss, loss
    logits, loss, aux = m(x, y, return_aux=True)
    off_total, _ = obj.multi_offset_lm_loss(aux["offset_logits"], y, OFFSET_W, label_smoothing=cfg.label_smoothing)
    labels = obj.termination_distance_bucket_labels(y, stop_ids=(2,))
    term = obj.termination_aux_loss(aux["termination_logits"], labels)
    return logits, loss, loss + off_total + TERM_W * term


def _oracle(cfg, params, x, y):
    if not (cfg.termination_aux or cfg.multi_offset_targets):
        o, grads = O.forward_backward(cfg, params, x, y)
        return o["logits"].detach(), float(o["loss"]), float(o["loss"]), grads
    parts, grads = O.objective_backward(cfg, params, x, y, OFFSET_W, TERM_W, (2,))
    with torch.no_grad():
        o = O.forward(cfg, params, x, y)
    return o["logits"], float(parts["loss"]), float(parts["total"]), grads


def _rel_l2(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a - b).norm() / max(1e-30, float(b.norm())))


_REF_CACHE = {}
DROP_P, DROP_SEED = 0.1, 90210


def _reference(name, variant="plain"):
    """(cfg, params, x, y, oracle results) for a config: variant "plain" (B=2, T=block_size),
    "ragged" (B=3, T=block_size/3 - 1: B*T % 64 != 0) or "dropout" (plain shapes, training-mode
    dropout 0.1 with DROP_SEED)."""
    key = (name, variant)
    if key not in _REF_CACHE:
        cfg, B = _cfg(name)
        params = O.synthetic_params(cfg, seed=11 + len(name))
        T = cfg.block_size
        if variant == "ragged":
            B, T = 3, cfg.block_size // 3 - 1
        x, y = packed_batch(B, T, seed=5)
        torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
        if variant == "dropout":
            cfg.dropout = DROP_P
            o, grads = O.forward_backward(cfg, params, x, y, training=True, dropout_seed=DROP_SEED)
            res = (o["logits"].detach(), float(o["loss"]), float(o["loss"]), grads)
        else:
            res = _oracle(cfg, params, x, y)
        _REF_CACHE[key] = (cfg, params, x, y, res)
    return _REF_CACHE[key]


@pytest.mark.parametrize("variant", ["plain", "ragged"])
@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_bf16_engine_matches_oracle(name, variant):
    cfg, params, x, y, (rlogits, rloss, rtotal, rgrads) = _reference(name, variant)
    if variant == "ragged":
        assert (x.shape[0] * x.shape[1]) % 64 != 0
    m = _model(cfg, params, "bf16", name=name)
    xd, yd = torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)
    logits, loss, total = _gpu_objective(m, cfg, xd, yd)
    total.backward()
    torch.cuda.synchronize()
    _check_bf16(m, cfg, name, logits, loss, total, rlogits, rloss, rtotal, rgrads)


@pytest.mark.parametrize("name", ["C2", "C3", "C4"])
def test_bf16_engine_dropout_matches_oracle(name):
    """Training-mode dropout 0.1 (embedding, attention probabilities via the precomputed keep
    bits, MLP output) at full depth: the masks are the oracle's hash, so the bounds are the
    dropout-free ones."""
    cfg, params, x, y, (rlogits, rloss, rtotal, rgrads) = _reference(name, "dropout")
    m = _model(cfg, params, "bf16", dropout=DROP_P, name=name)
    xd, yd = torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)
    logits, loss = m.engine.forward(xd, yd, training=True, seed=DROP_SEED)
    m.engine.backward(accumulate=False)
    torch.cuda.synchronize()
    _check_bf16(m, cfg, name + "-dropout", logits, loss, loss, rlogits, rloss, rtotal, rgrads)


def _check_bf16(m, cfg, name, logits, loss, total, rlogits, rloss, rtotal, rgrads):
    lg = logits.detach().float().cpu().reshape(rlogits.shape)
    el = _rel_l2(lg, rlogits)
    assert el <= LOGIT_REL_L2_BF16, (name, "logits", el)
    assert abs(loss.item() - rloss) <= 1e-2 * abs(rloss), (name, loss.item(), rloss)
    assert abs(total.item() - rtotal) <= 1e-2 * abs(rtotal), (name, total.item(), rtotal)
    # greedy next-codon ids agree wherever the oracle's top-2 margin exceeds the bf16 logit error
    top2 = torch.topk(rlogits, 2, dim=-1).values
    margin = (top2[..., 0] - top2[..., 1])
    resolvable = margin > 4 * LOGIT_REL_L2_BF16 * float(rlogits.abs().max())
    agree = (lg.argmax(-1) == rlogits.argmax(-1)) | ~resolvable
    assert bool(agree.all()), (name, int((~agree).sum()))
    worst, noise = [], []
    for k, p in m.named_parameters():
        ref = rgrads[k]
        got = p.grad.detach().float().cpu()
        if k.endswith("attn.key.bias") and not cfg.use_rope:  # (RoPE breaks the shift invariance)
            scale = max(float(rgrads[k.replace("key.bias", "query.bias")].abs().max()), 1e-6)
            noise.append((float(got.abs().max()) / scale, k))
            continue
        worst.append((_rel_l2(got, ref), k))
    worst.sort(reverse=True)
    print(f"[{name} bf16] logits rel-L2 {el:.2e}; worst grads {[(k, f'{e:.2e}') for e, k in worst[:4]]}")
    assert worst[0][0] <= GRAD_REL_L2_BF16, (name, worst[:4])
    assert all(r <= 2e-2 for r, _ in noise), (name, noise)


@pytest.mark.parametrize("variant", ["plain", "ragged"])
@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_fp32_engine_matches_oracle(name, variant):
    cfg, params, x, y, (rlogits, rloss, rtotal, rgrads) = _reference(name, variant)
    m = _model(cfg, params, "fp32")
    xd, yd = torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)
    logits, loss, total = _gpu_objective(m, cfg, xd, yd)
    total.backward()
    lg = logits.detach().cpu()
    scale = max(1.0, float(rlogits.abs().max()))
    abs_err = float((lg - rlogits).abs().max())
    print(f"[{name}-{variant} fp32] max |dlogit| {abs_err:.2e} (bound {FP32_LOGIT_ABS[name]:.1e} absolute; "
          f"max|logit| {scale:.2f}); loss {loss.item():.6f} vs {rloss:.6f}")
    assert abs_err <= FP32_LOGIT_ABS[name], (name, abs_err)
    assert abs(loss.item() - rloss) <= TOL_FP32 * max(1.0, abs(rloss)), name
    assert abs(total.item() - rtotal) <= TOL_FP32 * max(1.0, abs(rtotal)), name
    # bit-exact greedy ids wherever the oracle's top-2 margin is resolvable at fp32
    top2 = torch.topk(rlogits, 2, dim=-1).values
    resolvable = (top2[..., 0] - top2[..., 1]) > 1e-3 * scale
    assert bool(((lg.argmax(-1) == rlogits.argmax(-1)) | ~resolvable).all()), name
    for k, p in m.named_parameters():
        ref = rgrads[k]
        s = max(1e-3, float(ref.abs().max()))
        err = float((p.grad.detach().cpu() - ref).abs().max())
        assert err <= 2 * TOL_FP32 * s, (name, k, err, s)
