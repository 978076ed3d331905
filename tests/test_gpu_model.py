"""Model-level parity of the MI355X TinyGPT against the reference's golden vectors.

The golden fixtures (tests/golden/*.npz) hold outputs of the real reference TinyGPT
(src/codonlm/model_tiny_gpt.py) run in the build container.  fp32 mode must match them
to the north-star tolerance (logits within 1e-4 absolute or 5e-6 of the logit scale when that
is larger, loss within 1e-4, bit-exact greedy ids); bf16 mode is checked against the same vectors with a bf16 bound.
"""
import math

import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import tinygpt_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
CASES = ["mha_gelu_sep", "gqa_rope_swiglu_w", "untied_causal", "hd48_gqa", "window8", "c4_layer"]


def make_model(cfgd, g, dtype="fp32", dropout=0.0):
    from codonlm_amd import TinyGPT
    cfg = O.OracleConfig(**cfgd)
    params = ({k[6:]: v for k, v in g.items() if k.startswith("param/")}
              or O.synthetic_params(cfg, seed=int(g["param_seed"])))
    m = TinyGPT(cfg.vocab_size, cfg.block_size, n_layer=cfg.n_layer, n_head=cfg.n_head, n_embd=cfg.n_embd,
                dropout=dropout, label_smoothing=cfg.label_smoothing, sep_id=cfg.sep_id,
                tie_embeddings=cfg.tie_embeddings, n_kv_head=cfg.n_kv_head, loss_weights=cfg.loss_weights,
                termination_aux=cfg.termination_aux, termination_n_classes=cfg.termination_n_classes,
                multi_offset_targets=cfg.multi_offset_targets or None,
                use_swiglu=cfg.use_swiglu, use_rope=cfg.use_rope, compute_dtype=dtype, device=DEV)
    sd = {k: torch.from_numpy(v) for k, v in params.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected
    assert all(k.endswith("attn.mask") or k in ("loss_weights", "head.weight") for k in missing), missing
    return m, cfg, params


def _idx(g):
    return torch.from_numpy(g["idx"]).to(DEV), torch.from_numpy(g["targets"]).to(DEV)


@pytest.mark.parametrize("case", CASES)
def test_fp32_forward_matches_reference(case):
    cfgd, g = load_golden(case)
    m, cfg, _ = make_model(cfgd, g)
    m.eval()
    x, y = _idx(g)
    window = 8 if case == "window8" else None
    with torch.no_grad():
        logits, loss = m(x, y, attention_window=window)
    ref = g["logits"]
    got = logits.cpu().numpy()
    scale = max(1.0, float(np.abs(ref).max()))
    err = float(np.abs(got - ref).max())
    print(f"[{case} fp32] max |dlogit| {err:.2e}, max |logit| {scale:.2f}")
    # fp32 against the reference's own fp32 logits: the kernels' summation order only (measured at the
    # full-depth configs: <= 1.3e-6 of the logit scale); 5e-6 of the scale, absolute floor 1e-4
    assert err <= max(1e-4, 5e-6 * scale), (err, scale)
    assert abs(loss.item() - float(g["loss"])) <= 1e-4 * max(1.0, abs(float(g["loss"])))
    # greedy next-codon ids bit-exact wherever the reference's top-2 margin is resolvable
    greedy = got.argmax(-1)
    diff = greedy != g["greedy"]
    assert not np.any(diff & (g["top2_margin"] > 1e-3 * scale)), int(diff.sum())


@pytest.mark.parametrize("case,dtype", [("mha_gelu_sep", "fp32"), ("gqa_rope_swiglu_w", "fp32"),
                                        ("window8", "fp32"), ("hd48_gqa", "bf16")])
def test_last_attn_capture(case, dtype):
    """model.capture_attn = True records blocks[i].attn.last_attn (B, H, T, T), the softmax
    probabilities before dropout (reference manual path, model_tiny_gpt.py:128), against the
    oracle's (SEP segments, RoPE + GQA, local window; fp32 1e-5, bf16 operands 2e-2)."""
    cfgd, g = load_golden(case)
    m, cfg, params = make_model(cfgd, g, dtype=dtype)
    m.eval()
    m.capture_attn = True
    x, _ = _idx(g)
    window = 8 if case == "window8" else None
    with torch.no_grad():
        m(x, attention_window=window)
    ref = O.attention_probs(cfg, params, g["idx"], attention_window=window)
    tol = 1e-5 if dtype == "fp32" else 2e-2
    for i, blk in enumerate(m.blocks):
        got = blk.attn.last_attn.cpu()
        assert got.shape == ref[i].shape
        assert float((got - ref[i]).abs().max()) <= tol, (i, float((got - ref[i]).abs().max()))


@pytest.mark.parametrize("case", ["mha_gelu_sep", "gqa_rope_swiglu_w", "untied_causal", "hd48_gqa"])
def test_fp32_grads_match_reference(case):
    cfgd, g = load_golden(case)
    m, cfg, _ = make_model(cfgd, g)
    m.train()
    x, y = _idx(g)
    logits, loss = m(x, y)
    loss.backward()
    named = dict(m.named_parameters())
    for k, p in named.items():
        ref = g.get(f"grad/{k}")
        if ref is None:
            continue
        got = p.grad.detach().cpu().numpy()
        s = max(1e-3, float(np.abs(ref).max()))
        err = float(np.abs(got - ref).max())
        assert err <= 2e-4 * s, (k, err, s)


def test_c4_layer_grad_sums():
    cfgd, g = load_golden("c4_layer")
    m, cfg, _ = make_model(cfgd, g)
    m.train()
    x, y = _idx(g)
    _, loss = m(x, y)
    loss.backward()
    for k, p in m.named_parameters():
        ref = g.get(f"gradsum/{k}")
        if ref is None or k.endswith("attn.key.bias"):
            # softmax is shift-invariant per query row: d(loss)/d(key.bias) == 0 exactly,
            # both sides hold only rounding noise (~1e-8)
            continue
        gg = p.grad.detach().double().cpu()
        tot, asum, sq = float(gg.sum()), float(gg.abs().sum()), float(gg.pow(2).sum())
        assert abs(asum - ref[1]) <= 1e-3 * max(1e-6, ref[1]), (k, asum, ref[1])
        assert abs(sq - ref[2]) <= 2e-3 * max(1e-12, ref[2]), (k, sq, ref[2])
        assert abs(tot - ref[0]) <= 1e-3 * max(1e-6, ref[1]), (k, tot, ref[0])


@pytest.mark.parametrize("case", ["mha_gelu_sep", "hd48_gqa"])
def test_hidden_states_and_pooling(case):
    cfgd, g = load_golden(case)
    m, cfg, _ = make_model(cfgd, g)
    m.eval()
    x, _ = _idx(g)
    states = list(m.iter_hidden_states(x))
    assert [s[0] for s in states] == list(range(cfg.n_layer + 1)) + ["final"]
    for layer, h in states:
        ref = g[f"hidden/{layer}"]
        s = max(1.0, float(np.abs(ref).max()))
        assert float(np.abs(h.cpu().numpy() - ref).max()) <= 2e-5 * s
        for mode in ("mean_nonpad", "mean_content", "eos"):
            pooled = O.pool_state(h.cpu(), g["idx"], mode, list(range(4, 68))).numpy()
            assert float(np.abs(pooled - g[f"pooled/{layer}/{mode}"]).max()) <= 2e-5 * s


def test_adamw_two_steps_match_reference():
    from codonlm_amd.optim import FusedAdamW
    cfgd, g = load_golden("mha_gelu_sep")
    m, cfg, _ = make_model(cfgd, g)
    m.train()
    opt = FusedAdamW(m, lr=float(g["adamw_lr"]), weight_decay=float(g["adamw_wd"]))
    x, y = _idx(g)
    for _ in range(2):
        opt.zero_grad()
        _, loss = m(x, y)
        loss.backward()
        opt.step()
    for k, p in m.named_parameters():
        ref = g.get(f"adamw2/{k}")
        if ref is None:
            continue
        atol = 2.5 * float(g["adamw_lr"]) if k.endswith("attn.key.bias") else 2e-6
        np.testing.assert_allclose(p.detach().cpu().numpy(), ref, rtol=1e-5, atol=atol, err_msg=k)


@pytest.mark.parametrize("case", ["mha_gelu_sep", "gqa_rope_swiglu_w"])
def test_dropout_training_matches_oracle(case):
    """Dropout masks come from the counter hash the oracle restates bit-for-bit."""
    cfgd, g = load_golden(case)
    m, cfg, params = make_model(cfgd, g, dropout=0.1)
    cfg.dropout = 0.1
    x, y = _idx(g)
    seed = 4242
    m.train()
    logits, loss = m.engine.forward(x, y, training=True, seed=seed)
    m.engine.backward(accumulate=False)
    o, grads = O.forward_backward(cfg, params, g["idx"], g["targets"], training=True, dropout_seed=seed)
    assert abs(loss.item() - float(o["loss"])) <= 1e-4 * max(1.0, abs(float(o["loss"])))
    named = dict(m.named_parameters())
    for k, ref in grads.items():
        got = named[k].grad.detach().cpu().numpy()
        ref = ref.numpy()
        s = max(1e-3, float(np.abs(ref).max()))
        assert float(np.abs(got - ref).max()) <= 2e-4 * s, k


@pytest.mark.parametrize("case", ["mha_gelu_sep", "gqa_rope_swiglu_w", "hd48_gqa", "c4_layer"])
def test_bf16_forward_close_to_reference(case):
    cfgd, g = load_golden(case)
    m, cfg, _ = make_model(cfgd, g, dtype="bf16")
    m.eval()
    x, y = _idx(g)
    with torch.no_grad():
        logits, loss = m(x, y)
    ref = g["logits"]
    got = logits.cpu().numpy()
    rel = float(np.abs(got - ref).max()) / max(1.0, float(np.abs(ref).max()))
    assert rel < 3e-2, rel
    assert abs(loss.item() - float(g["loss"])) <= 3e-2 * abs(float(g["loss"])) + 0.05
    agree = (got.argmax(-1) == g["greedy"]).mean()
    assert agree > 0.9, agree


def test_bf16_training_reduces_loss():
    from codonlm_amd import TinyGPT
    from codonlm_amd.optim import FusedAdamW
    torch.manual_seed(0)
    m = TinyGPT(68, 128, n_layer=2, n_head=4, n_embd=128, dropout=0.1, label_smoothing=0.05,
                compute_dtype="bf16", device=DEV)
    opt = FusedAdamW(m, lr=1e-3, weight_decay=0.05)
    rng = np.random.default_rng(1)
    # a learnable pattern: periodic codon sequences
    base = rng.integers(4, 68, size=(8, 16))
    seq = np.tile(base, (1, 9))[:, :129]
    x = torch.from_numpy(seq[:, :-1]).to(DEV)
    y = torch.from_numpy(seq[:, 1:]).to(DEV)
    m.train()
    losses = []
    for _ in range(60):
        opt.zero_grad()
        _, loss = m(x, y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert all(math.isfinite(v) for v in losses)
    assert losses[-1] < 0.5 * losses[0], (losses[0], losses[-1])
