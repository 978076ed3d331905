"""The grouped weight-gradient plan of the bf16 engine (engine.cpp dw_plan / flush_dw).

* the tied head's weight gradient, deferred from backward phase 0 into the first grouped dW
  launch: deferral on vs off, and the phase-2 fallback of a partial phase sequence
  (phase 0 then phase 2, no dW group to take the product);
* the token-range split of the grouped dW tiles (engine_opts dw_ksplit 2 / 3 against 1) at C2
  geometry, where the planner's own choice is a 3-way split, and cg_model_dw_plan reporting it;
* the group plans priced by tools/bucket_replay.py (short group first / last, 4/4/4, 6/6) give
  the gradients of one block per launch, and fire every block's bucket hook exactly once.

Reference: the head is tied to tok_emb (model_tiny_gpt.py:217-219), so d(tok_emb) = the head's
dlogits^T . ln_f(x) plus the embedding scatter-add (loss.backward(), loop.py:1233).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(seed=7, **opts):
    from codonlm_amd import TinyGPT
    torch.manual_seed(seed)
    m = TinyGPT(68, 128, n_layer=3, n_head=4, n_embd=128, dropout=0.0, label_smoothing=0.05,
                compute_dtype="bf16", device=DEV, engine_opts=opts)
    m.train()
    return m


def _batch(B=4, T=128, seed=3):
    g = torch.Generator().manual_seed(seed)
    t = torch.randint(4, 68, (B, T + 1), generator=g)
    t[:, 40] = 3  # a SEP segment
    return t[:, :-1].to(DEV), t[:, 1:].to(DEV)


def _grads(defer, partial):
    m = _model(head_dw_separate=int(not defer))
    x, y = _batch()
    m.flat_grads().zero_()
    _, loss = m(x, y)
    if partial:
        eng = m.engine
        eng.set_head_grads(1.0)
        eng.backward_phase(0, 0, False)
        eng.backward_phase(2, 0, False)
    else:
        loss.backward()
    torch.cuda.synchronize()
    return {k: v.grad.detach().clone() for k, v in m.named_parameters() if v.grad is not None}


def _rel(a, b):
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _fc1_bias_mask(m):
    """Flat-gradient mask of the fc1 biases (mlp.0.bias).  Their gradient, the column sums of dH,
    comes from the block's grouped dW launch (bf16 dH, the fragments the tiles stream) when that
    launch does not split the tokens, else from the dGELU product's epilogue (fp32 dH before its
    bf16 rounding): plans with different token splits differ there by dH's rounding, so those
    entries are compared at 1e-3 and everything else at the plan-invariance bound."""
    flat = m.flat_parameters()
    mask = torch.zeros(flat.numel(), dtype=torch.bool, device=flat.device)
    for k, v in m.named_parameters():
        if k.endswith("mlp.0.bias"):
            off = v.data_ptr() // 4 - flat.data_ptr() // 4
            mask[off:off + v.numel()] = True
    return mask


def _same_grads(g, ref, mask, bound=1e-6):
    assert _rel(g[~mask], ref[~mask]) < bound, _rel(g[~mask], ref[~mask])
    assert _rel(g[mask], ref[mask]) < 1e-3, _rel(g[mask], ref[mask])


def test_head_dw_defer_on_equals_off():
    on, off = _grads(True, False), _grads(False, False)
    assert on.keys() == off.keys()
    # tok_emb: the same fp32-accumulated product over the same bf16 operands in another
    # summation order (grouped dW tile vs split-K slabs)
    assert _rel(on["tok_emb.weight"], off["tok_emb.weight"]) < 1e-5
    for k in on:
        if k != "tok_emb.weight":
            assert _rel(on[k], off[k]) < 1e-6, k


def test_head_dw_partial_phases_runs_deferred_product():
    """phase 0 then phase 2: with deferral on, no dW group took the head's product, so phase 2
    must run it -- tok_emb.grad equals the non-deferred sequence's."""
    on, off = _grads(True, True), _grads(False, True)
    te_on, te_off = on["tok_emb.weight"], off["tok_emb.weight"]
    assert float(te_off.abs().max()) > 0
    assert _rel(te_on, te_off) < 1e-5


def test_dw_group_orders_give_the_same_gradients():
    from codonlm_amd import TinyGPT
    x, y = _batch()

    def run(order, group):
        torch.manual_seed(5)
        m = TinyGPT(68, 128, n_layer=12, n_head=4, n_embd=128, dropout=0.0, compute_dtype="bf16", device=DEV,
                    engine_opts={"dw_remainder_first": int(order == 0), "dw_group": group})
        m.train()
        fired = []
        m._bucket_hook = fired.append
        _, loss = m(x, y)
        loss.backward()
        torch.cuda.synchronize()
        return m.flat_grads().detach().clone(), fired, _fc1_bias_mask(m)

    ref, fired_ref, mask = run(0, 1)
    assert sorted(map(str, fired_ref)) == sorted(map(str, ["head", "embed", *range(12)]))
    assert int(mask.sum()) == 12 * 512
    for order, group in ((0, 5), (1, 5), (0, 4), (1, 6), (1, 12)):
        g, fired, _ = run(order, group)
        assert sorted(map(str, fired)) == sorted(map(str, fired_ref)), (order, group, fired)
        _same_grads(g, ref, mask)


@pytest.mark.parametrize("hd,dropout", [(48, 0.0), (64, 0.1), (32, 0.1)])
def test_rope_fused_equals_table_passes(hd, dropout):
    """RoPE models (model_tiny_gpt.py:91-93): the rotation fused into the qkv projection's GEMM
    epilogue and the attention backward's dQ / dK stores (the default) against the separate
    cg_rope_tab passes (engine_opts rope_tables=1).  The fused forward rounds q / k to bf16 once
    instead of twice, so loss within 2e-3 relative and every gradient within rel-L2 3e-2 (the
    bf16 step's own noise between two roundings of the same values)."""
    from codonlm_amd import TinyGPT

    def run(fused):
        torch.manual_seed(11)
        m = TinyGPT(68, 256, n_layer=2, n_head=4, n_kv_head=2, n_embd=4 * hd, dropout=dropout,
                    label_smoothing=0.05, use_rope=True, use_swiglu=True, compute_dtype="bf16", device=DEV,
                    engine_opts={"rope_tables": int(not fused)})
        m.train()
        x, y = _batch(B=4, T=256, seed=5)
        m.flat_grads().zero_()
        _, loss = m(x, y)
        loss.backward()
        torch.cuda.synchronize()
        return float(loss), {k: v.grad.detach().clone() for k, v in m.named_parameters() if v.grad is not None}
    lf, gf = run(True)
    lu, gu = run(False)
    assert abs(lf - lu) <= 2e-3 * abs(lu), (lf, lu)
    assert gf.keys() == gu.keys()
    for k in gf:
        assert _rel(gf[k], gu[k]) < 3e-2, (k, _rel(gf[k], gu[k]))


def test_dw_ksplit_gives_the_same_gradients():
    """C2 geometry (d256, H4, T512 -- the planner splits its one 6-block group 3 ways): every
    block's dW with the token range cut into 1, 2 or 3 slices (slices summed in order into the
    fp32 gradient) -- the same products in another summation order."""
    import ctypes as C

    from codonlm_amd import TinyGPT, _lib as L
    x, y = _batch(B=8, T=512, seed=9)

    def run(ks):
        torch.manual_seed(13)
        m = TinyGPT(68, 512, n_layer=6, n_head=4, n_embd=256, dropout=0.1, label_smoothing=0.05,
                    compute_dtype="bf16", device=DEV, engine_opts={"dw_ksplit": ks})
        m.train()
        m.flat_grads().zero_()
        _, loss = m(x, y)
        loss.backward()
        torch.cuda.synchronize()
        return m.flat_grads().detach().clone(), m

    # the plan depends on the step's token count: at the C2 bench's B = 64 the one 6-block group is
    # split 3 ways over the tokens, at this test's B = 8 it is not -- unless the model is told to
    # plan as for the bench's token count (dw_plan_tokens)
    _, m0 = run(0)
    cfg = m0.engine.model.cfg
    G, tm, ks = C.c_int(0), C.c_int(0), C.c_int(0)

    def plan(B):
        L.check(L.lib.cg_model_dw_plan(C.byref(cfg), B, 512, C.byref(G), C.byref(tm), C.byref(ks)), "cg_model_dw_plan")
        return G.value, ks.value
    assert plan(64) == (6, 3) and plan(8) == (6, 1), (plan(64), plan(8))
    cfg.opts.dw_plan_tokens = 64 * 512
    assert plan(8) == (6, 3)
    cfg.opts.dw_plan_tokens = 0
    cfg.opts.dw_ksplit = 4  # out of range: an error, not a silent default
    assert L.lib.cg_model_dw_plan(C.byref(cfg), 8, 512, C.byref(G), C.byref(tm), C.byref(ks)) == L.CG_EINVAL
    cfg.opts.dw_ksplit = 0
    ref, m1 = run(1)
    mask = _fc1_bias_mask(m1)
    assert float(ref.abs().max()) > 0
    for ks in (0, 2, 3):
        g = run(ks)[0]
        _same_grads(g, ref, mask)
        assert torch.equal(g, run(ks)[0]), ks  # deterministic: slabs reduced in slice order


def test_attention_keep_word_sources_give_the_same_step():
    """The attention-dropout keep words of a training step made by the attention forward itself
    (default), by the separate mask kernel (engine option attn_mask_kernel=1) or in the launch of the
    block's LN1 (attn_mask_kernel=2, cg_layernorm_fwd_mask): the same words, so the same loss and
    the same gradients, bit for bit (model_tiny_gpt.py:104-114 dropout on the attention
    probabilities, one mask per step and block)."""
    from codonlm_amd import TinyGPT
    x, y = _batch(B=4, T=256, seed=21)

    def run(mode):
        torch.manual_seed(17)
        m = TinyGPT(68, 256, n_layer=3, n_head=4, n_embd=256, dropout=0.1, label_smoothing=0.05,
                    compute_dtype="bf16", device=DEV, engine_opts={"attn_mask_kernel": mode})
        m.train()
        m.flat_grads().zero_()
        _, loss = m(x, y)
        loss.backward()
        torch.cuda.synchronize()
        return float(loss), m.flat_grads().detach().clone()

    l0, g0 = run(0)
    for mode in (1, 2):
        lm, gm = run(mode)
        assert lm == l0, (mode, lm, l0)
        assert torch.equal(gm, g0), mode


def test_persistent_grid_cap_gives_the_same_step():
    """cg_model_opts.pers_max_wg (the grid cap a data-parallel run could use to leave CUs to RCCL,
    priced in profiles/round6/dp_reserve_replay.txt) only changes which workgroup walks which tile:
    every tile is reduced in the same order, so the loss and every gradient are bitwise those of
    the uncapped grid (forward / dX persistent GEMMs and the grouped dW launches)."""
    from codonlm_amd import TinyGPT, _lib as L
    x, y = _batch(B=4, T=256, seed=23)
    cus = int(L.lib.cg_pers_cus())

    def run(cap):
        torch.manual_seed(19)
        m = TinyGPT(68, 256, n_layer=3, n_head=4, n_embd=256, dropout=0.1, label_smoothing=0.05,
                    compute_dtype="bf16", device=DEV, engine_opts={"pers_max_wg": cap})
        m.train()
        m.flat_grads().zero_()
        _, loss = m(x, y)
        loss.backward()
        torch.cuda.synchronize()
        return float(loss), m.flat_grads().detach().clone()

    l0, g0 = run(0)
    for cap in (cus - 16, 37):
        lc, gc = run(cap)
        assert lc == l0, (cap, lc, l0)
        assert torch.equal(gc, g0), cap
