"""Aux heads + objectives on the MI355X path vs the reference.

Golden vectors: tests/golden/aux_heads.npz (forward of the termination / multi-offset
heads), aux_objective.npz (the trainer's full objective loop.py:1075-1112 and every
parameter grad), objectives.npz (objectives.py label construction and losses).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import tinygpt_oracle as O
from test_gpu_model import DEV, make_model, _idx
from test_oracle_golden import aux_objective_args

pytestmark = pytest.mark.gpu


def _objective(m, x, y, cfg, args, return_parts=False):
    from codonlm_amd.training import objectives as obj
    logits, loss, aux = m(x, y, return_aux=True)
    lw = m.loss_weights if not torch.all(m.loss_weights == 1.0).item() else None
    off_total, off_losses = obj.multi_offset_lm_loss(aux["offset_logits"], y, args["offset_weights"],
                                                     label_smoothing=cfg.label_smoothing, loss_weights=lw)
    labels = obj.termination_distance_bucket_labels(y, stop_ids=args["stop_ids"], bucket_edges=args["bucket_edges"])
    cw = torch.tensor(args["term_class_weights"], device=DEV)
    term = obj.termination_aux_loss(aux["termination_logits"], labels, class_weights=cw)
    total = loss + off_total + args["term_weight"] * term
    parts = {"loss": loss, "total": total, "term_loss": term, "term_labels": labels,
             **{f"offset_loss_{k}": v for k, v in off_losses.items()}}
    return (total, parts, aux) if return_parts else total


@pytest.mark.parametrize("case", ["aux_heads", "aux_objective"])
def test_aux_forward_matches_reference(case):
    cfgd, g = load_golden(case)
    if "param_seed" not in g:
        g = dict(g, param_seed=np.array(0))
    m, cfg, _ = make_model(cfgd, g)
    m.eval()
    x, y = _idx(g)
    with torch.no_grad():
        logits, loss, aux = m(x, y, return_aux=True)
    tl = aux["termination_logits"].cpu().numpy()
    assert tl.shape == g["termination_logits"].shape
    np.testing.assert_allclose(tl, g["termination_logits"], rtol=1e-4, atol=1e-4)
    for k in cfg.multi_offset_targets:
        ref = g[f"offset_logits_{k}"]
        got = aux["offset_logits"][k].cpu().numpy()
        scale = max(1.0, float(np.abs(ref).max()))
        assert np.abs(got - ref).max() <= 1e-4 * scale, k
    assert abs(loss.item() - float(g["loss"])) <= 1e-4 * max(1.0, abs(float(g["loss"])))


def test_aux_objective_grads_match_reference():
    cfgd, g = load_golden("aux_objective")
    m, cfg, _ = make_model(cfgd, dict(g, param_seed=np.array(0)))
    m.train()
    x, y = _idx(g)
    total, parts, _ = _objective(m, x, y, cfg, aux_objective_args(g), return_parts=True)
    total.backward()
    assert np.array_equal(parts["term_labels"].cpu().numpy(), g["term_labels"])
    for key in ("loss", "total", "term_loss", "offset_loss_2", "offset_loss_4"):
        assert abs(parts[key].item() - float(g[key])) <= 1e-4 * max(1.0, abs(float(g[key]))), key
    for k, p in m.named_parameters():
        ref = g[f"grad/{k}"]
        got = p.grad.detach().cpu().numpy()
        s = max(1e-3, float(np.abs(ref).max()))
        err = float(np.abs(got - ref).max())
        assert err <= 2e-4 * s, (k, err, s)


def test_aux_objective_bf16_close_and_trains():
    from codonlm_amd.optim import FusedAdamW
    cfgd, g = load_golden("aux_objective")
    gg = dict(g, param_seed=np.array(0))
    m, cfg, _ = make_model(cfgd, gg, dtype="bf16")
    m32, _, _ = make_model(cfgd, gg)
    m.train()
    m32.train()
    x, y = _idx(g)
    args = aux_objective_args(g)
    t16 = _objective(m, x, y, cfg, args)
    t16.backward()
    t32 = _objective(m32, x, y, cfg, args)
    t32.backward()
    assert abs(t16.item() - t32.item()) <= 2e-2 * abs(t32.item())
    for (k, p), (_, q) in zip(m.named_parameters(), m32.named_parameters()):
        a, b = p.grad.detach().float().flatten(), q.grad.detach().float().flatten()
        if float(b.norm()) < 1e-6:
            continue
        cos = float(torch.nn.functional.cosine_similarity(a, b, dim=0))
        assert cos > 0.98, (k, cos)
    opt = FusedAdamW(m, lr=1e-3, weight_decay=0.0)
    first = None
    for _ in range(12):
        opt.zero_grad()
        t = _objective(m, x, y, cfg, args)
        t.backward()
        opt.step()
        first = first if first is not None else t.item()
    assert t.item() < first


def test_objective_labels_and_losses_match_reference():
    from codonlm_amd.training import objectives as obj
    _, g = load_golden("objectives")
    y = torch.from_numpy(g["y"]).to(DEV)
    for k in (2, 3, 4, 8):
        assert np.array_equal(obj.offset_target_mask(y, k).cpu().numpy(), g[f"offset_mask_{k}"]), k
    stop = tuple(int(s) for s in g["stop_ids"])
    lab = obj.termination_distance_bucket_labels(y, stop_ids=stop)
    assert np.array_equal(lab.cpu().numpy(), g["term_labels"])
    logits = torch.from_numpy(g["mo_logits"]).to(DEV)
    tot, losses = obj.multi_offset_lm_loss(logits, y, {2: 0.5, 4: 0.25}, label_smoothing=0.05)
    assert abs(tot.item() - float(g["mo_total"])) < 1e-5
    for k, v in losses.items():
        assert abs(v.item() - float(g[f"mo_loss_{k}"])) < 1e-5
    tl = torch.from_numpy(g["term_logits"]).to(DEV)
    cw = torch.from_numpy(g["term_cw"]).to(DEV)
    term = obj.termination_aux_loss(tl, lab, class_weights=cw)
    assert abs(term.item() - float(g["term_loss"])) < 1e-5
    # edge cases the reference handles: offset beyond T, empty input, errors
    assert obj.offset_target_mask(y, y.shape[1] + 1).shape == (y.shape[0], 0)
    with pytest.raises(ValueError):
        obj.offset_target_mask(y, 0)
    with pytest.raises(ValueError):
        obj.termination_distance_bucket_labels(y, stop_ids=())
    with pytest.raises(ValueError):
        obj.termination_distance_bucket_labels(y, stop_ids=(2,), bucket_edges=(3, 0))
    # all-invalid offsets are skipped like the reference (no NaN)
    pad = torch.zeros(2, 8, dtype=torch.long, device=DEV)
    tot0, l0 = obj.multi_offset_lm_loss(torch.zeros(2, 8, 68, device=DEV), pad, {2: 1.0})
    assert l0 == {} and tot0.item() == 0.0


def test_objective_labels_random_vs_oracle():
    """Integer label kernels bit-exact vs the oracle on random SEP/EOS/PAD-laden inputs."""
    from codonlm_amd.training import objectives as obj
    rng = np.random.default_rng(3)
    for B, T in ((3, 17), (4, 256), (2, 1024)):
        y = rng.integers(0, 69, size=(B, T)).astype(np.int64)
        y[rng.random((B, T)) < 0.05] = 2
        y[rng.random((B, T)) < 0.05] = 3
        yt = torch.from_numpy(y)
        yd = yt.to(DEV)
        for k in (2, 5, 16, 32):
            assert np.array_equal(obj.offset_target_mask(yd, k).cpu().numpy(), O.offset_target_mask(yt, k).numpy())
        for stop, edges in (((2,), (0, 3, 10, 30)), ((2, 52, 54, 60), (0, 1, 2, 5, 8, 100))):
            lab = obj.termination_distance_bucket_labels(yd, stop_ids=stop, bucket_edges=edges).cpu().numpy()
            assert np.array_equal(lab, O.termination_labels(y, stop, edges))


def test_scaled_loss_and_aux_only_backward():
    """Autograd through the engine: d(c * loss) = c * d(loss); a termination-only objective with
    no targets (the replay-batch shape, loop.py:1133) matches the oracle's autograd."""
    from codonlm_amd.training import objectives as obj
    cfgd, g = load_golden("aux_objective")
    gg = dict(g, param_seed=np.array(0))
    m, cfg, params = make_model(cfgd, gg)
    m.train()
    x, y = _idx(g)
    _, loss = m(x, y)
    loss.backward()
    ref = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
    m.zero_grad()
    _, loss = m(x, y)
    (2.5 * loss).backward()
    # the scale d(2.5 loss)/d(loss) is applied on the device to the head gradient before the
    # backward products: equal up to fp32 rounding of the scaled operands
    for k, p in m.named_parameters():
        # (key biases' exact gradient is 0 -- softmax shift invariance -- so they hold rounding
        # noise only: compared at the query bias' scale)
        sk = k.replace("key.bias", "query.bias") if k.endswith("attn.key.bias") else k
        atol = 2e-6 * float(ref[sk].abs().max()) + 1e-12
        torch.testing.assert_close(p.grad, 2.5 * ref[k], rtol=1e-5, atol=atol, msg=k)
    # aux-only objective (no targets): termination loss alone
    m.zero_grad()
    _, none_loss, aux = m(x, return_aux=True)
    assert none_loss is None
    lab = obj.termination_distance_bucket_labels(y, stop_ids=(2,))
    term = obj.termination_aux_loss(aux["termination_logits"], lab)
    term.backward()
    P = O._to_t(params, True)
    o = O.forward(cfg, P, g["idx"])
    tl = O.termination_loss(o["aux"]["termination_logits"], O.termination_labels(g["targets"], (2,)))
    tl.backward()
    assert abs(term.item() - float(tl)) <= 1e-5 * max(1.0, abs(float(tl)))
    for k, p in m.named_parameters():
        r = P[k].grad if P[k].grad is not None else torch.zeros_like(P[k])
        s = max(1e-3, float(r.abs().max()))
        err = float((p.grad.detach().cpu() - r).abs().max())
        assert err <= 2e-4 * s, (k, err, s)


def test_adamw_fast_group_matches_oracle():
    """The reference's two AdamW groups (loop.py:685-718): offset_projs / termination_head in the
    fast group (lr_embedding, weight_decay 0), everything else -- embeddings, LN, biases -- in the
    backbone group (lr, weight_decay).  FusedAdamW runs both as ranges of the flat buffer (the
    fast params form its tail); two steps against the oracle's per-tensor AdamW fed the same
    gradients."""
    from codonlm_amd.optim import FusedAdamW
    cfgd, g = load_golden("aux_objective")
    gg = dict(g, param_seed=np.array(0))
    m, cfg, params = make_model(cfgd, gg)
    m.train()
    x, y = _idx(g)
    args = aux_objective_args(g)
    lr, lr_emb, wd = 2e-3, 7e-3, 0.05
    opt = FusedAdamW(m, lr=lr, weight_decay=wd, lr_embedding=lr_emb)
    fast_names = {k for k, _ in m.named_parameters() if k.startswith(("offset_projs", "termination_head"))}
    assert fast_names and len(opt.param_groups) == 2
    P = {k: p.detach().cpu().clone() for k, p in m.named_parameters()}
    mo = {k: torch.zeros_like(v) for k, v in P.items()}
    vo = {k: torch.zeros_like(v) for k, v in P.items()}
    for step in (1, 2):
        opt.zero_grad()
        _objective(m, x, y, cfg, args).backward()
        grads = {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters()}
        opt.step()
        for k in P:
            fast = k in fast_names
            O.adamw_step(P[k], grads[k], mo[k], vo[k], step, lr_emb if fast else lr, 0.0 if fast else wd)
    for k, p in m.named_parameters():
        atol = 2.5 * lr if k.endswith("attn.key.bias") else 2e-6
        np.testing.assert_allclose(p.detach().cpu().numpy(), P[k].numpy(), rtol=1e-5, atol=atol, err_msg=k)
