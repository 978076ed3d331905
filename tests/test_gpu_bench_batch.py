"""C4 at the bench line's own geometry: B=32 sequences x T=1024 per GPU (bench.py CONFIGS["c4"]).

test_gpu_configs.py pins every config at B=2 with the dW plan of the bench token count; this
module runs the bench's real batch, so every kernel sees the bench's M = 32768 rows, grid sizes,
persistent-tile walks, dW group plan and token-range split:

  * the bf16 engine step (fwd + CE + bwd) against the fp32 oracle at B=32 (same bounds as the
    B=2 tests: logits rel-L2 <= 5e-3, every parameter gradient rel-L2 <= 1.5e-2, greedy ids
    wherever the oracle's top-2 margin is resolvable) -- the oracle's autograd at this size takes
    about a minute on 8-16 host threads and ~40 GB of host memory;
  * batch invariance of the forward: rows 0-1 and 30-31 of the B=32 logits against B=2 runs of
    the same rows (each sequence's logits depend only on its own tokens; bf16 products of other
    M-tilings may round differently, so the bound is bf16-level, and the max |difference| is
    printed).

B=32 is the reference's 32 sequences per optimizer step of its 12L8H d512 run (batch_size 2 x
grad_accum_steps 16, runs/2025-11-05_tiny_12L8H_d512_e5/log.txt:30-31).
"""
import ctypes as C

import pytest
import torch

from oracle import tinygpt_oracle as O
from test_gpu_configs import LOGIT_REL_L2_BF16, _cfg, _check_bf16, _model, _rel_l2, packed_batch

pytestmark = pytest.mark.gpu
DEV = "cuda"
B_BENCH = 32


@pytest.fixture(scope="module")
def c4_bench():
    cfg, _ = _cfg("C4")
    params = O.synthetic_params(cfg, seed=13)
    x, y = packed_batch(B_BENCH, cfg.block_size, seed=5)
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    o, grads = O.forward_backward(cfg, params, x, y)
    return cfg, params, x, y, (o["logits"].detach(), float(o["loss"]), grads)


def test_c4_bench_batch_matches_oracle(c4_bench):
    from codonlm_amd import _lib as L
    cfg, params, x, y, (rlogits, rloss, rgrads) = c4_bench
    m = _model(cfg, params, "bf16")  # (no dw_plan_tokens: the plan of the real token count, as in bench.py)
    G, tm, ks = C.c_int(0), C.c_int(0), C.c_int(0)
    L.check(L.lib.cg_model_dw_plan(C.byref(m.engine.model.cfg), B_BENCH, cfg.block_size, C.byref(G), C.byref(tm),
                                   C.byref(ks)), "cg_model_dw_plan")
    print(f"[C4 B={B_BENCH}] dW plan: groups of {G.value} blocks, tile_m {tm.value}, token split {ks.value}")
    xd, yd = torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)
    logits, loss = m(xd, yd)
    loss.backward()
    torch.cuda.synchronize()
    _check_bf16(m, cfg, f"C4-B{B_BENCH}", logits, loss, loss, rlogits, rloss, rloss, rgrads)


def test_c4_bench_batch_rows_match_small_batch(c4_bench):
    cfg, params, x, y, _ = c4_bench
    m = _model(cfg, params, "bf16")
    m.eval()
    with torch.no_grad():
        full, _ = m(torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV))
        full = full.float().cpu()
        for r in (0, 30):
            part, _ = m(torch.from_numpy(x[r:r + 2]).to(DEV), torch.from_numpy(y[r:r + 2]).to(DEV))
            part = part.float().cpu()
            d = float((part - full[r:r + 2]).abs().max())
            e = _rel_l2(part, full[r:r + 2])
            print(f"[C4 rows {r}-{r + 1}] B=2 vs B={B_BENCH}: max |dlogit| {d:.3e}, rel-L2 {e:.2e}")
            assert e <= LOGIT_REL_L2_BF16 / 5, (r, e)


# the other configs' bench batches (bench.py CONFIGS): the reference's sequences per optimizer step
def _bench_batch(name):
    from bench import CONFIGS as BC
    return BC[name.lower()]["batch"]


@pytest.mark.parametrize("name", ["C2", "C3", "C5"])
def test_bench_batch_consistency(name):
    """C2 / C3 / C5 at their bench batch (the B=2 oracle parity of test_gpu_configs plans the dW
    groups for the same token count; here the kernels run the full geometry): the bf16 step's
    logits rows equal B=2 runs of the same rows (bf16-level), and its parameter gradients equal the
    loss-weight-weighted sum of four quarter-batch steps (each with its own, different dW plan) --
    the LM loss is a weighted mean over valid targets, so grad(B) = sum_i (W_i / W) grad(B_i)."""
    cfg, _ = _cfg(name)
    params = O.synthetic_params(cfg, seed=17 + len(name))
    B, T = _bench_batch(name), cfg.block_size
    x, y = packed_batch(B, T, seed=9)
    m = _model(cfg, params, "bf16")
    xd, yd = torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)
    w = torch.tensor(cfg.loss_weights if cfg.loss_weights else [1.0] * cfg.vocab_size, dtype=torch.float64)

    def wsum(yy):
        yy = torch.from_numpy(yy)
        return float(torch.where(yy != 0, w[yy], torch.zeros(()).double()).sum())

    m.zero_grad(set_to_none=True)
    logits, loss = m(xd, yd)
    loss.backward()
    torch.cuda.synchronize()
    full = {k: p.grad.detach().double().cpu().clone() for k, p in m.named_parameters() if p.grad is not None}
    lg = logits.detach().float().cpu().reshape(B, T, -1)
    acc = {k: torch.zeros_like(v) for k, v in full.items()}
    W = wsum(y)
    q = B // 4
    for i in range(4):
        sl = slice(i * q, (i + 1) * q)
        m.zero_grad(set_to_none=True)
        li, lossi = m(xd[sl].contiguous(), yd[sl].contiguous())
        lossi.backward()
        torch.cuda.synchronize()
        if i in (0, 3):
            part = li.detach().float().cpu().reshape(q, T, -1)
            e = _rel_l2(part, lg[sl])
            print(f"[{name} B={B}] logits rows {sl.start}-{sl.stop - 1} vs quarter run: rel-L2 {e:.2e}")
            assert e <= LOGIT_REL_L2_BF16 / 5, (name, i, e)
        wi = wsum(y[sl]) / W
        for k, p in m.named_parameters():
            if k in acc and p.grad is not None:
                acc[k] += wi * p.grad.detach().double().cpu()
    # (without RoPE the key biases' gradients are zero in exact arithmetic -- softmax shift
    # invariance -- so both sides are rounding noise and are left out, as in _check_bf16)
    worst = sorted(((_rel_l2(acc[k], v), k) for k, v in full.items()
                    if float(v.norm()) > 0 and not (k.endswith("attn.key.bias") and not cfg.use_rope)), reverse=True)
    print(f"[{name} B={B}] gradient vs weighted quarter sum: worst {[(k, f'{e:.2e}') for e, k in worst[:3]]}")
    assert worst[0][0] <= 1e-2, (name, worst[:3])
