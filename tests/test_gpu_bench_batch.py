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
