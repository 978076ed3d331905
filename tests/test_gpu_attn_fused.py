"""The fused bf16 attention backward (cg_attn_bwd_algo(CG_ATTN_BWD_FUSED, ...),
attention_mfma.h attn_bwd_fused_mfma): one pass per (batch, kv head) that computes S, dP, dV, dK
and dQ for every key block, dQ summed over the key blocks in an fp32 accumulator only that
workgroup writes.  It replaces the autograd of the reference attention
(/root/reference/src/codonlm/model_tiny_gpt.py:102-131) like the split two-kernel pass does, so
it is held to the same bounds against fp32 autograd of the same bf16-rounded inputs (rel-L2 <= 2e-2
per q / k / v block), to the split pass (rel <= 1e-2 for dQ / dK, whose delta rows are summed in
another order; dV bitwise, same products in the same order), and to itself (bitwise reproducible:
no atomics).  Geometries: the benchmarked C4 (T1024 hd64, dropout 0.1), C3 (T512 hd48 GQA-4 RoPE),
C5 (hd48 MHA), ragged T (not a multiple of the 64-query tile or the 256-key block), local windows
across key blocks, SEP segments, T < 64.
"""
import numpy as np
import pytest
import torch

from oracle import tinygpt_oracle as O
from tests.test_gpu_ops import _attn_ref, _bf, _rope_ref, _rope_tabs

pytestmark = pytest.mark.gpu

DEV = "cuda"

CASES = [
    # B, T, H, KV, hd, window, p, rope
    (2, 1024, 8, 8, 64, 0, 0.1, False),
    (2, 512, 8, 4, 48, 0, 0.0, True),
    (2, 512, 8, 4, 48, 0, 0.1, True),
    (2, 512, 8, 8, 48, 0, 0.1, False),
    (2, 300, 4, 2, 64, 0, 0.1, False),
    (3, 700, 4, 4, 64, 100, 0.1, False),
    (1, 130, 2, 1, 32, 17, 0.0, False),
    (2, 40, 4, 2, 48, 0, 0.0, True),
    (2, 5, 2, 1, 64, 0, 0.1, False),
]


def _rel(a, b):
    return float((a.double() - b.double()).norm() / max(b.double().norm(), 1e-30))


@pytest.mark.parametrize("B,T,H,KV,hd,window,p,rope", CASES)
def test_attention_bwd_fused(B, T, H, KV, hd, window, p, rope):
    from codonlm_amd import ops
    g = torch.Generator().manual_seed(T * 7 + hd + H)
    N = (H + 2 * KV) * hd
    proj = _bf(torch.randn(B * T, N, generator=g))
    idx = torch.randint(4, 68, (B, T), generator=g)
    for pos in (T // 5, T // 2):
        idx[0, pos] = 3
    idx[B - 1, T // 3] = 3
    seed = 1234 + T
    pr = proj.clone().requires_grad_(True)
    if rope:
        cos, sin = _rope_tabs(T, hd)
        q = _rope_ref(pr[:, :H * hd], cos, sin, H, hd)
        k = _rope_ref(pr[:, H * hd:(H + KV) * hd], cos, sin, KV, hd)
        src = torch.cat([q, k, pr[:, (H + KV) * hd:]], 1)
    else:
        src = pr
    drop = None
    if p > 0:
        keep = O.dropout_keep(seed, np.arange(B * H * T)[:, None], np.arange(T)[None, :], p)
        drop = torch.from_numpy(keep.astype(np.float32) / (1 - p)).view(B, H, T, T)
    ref = _attn_ref(src, idx, B, T, H, KV, hd, 3, window or None, drop)
    dy = _bf(torch.randn(B * T, H * hd, generator=g))
    ref.backward(dy)
    seg = ops.segment_starts(idx.to(DEV), 3)
    qkv = proj.to(DEV, torch.bfloat16)
    tabs = None
    if rope:
        tabs = (cos.to(DEV), sin.to(DEV))
        ops.rope_(qkv, B, T, H, KV, hd, *tabs)
    if p > 0:
        y, lse, mask = ops.attn_fwd_keep(qkv, seg, B, T, H, KV, hd, seed, p, window=window)
    else:
        y, lse = ops.attn_fwd(qkv, seg, B, T, H, KV, hd, window=window)
        mask = None
    dyd = dy.to(DEV, torch.bfloat16)
    nrb = B * ((T + 127) // 128)
    res = {}
    for algo in ("fused", "split", "fused2"):
        part = torch.full((nrb, N + 8), float("nan"), device=DEV)
        d = ops.attn_bwd(qkv, seg, y, dyd, lse, B, T, H, KV, hd, window=window, drop_seed=seed, drop_p=p,
                         drop_mask=mask, bias_part=part, rope=tabs, algo=algo.rstrip("2"))
        res[algo] = (d.float().cpu(), part[:, :N].cpu())
    fz, fpart = res["fused"]
    sp, _ = res["split"]
    blocks = (("dq", slice(0, H * hd)), ("dk", slice(H * hd, (H + KV) * hd)), ("dv", slice((H + KV) * hd, N)))
    for name, sl in blocks:
        e_ref = _rel(fz[:, sl], pr.grad[:, sl])
        e_split = _rel(fz[:, sl], sp[:, sl])
        print(f"{name}: rel vs autograd {e_ref:.3e}  vs split {e_split:.3e}")
        assert e_ref <= 2e-2, (name, e_ref)
        assert e_split <= 1e-2, (name, e_split)
    assert torch.equal(fz[:, (H + KV) * hd:], sp[:, (H + KV) * hd:])  # dV: the same products, same order
    # bitwise reproducible (no atomics), bias partials included
    assert torch.equal(res["fused2"][0], fz)
    assert torch.equal(res["fused2"][1], fpart)
    # bias partials: every row written, reducing to the column sums of the returned dqkv
    assert torch.isfinite(fpart).all()
    colsum = fz.sum(0)
    assert float((fpart.sum(0) - colsum).abs().max() / colsum.abs().max()) <= 2e-3


def test_attention_bwd_algo_errors():
    """A forced fused pass that cannot run is CG_EUNSUPPORTED (ValueError), never a silent fallback:
    dropout without keep words, and the fp32 dtype; an unknown algo is CG_EINVAL."""
    from codonlm_amd import ops
    B, T, H, KV, hd = 1, 64, 2, 2, 64
    qkv = torch.randn(B * T, (H + 2 * KV) * hd, device=DEV).to(torch.bfloat16)
    y, lse = ops.attn_fwd(qkv, None, B, T, H, KV, hd)
    dy = torch.randn(B * T, H * hd, device=DEV).to(torch.bfloat16)
    with pytest.raises(ValueError):
        ops.attn_bwd(qkv, None, y, dy, lse, B, T, H, KV, hd, drop_seed=1, drop_p=0.1, algo="fused")
    q32 = qkv.float()
    y32, lse32 = ops.attn_fwd(q32, None, B, T, H, KV, hd)
    with pytest.raises(ValueError):
        ops.attn_bwd(q32, None, y32, dy.float(), lse32, B, T, H, KV, hd, algo="fused")
    ops.ATTN_BWD_ALGO["bogus"] = 7
    try:
        with pytest.raises(ValueError):
            ops.attn_bwd(qkv, None, y, dy, lse, B, T, H, KV, hd, algo="bogus")
    finally:
        del ops.ATTN_BWD_ALGO["bogus"]
