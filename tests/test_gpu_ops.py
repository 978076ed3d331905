"""Op-level parity of the HIP kernels against plain PyTorch fp32 (CPU) references.

Every test here needs the MI355X (marker ``gpu``) and calls through the C-ABI
(libcodonlm_hip.so) via codonlm_amd.ops.
"""
import functools
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import tinygpt_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ops():
    from codonlm_amd import ops
    return ops


def _bf(x):
    return x.to(torch.bfloat16).float()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ak,bk", [(1, 1), (1, 0), (0, 0), (0, 1)])
@pytest.mark.parametrize("M,N,K", [(128, 64, 64), (200, 136, 72), (1024, 512, 384), (96, 80, 1000)])
def test_gemm_layouts(dtype, ak, bk, M, N, K):
    ops = _ops()
    g = torch.Generator().manual_seed(M * 7 + N + K)
    Am = torch.randn(M, K, generator=g)
    Bn = torch.randn(N, K, generator=g)
    a = (Am if ak else Am.t().contiguous()).to(DEV, dtype)
    b = (Bn if bk else Bn.t().contiguous()).to(DEV, dtype)
    out = ops.gemm(a, b, a_kcontig=bool(ak), b_kcontig=bool(bk), M=M, N=N, K=K, out_dtype=torch.float32)
    # exact product of the (bf16-rounded) operands; the only error left is the fp32 accumulation,
    # bounded elementwise by a few ulps of sum_k |a_mk b_nk| (K <= 1000 here)
    Ar, Br = (_bf(Am), _bf(Bn)) if dtype == torch.bfloat16 else (Am, Bn)
    ref = Ar.double() @ Br.double().t()
    bound = 2e-5 * (Ar.double().abs() @ Br.double().abs().t()) + 1e-30
    err = ((out.cpu().double() - ref).abs() / bound).max().item()
    assert err <= 1.0, err


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogues(dtype):
    ops = _ops()
    L = __import__("codonlm_amd._lib", fromlist=["x"])
    M, N, K = 256, 192, 128
    g = torch.Generator().manual_seed(3)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) * 0.1
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    xd, wd = x.to(DEV, dtype), w.to(DEV, dtype)
    base = (_bf(x) @ _bf(w).t()) if dtype == torch.bfloat16 else x @ w.t()
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-4
    # bias + gelu with pre-activation saved
    aux = torch.empty(M, N, dtype=dtype, device=DEV)
    y = ops.gemm(xd, wd, out_dtype=dtype, bias=bias.to(DEV), epilogue=L.EPI_BIAS | L.EPI_GELU, aux_out=aux)
    pre = base + bias
    assert (aux.float().cpu() - pre).abs().max() < tol * 4
    assert (y.float().cpu() - F.gelu(pre)).abs().max() < tol * 4
    # dgelu
    y2 = ops.gemm(xd, wd, out_dtype=dtype, epilogue=L.EPI_DGELU, aux=aux)
    xa = aux.float().cpu().requires_grad_(True)
    F.gelu(xa).sum().backward()
    ref2 = base * xa.grad
    assert (y2.float().cpu() - ref2).abs().max() < tol * 4
    # bias + dropout + residual (fp32 out)
    p = 0.25
    seed = 12345
    y3 = ops.gemm(xd, wd, out_dtype=torch.float32, bias=bias.to(DEV), resid=res.to(DEV),
                  epilogue=L.EPI_BIAS | L.EPI_DROPOUT | L.EPI_RESID, drop_seed=seed, drop_p=p)
    keep = torch.from_numpy(O.dropout_keep(seed, np.arange(M)[:, None], np.arange(N)[None, :], p))
    ref3 = res + torch.where(keep, (base + bias) / (1 - p), torch.zeros(()))
    assert (y3.cpu() - ref3).abs().max() < tol * 4
    # accumulate + split-K
    acc0 = torch.randn(M, N, generator=g)
    out = acc0.clone().to(DEV)
    ops.gemm(xd, wd, out=out, epilogue=L.EPI_ACCUM, split_k=3, alpha=0.5)
    assert (out.cpu() - (acc0 + 0.5 * base)).abs().max() < tol * 4


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cols", [64, 384, 512, 100])
def test_layernorm_fwd_bwd(out_dtype, cols):
    ops = _ops()
    rows = 300
    g = torch.Generator().manual_seed(cols)
    x = torch.randn(rows, cols, generator=g) * 3 + 1
    w = 1 + 0.1 * torch.randn(cols, generator=g)
    b = 0.1 * torch.randn(cols, generator=g)
    y, mean, rstd = ops.layernorm_fwd(x.to(DEV), w.to(DEV), b.to(DEV), out_dtype=out_dtype)
    xr = x.clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    ref = F.layer_norm(xr, (cols,), wr, br, 1e-5)
    tol = 2e-2 if out_dtype == torch.bfloat16 else 1e-5
    assert (y.float().cpu() - ref.detach()).abs().max() < tol * 4
    dy = torch.randn(rows, cols, generator=g)
    gin = torch.randn(rows, cols, generator=g)
    ref.backward(dy)
    go, dgam, dbet = ops.layernorm_bwd(dy.to(DEV), x.to(DEV), mean, rstd, w.to(DEV), g_in=gin.to(DEV))
    assert (go.cpu() - (xr.grad + gin)).abs().max() < 1e-4
    assert (dgam.cpu() - wr.grad).abs().max() < 1e-3
    assert (dbet.cpu() - br.grad).abs().max() < 1e-3
    # consumer-branch copy (dropout-masked, out_dtype) + its fused column sum (= bias grad)
    p, seed = 0.2, 777
    go2, dgam2, dbet2, br_t, csum = ops.layernorm_bwd(dy.to(DEV), x.to(DEV), mean, rstd, w.to(DEV),
                                                      g_in=gin.to(DEV), branch_dtype=out_dtype,
                                                      drop_seed=seed, drop_p=p)
    exp = xr.grad + gin
    keep = torch.from_numpy(O.dropout_keep(seed, np.arange(rows)[:, None], np.arange(cols)[None, :], p))
    exp_t = torch.where(keep, exp / (1 - p), torch.zeros(()))
    assert torch.equal(go2.cpu(), go.cpu()) and torch.equal(dgam2.cpu(), dgam.cpu())
    assert (br_t.float().cpu() - exp_t).abs().max() < tol * 4 + 1e-4
    assert (csum.cpu() - exp_t.sum(0)).abs().max() < 2e-3


@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,cols,B,T,H", [(2048, 512, 2, 1024, 8), (1536, 384, 3, 512, 8), (300, 100, 2, 150, 4),
                                             (64, 256, 1, 64, 2), (4000, 512, 1, 700, 1)])
def test_layernorm_fwd_mask_equals_two_launches(out_dtype, rows, cols, B, T, H):
    """cg_layernorm_fwd_mask (a block's LN1 rows and its attention keep words in one launch, engine
    option attn_mask_kernel=2) against cg_layernorm_fwd + cg_attn_drop_mask: every output bit for
    bit, the grid's LayerNorm and keep-word workgroups in every proportion (more rows than mask
    blocks and the reverse), a LayerNorm width without the vector path (100: the two-launch route),
    and every causal keep bit against the oracle's dropout_keep."""
    ops = _ops()
    g = torch.Generator().manual_seed(rows + cols)
    x = (torch.randn(rows, cols, generator=g) * 2 + 0.5).to(DEV)
    w = (1 + 0.1 * torch.randn(cols, generator=g)).to(DEV)
    b = (0.1 * torch.randn(cols, generator=g)).to(DEV)
    seed, p = 4242 + T, 0.1
    y, mean, rstd, mask = ops.layernorm_fwd_mask(x, w, b, B, T, H, seed, p, out_dtype=out_dtype)
    y2, mean2, rstd2 = ops.layernorm_fwd(x, w, b, out_dtype=out_dtype)
    ref = torch.zeros_like(mask)
    import ctypes as C
    L = __import__("codonlm_amd._lib", fromlist=["x"])
    L.check(L.lib.cg_attn_drop_mask(B, T, H, seed, C.c_float(p), ref.data_ptr(), L.stream_ptr(x.device)), "mask")
    torch.cuda.synchronize()
    assert torch.equal(y, y2) and torch.equal(mean, mean2) and torch.equal(rstd, rstd2)
    assert torch.equal(mask, ref)
    # the words decode to the oracle's keep bits on the causal triangle (pair-split order, tile-major)
    nt = (T + 63) // 64
    words = mask.cpu().numpy().view(np.uint32)[: B * H * nt * T * 2].reshape(B * H, nt, T, 2)
    bh = np.arange(B * H)[:, None, None]
    q = np.arange(T)[None, :, None]
    k = np.arange(T)[None, None, :]
    keep = O.dropout_keep(seed, bh * T + q, np.broadcast_to(k, (1, 1, T)), p)
    kt, kw, kc = k // 64, (k % 64) // 32, k % 32
    bit = np.where(kc % 2 == 0, kc // 2, 16 + kc // 2)
    got = (words[bh, kt, q, kw] >> bit) & 1
    causal = np.broadcast_to(k <= q, got.shape)
    assert np.array_equal(got[causal].astype(bool), np.broadcast_to(keep, got.shape)[causal])


@pytest.mark.parametrize("cols", [512, 100])
def test_layernorm_bwd_partials_deferred_reduce(cols):
    """The engine's deferred path (row pass writing partials + one batched cg_reduce_columns over
    several layers' partials) gives bitwise the in-call reduction of cg_layernorm_bwd."""
    ops = _ops()
    rows = 4096 + 37
    g = torch.Generator().manual_seed(11 + cols)
    x = (torch.randn(rows, cols, generator=g) * 2 + 0.5).to(DEV)
    w = (1 + 0.1 * torch.randn(cols, generator=g)).to(DEV)
    b = (0.1 * torch.randn(cols, generator=g)).to(DEV)
    _, mean, rstd = ops.layernorm_fwd(x, w, b, out_dtype=torch.bfloat16)
    dy = torch.randn(rows, cols, generator=g).to(DEV).to(torch.bfloat16)
    gin = torch.randn(rows, cols, generator=g).to(DEV)
    go, dgam, dbet, br_t, csum = ops.layernorm_bwd(dy, x, mean, rstd, w, g_in=gin, branch_dtype=torch.bfloat16,
                                                   drop_seed=5, drop_p=0.1)
    go_p, part, br_p = ops.layernorm_bwd_partials(dy, x, mean, rstd, w, g_in=gin, branch_dtype=torch.bfloat16,
                                                  drop_seed=5, drop_p=0.1)
    assert torch.equal(go_p, go) and torch.equal(br_p, br_t)
    # a second, unrelated job in the same batch (accumulating) and a 2-wide LayerNorm job
    other = torch.randn(96, 2048, generator=g).to(DEV)
    acc0 = torch.randn(2048, generator=g).to(DEV)
    acc = acc0.clone()
    outs = [torch.full((cols,), float("nan"), device=DEV) for _ in range(3)]
    ops.reduce_columns([(part[:, :cols], outs[0], 0), (other, acc, 1), (part[:, cols:2 * cols], outs[1], 0),
                        (part[:, 2 * cols:], outs[2], 0)])
    torch.cuda.synchronize()
    # bitwise where the vectorised row pass ran (its in-call reduction has the batched kernel's order)
    same = torch.equal if cols % 128 == 0 else (lambda a, e: (a - e).abs().max().item() <= 1e-4 * (1 + e.abs().max().item()))
    assert same(outs[0], dgam) and same(outs[1], dbet) and same(outs[2], csum)
    ref = acc0.double() + other.double().sum(0)
    assert (acc.double() - ref).abs().max().item() < 1e-4
    _, part2, _ = ops.layernorm_bwd_partials(dy, x, mean, rstd, w)
    assert part2.shape[1] == 2 * cols
    d2 = torch.empty(cols, device=DEV)
    ops.reduce_columns([(part2[:, :cols], d2, 0)])
    assert same(d2, dgam)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("H,Hp,ld_pad", [(1024, 1024, 0), (1365, 1408, 0), (100, 104, 8), (50, 51, 0)])
def test_swiglu_fwd_bwd(dtype, H, Hp, ld_pad):
    """model_tiny_gpt.py:47-57: vectorised 8-element runs (Hp % 8 == 0, aligned rows) and the scalar
    fallback (odd Hp), against torch autograd of silu(g) * u."""
    ops = _ops()
    rows = 333
    g = torch.Generator().manual_seed(H)
    full = torch.randn(rows, 2 * Hp + ld_pad, generator=g) * 2
    gu = full.to(DEV, dtype)[:, :2 * Hp]
    ds = torch.randn(rows, Hp, generator=g).to(DEV, dtype)
    s = ops.swiglu_fwd(gu, H)
    dgu = ops.swiglu_bwd(gu, ds, H)
    gr = gu.float().cpu()[:, :H].clone().requires_grad_(True)
    ur = gu.float().cpu()[:, Hp:Hp + H].clone().requires_grad_(True)
    ref = F.silu(gr) * ur
    ref.backward(ds.float().cpu()[:, :H])
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    sc = s.float().cpu()
    assert (sc[:, :H] - ref.detach()).abs().max() <= tol * (1 + ref.abs().max())
    assert torch.all(sc[:, H:] == 0)
    d = dgu.float().cpu()
    assert (d[:, :H] - gr.grad).abs().max() <= tol * (1 + gr.grad.abs().max())
    assert (d[:, Hp:Hp + H] - ur.grad).abs().max() <= tol * (1 + ur.grad.abs().max())
    assert torch.all(d[:, H:Hp] == 0) and torch.all(d[:, Hp + H:] == 0)


@pytest.mark.parametrize("tile", [0, 3])
@pytest.mark.parametrize("M,Hp,H,K", [(1024, 1024, 1024, 384), (700, 1408, 1365, 512), (256, 128, 100, 128)])
def test_gemm_swiglu_epilogues(M, Hp, H, K, tile):
    """The gate|up product with SwiGLU in the persistent tile's epilogue (CG_EPI_SWIGLU: B rows
    remapped so one lane holds gate j and up j) and the dL/ds product with the SwiGLU backward in
    its epilogue (CG_EPI_DSWIGLU), against the separate passes (cg_swiglu_fwd / _bwd) on the same
    bf16 products.  tile 0: automatic (the forward on the loader-wave kernel); 3 = CG_TILE_PERS:
    both on the eight-wave kernel."""
    ops = _ops()
    L = __import__("codonlm_amd._lib", fromlist=["x"])
    _swiglu_epilogues(ops, L, M, Hp, H, K, tile)


def _swiglu_epilogues(ops, L, M, Hp, H, K, tile=0):
    g = torch.Generator().manual_seed(M + Hp)
    x = (torch.randn(M, K, generator=g) * 0.5).to(DEV, torch.bfloat16)
    wgu = torch.randn(2 * Hp, K, generator=g) * K ** -0.5
    wgu[H:Hp] = 0
    wgu[Hp + H:] = 0
    wgu = wgu.to(DEV, torch.bfloat16)
    gu_ref = ops.gemm(x, wgu)                                  # [M][2Hp]
    s_ref = ops.swiglu_fwd(gu_ref, H)
    gu = torch.full((M, 2 * Hp), float("nan"), device=DEV, dtype=torch.bfloat16)
    s = ops.gemm(x, wgu, N=Hp, epilogue=L.EPI_SWIGLU, aux_out=gu, n_valid=H, tile=tile)
    torch.cuda.synchronize()
    assert torch.equal(gu, gu_ref)  # same products, same k order: bitwise
    # s from the unrounded fp32 g, u (the separate pass reads them in bf16): bf16-rounding close
    err = (s.float() - s_ref.float()).abs().max().item()
    assert err <= 1.6e-2 * (1 + s_ref.float().abs().max().item()), err
    assert torch.all(s[:, H:] == 0)
    # backward: dL/ds = gin . wd  (wd [d][Hp], K-contiguous operand wd^T [Hp][d])
    dmod = K
    gin = torch.randn(M, dmod, generator=g).to(DEV, torch.bfloat16)
    wdT = (torch.randn(Hp, dmod, generator=g) * dmod ** -0.5).to(DEV, torch.bfloat16)
    ds = ops.gemm(gin, wdT)                                    # [M][Hp]
    dgu_ref = ops.swiglu_bwd(gu_ref, ds, H)
    dgu = torch.full((M, 2 * Hp), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.gemm(gin, wdT, N=Hp, out=dgu, epilogue=L.EPI_DSWIGLU, aux=gu_ref, n_valid=H, tile=tile)
    torch.cuda.synchronize()
    # same fp32 product, dgu computed from it before rounding (the separate pass reads ds in
    # bf16): equal to bf16 rounding
    ref = dgu_ref.float()
    err = (dgu.float() - ref).abs().max().item()
    assert err <= 1.6e-2 * (1 + ref.abs().max().item()), err
    assert torch.all(dgu[:, H:Hp] == 0) and torch.all(dgu[:, Hp + H:] == 0)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("H,KV,hd", [(8, 4, 48), (4, 4, 64), (2, 1, 20)])
def test_rope_forward_inverse(dtype, H, KV, hd):
    """model_tiny_gpt.py:9-45 rotate-half RoPE on the q and k heads (v untouched); inverse undoes it.
    hd 48 / 64 take the vectorised path, hd 20 (half = 10) the scalar one."""
    ops = _ops()
    B, T = 3, 77
    ld = (H + 2 * KV) * hd
    g = torch.Generator().manual_seed(hd)
    qkv0 = torch.randn(B * T, ld, generator=g)
    half = hd // 2
    inv = 1.0 / (10000 ** (torch.arange(half, dtype=torch.float64) / half))
    ang = torch.arange(T, dtype=torch.float64)[:, None] * inv[None, :]
    cos, sin = torch.cos(ang).float(), torch.sin(ang).float()
    x = qkv0.to(DEV, dtype)
    ops.rope_(x, B, T, H, KV, hd, cos.to(DEV), sin.to(DEV))
    xr = x.float().cpu().view(B, T, -1)
    src = qkv0.to(dtype).float().view(B, T, -1)
    for h in range(H + KV):
        a = src[..., h * hd:h * hd + half]
        b = src[..., h * hd + half:(h + 1) * hd]
        exp = torch.cat([a * cos - b * sin, b * cos + a * sin], -1)
        tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
        assert (xr[..., h * hd:(h + 1) * hd] - exp).abs().max() <= tol * 4
    assert torch.equal(xr[..., (H + KV) * hd:], src[..., (H + KV) * hd:])
    ops.rope_(x, B, T, H, KV, hd, cos.to(DEV), sin.to(DEV), inverse=True)
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-5
    assert (x.float().cpu() - qkv0.to(dtype).float()).abs().max() <= tol * 4


def test_segment_starts():
    ops = _ops()
    idx = torch.randint(4, 68, (3, 700))
    idx[0, 5] = 3
    idx[0, 300] = 3
    idx[1, 0] = 3
    idx[2, 699] = 3
    got = ops.segment_starts(idx.to(DEV), 3).cpu()
    exp = torch.zeros_like(got)
    for b in range(3):
        last = 0
        for t in range(700):
            if idx[b, t] == 3:
                last = t
            exp[b, t] = last
    assert torch.equal(got, exp)


def _attn_ref(qkv, idx, B, T, H, KV, hd, sep, window, drop=None):
    q = qkv[:, : H * hd].view(B, T, H, hd).transpose(1, 2)
    k = qkv[:, H * hd: (H + KV) * hd].view(B, T, KV, hd).transpose(1, 2)
    v = qkv[:, (H + KV) * hd:].view(B, T, KV, hd).transpose(1, 2)
    k = k.repeat_interleave(H // KV, 1)
    v = v.repeat_interleave(H // KV, 1)
    att = (q @ k.transpose(-2, -1)) / math.sqrt(hd)
    m = O.attention_mask(idx, sep, window)
    att = att.masked_fill(~m[:, None], float("-inf")).softmax(-1)
    if drop is not None:
        att = att * drop
    return (att @ v).transpose(1, 2).reshape(B * T, H * hd)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,T,H,KV,hd,window,p", [
    (2, 64, 4, 4, 16, 0, 0.0), (2, 200, 4, 2, 64, 0, 0.0), (1, 256, 8, 4, 48, 0, 0.0),
    (2, 130, 2, 1, 32, 17, 0.0), (2, 96, 4, 4, 64, 0, 0.2)])
def test_attention_fwd_bwd(dtype, B, T, H, KV, hd, window, p):
    ops = _ops()
    g = torch.Generator().manual_seed(T + H)
    N = (H + 2 * KV) * hd
    qkv = torch.randn(B * T, N, generator=g)
    if dtype == torch.bfloat16:
        qkv = _bf(qkv)
    idx = torch.randint(4, 68, (B, T), generator=g)
    idx[:, T // 3] = 3
    idx[0, T // 2] = 3
    seed = 777
    drop = None
    if p > 0:
        keep = O.dropout_keep(seed, np.arange(B * H * T)[:, None], np.arange(T)[None, :], p)
        drop = torch.from_numpy(keep.astype(np.float32) / (1 - p)).view(B, H, T, T)
    qr = qkv.clone().requires_grad_(True)
    ref = _attn_ref(qr, idx, B, T, H, KV, hd, 3, window or None, drop)
    seg = ops.segment_starts(idx.to(DEV), 3)
    qd = qkv.to(DEV, dtype)
    y, lse = ops.attn_fwd(qd, seg, B, T, H, KV, hd, window=window, drop_seed=seed, drop_p=p)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert (y.float().cpu() - ref.detach()).abs().max() < tol
    dy = torch.randn(B * T, H * hd, generator=g)
    if dtype == torch.bfloat16:
        dy = _bf(dy)
    ref.backward(dy)
    dq = ops.attn_bwd(qd, seg, y, dy.to(DEV, dtype), lse, B, T, H, KV, hd, window=window, drop_seed=seed, drop_p=p)
    err = (dq.float().cpu() - qr.grad).abs().max().item()
    scale = qr.grad.abs().max().item()
    assert err < (5e-2 if dtype == torch.bfloat16 else 1e-4) * max(1.0, scale), err


@pytest.mark.parametrize("B,T,H,KV,hd,p", [(2, 1024, 8, 8, 64, 0.0), (2, 1024, 8, 8, 64, 0.1),
                                             (2, 512, 8, 4, 48, 0.0), (2, 512, 8, 4, 48, 0.1)])
def test_attention_mfma_full_geometry(B, T, H, KV, hd, p):
    """The bf16 MFMA attention kernels at the benchmarked geometries (C4: T1024 hd64, dropout
    0.1; C3/C5: T512 hd48 GQA-4) against fp32 autograd of the same bf16-rounded inputs.
    Bounds: bf16 output / probability rounding (2^-9 relative) -> rel-L2 <= 1e-2 forward,
    <= 2e-2 for the q/k/v gradients."""
    ops = _ops()
    g = torch.Generator().manual_seed(T * 3 + hd)
    N = (H + 2 * KV) * hd
    qkv = _bf(torch.randn(B * T, N, generator=g))
    idx = torch.randint(4, 68, (B, T), generator=g)
    for pos in (T // 5, T // 2, T - 300):
        idx[0, pos] = 3
    idx[1, T // 3] = 3
    seed = 9001
    drop = None
    if p > 0:
        keep = O.dropout_keep(seed, np.arange(B * H * T)[:, None], np.arange(T)[None, :], p)
        drop = torch.from_numpy(keep.astype(np.float32) / (1 - p)).view(B, H, T, T)
    qr = qkv.clone().requires_grad_(True)
    ref = _attn_ref(qr, idx, B, T, H, KV, hd, 3, None, drop)
    seg = ops.segment_starts(idx.to(DEV), 3)
    qd = qkv.to(DEV, torch.bfloat16)
    y, lse = ops.attn_fwd(qd, seg, B, T, H, KV, hd, drop_seed=seed, drop_p=p)
    yf = y.float().cpu()

    def rel(a, b):
        return float((a.double() - b.double()).norm() / b.double().norm())
    assert rel(yf, ref.detach()) <= 1e-2
    dy = _bf(torch.randn(B * T, H * hd, generator=g))
    ref.backward(dy)
    dq = ops.attn_bwd(qd, seg, y, dy.to(DEV, torch.bfloat16), lse, B, T, H, KV, hd, drop_seed=seed, drop_p=p)
    dqf = dq.float().cpu()
    for name, sl in (("dq", slice(0, H * hd)), ("dk", slice(H * hd, (H + KV) * hd)),
                     ("dv", slice((H + KV) * hd, N))):
        e = rel(dqf[:, sl], qr.grad[:, sl])
        assert e <= 2e-2, (name, e)


@pytest.mark.parametrize("ksplit", [1, 2, 3])
@pytest.mark.parametrize("K", [2048, 1023, 37])
@pytest.mark.parametrize("tile", [128, 129, 256, 512])
def test_gemm_dw_grouped_tiles(tile, K, ksplit):
    """Grouped full-reduction dW (cg_gemm_dw_grouped) for every tile code, against fp32 products
    of the same bf16 operands: ragged N_out / K_out (partial tiles), strided operands, alpha and
    accumulate, products of different shapes in one launch, and token counts K that are not a
    multiple of the 64-row k-step (the dynamic-length loader's B*T; the last step's rows >= K are
    zero-filled by the buffer range check).  Bound: fp32 accumulation of exact bf16 products over
    K rows -> max error <= 1e-5 of the output scale."""
    ops = _ops()
    g = torch.Generator().manual_seed(tile + K)
    shapes = [(200, 136), (512, 384), (72, 520), (1536, 512)]
    prods, refs = [], []
    for i, (n, k) in enumerate(shapes):
        dy_full = _bf(torch.randn(K, n + 8, generator=g)).to(DEV, torch.bfloat16)
        dy = dy_full[:, :n]  # row stride n + 8
        x = _bf(torch.randn(K, k, generator=g)).to(DEV, torch.bfloat16)
        alpha, acc = (0.5, True) if i % 2 else (1.0, False)
        out = torch.randn(n, k, generator=g).to(DEV) if acc else torch.empty(n, k, device=DEV)
        ref = alpha * (dy.float().t() @ x.float()) + (out.clone() if acc else 0)
        prods.append((dy, x, out, alpha, acc))
        refs.append(ref)
    first = [p[2].clone() for p in prods]
    ops.gemm_dw_grouped(prods, tile_m=tile, ksplit=ksplit)
    torch.cuda.synchronize()
    for (dy, x, out, _, _), ref in zip(prods, refs):
        err = ((out - ref).abs().max() / ref.abs().max()).item()
        assert err <= 1e-5, (tile, ksplit, tuple(out.shape), err)
    if ksplit > 1:  # the split (slabs + in-order reduction) is deterministic: a rerun is bitwise equal
        again = []
        for (dy, x, out, alpha, acc), f in zip(prods, first):
            o2 = f.clone()
            again.append((dy, x, o2, alpha, acc))
        ops.gemm_dw_grouped(again, tile_m=tile, ksplit=ksplit)
        torch.cuda.synchronize()
        for (_, _, o2, _, _), (_, _, out, _, _) in zip(again, prods):
            assert torch.equal(o2, out)


@pytest.mark.parametrize("K", [2048, 1023, 37])
@pytest.mark.parametrize("tile", [128, 129, 256, 512])
def test_gemm_dw_grouped_colsum(tile, K):
    """The grouped dW's column-sum output (cg_dw_product.col_sum: the bias gradient of the
    nn.Linear, the column sums of dY taken from the fragments the tiles stream) for every tile
    code: products with and without it in one launch, alpha and accumulate, ragged N_out (partial
    row tiles) and K.  The dW results stay as without it (bitwise), the sums within fp32 summation
    order of the exact bf16 values (1e-5 of the scale); with a token split it is CG_EUNSUPPORTED."""
    ops = _ops()
    g = torch.Generator().manual_seed(7 * tile + K)
    shapes = [(2048, 512), (200, 136), (512, 384), (72, 520)]
    prods, plain, refs = [], [], []
    for i, (n, k) in enumerate(shapes):
        dy = _bf(torch.randn(K, n, generator=g) + 0.3).to(DEV, torch.bfloat16)
        x = _bf(torch.randn(K, k, generator=g)).to(DEV, torch.bfloat16)
        alpha, acc = (0.5, True) if i % 2 else (1.0, False)
        out = torch.randn(n, k, generator=g).to(DEV)
        cs = torch.randn(n, generator=g).to(DEV) if i != 2 else None
        ref = alpha * dy.float().sum(0) + (cs.clone() if acc else 0) if cs is not None else None
        prods.append((dy, x, out.clone(), alpha, acc, cs))
        plain.append((dy, x, out.clone(), alpha, acc))
        refs.append(ref)
    ops.gemm_dw_grouped(prods, tile_m=tile)
    ops.gemm_dw_grouped(plain, tile_m=tile)
    torch.cuda.synchronize()
    for p, q, ref in zip(prods, plain, refs):
        assert torch.equal(p[2], q[2])
        if ref is not None:
            err = ((p[5] - ref).abs().max() / ref.abs().max()).item()
            assert err <= 1e-5, (tile, K, tuple(p[2].shape), err)
    with pytest.raises(ValueError):
        ops.gemm_dw_grouped(prods[:1], tile_m=tile, ksplit=2)


@pytest.mark.parametrize("B,T,H,KV,hd,p", [(2, 1024, 8, 8, 64, 0.1), (2, 200, 4, 2, 48, 0.0), (1, 130, 2, 1, 32, 0.1)])
def test_attention_bwd_bias_partials(B, T, H, KV, hd, p):
    """The q/k/v bias-gradient partials written by the MFMA attention backward reduce to the
    column sums of its dqkv (fp32 sums of the unrounded values vs sums of the bf16 output:
    within bf16 rounding of the rows, rel <= 2e-3 of the column-sum scale)."""
    ops = _ops()
    g = torch.Generator().manual_seed(T + hd)
    N = (H + 2 * KV) * hd
    qkv = _bf(torch.randn(B * T, N, generator=g)).to(DEV, torch.bfloat16)
    idx = torch.randint(4, 68, (B, T), generator=g)
    idx[0, T // 2] = 3
    seg = ops.segment_starts(idx.to(DEV), 3)
    y, lse = ops.attn_fwd(qkv, seg, B, T, H, KV, hd, drop_seed=5, drop_p=p)
    dy = _bf(torch.randn(B * T, H * hd, generator=g)).to(DEV, torch.bfloat16)
    nrb = B * ((T + 127) // 128)
    part = torch.full((nrb, N + 8), float("nan"), device=DEV)
    dqkv = ops.attn_bwd(qkv, seg, y, dy, lse, B, T, H, KV, hd, drop_seed=5, drop_p=p, bias_part=part)
    got = part[:, :N].sum(0)
    ref = dqkv.float().sum(0)
    assert torch.isfinite(got).all()
    assert float((got - ref).abs().max() / ref.abs().max()) <= 2e-3


def _rope_tabs(T, hd):
    half = hd // 2
    inv = 1.0 / (10000 ** (torch.arange(half, dtype=torch.float64) / half))
    ang = torch.arange(T, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.cos(ang).float(), torch.sin(ang).float()


def _rope_ref(x, cos, sin, nh, hd):
    """rotate-half RoPE (model_tiny_gpt.py:35-45) on nh heads of x [B*T][nh*hd] (T = cos rows)."""
    T, half = cos.shape
    xv = x.view(-1, T, nh, hd)
    a, b = xv[..., :half], xv[..., half:]
    c, s = cos[None, :, None, :], sin[None, :, None, :]
    return torch.cat([a * c - b * s, b * c + a * s], -1).reshape(x.shape)


@pytest.mark.parametrize("B,T,H,KV,hd,p", [(2, 1024, 8, 8, 64, 0.1), (2, 512, 8, 4, 48, 0.0),
                                             (2, 300, 8, 4, 48, 0.1), (1, 130, 4, 2, 32, 0.0)])
def test_attention_bwd_rope_fused(B, T, H, KV, hd, p):
    """cg_attn_bwd_rope: the inverse RoPE rotation of dQ / dK inside the MFMA backward kernels
    (model_tiny_gpt.py:91-93 rotates q, k after the projection; the engine's RoPE backward since
    round 4) against fp32 autograd through rotation + attention of the same bf16-rounded
    projections (rel-L2 <= 2e-2 per q / k / v block, as the plain MFMA backward), against the
    unfused path (backward, then the cg_rope_tab inverse pass; the fused one rounds once instead
    of twice: rel <= 1e-2), and its bias partials against the column sums of its own dqkv."""
    ops = _ops()
    g = torch.Generator().manual_seed(T + hd + 1)
    N = (H + 2 * KV) * hd
    proj = _bf(torch.randn(B * T, N, generator=g))
    idx = torch.randint(4, 68, (B, T), generator=g)
    idx[0, T // 2] = 3
    cos, sin = _rope_tabs(T, hd)
    pr = proj.clone().requires_grad_(True)
    q = _rope_ref(pr[:, :H * hd], cos, sin, H, hd)
    k = _rope_ref(pr[:, H * hd:(H + KV) * hd], cos, sin, KV, hd)
    rot = torch.cat([q, k, pr[:, (H + KV) * hd:]], 1)
    seed = 4242
    drop = None
    if p > 0:
        keep = O.dropout_keep(seed, np.arange(B * H * T)[:, None], np.arange(T)[None, :], p)
        drop = torch.from_numpy(keep.astype(np.float32) / (1 - p)).view(B, H, T, T)
    ref = _attn_ref(rot, idx, B, T, H, KV, hd, 3, None, drop)
    dy = _bf(torch.randn(B * T, H * hd, generator=g))
    ref.backward(dy)
    seg = ops.segment_starts(idx.to(DEV), 3)
    cd, sd = cos.to(DEV), sin.to(DEV)
    qkv = proj.to(DEV, torch.bfloat16)
    ops.rope_(qkv, B, T, H, KV, hd, cd, sd)
    y, lse = ops.attn_fwd(qkv, seg, B, T, H, KV, hd, drop_seed=seed, drop_p=p)
    dyd = dy.to(DEV, torch.bfloat16)
    nrb = B * ((T + 127) // 128)
    part = torch.full((nrb, N), float("nan"), device=DEV)
    fused = ops.attn_bwd(qkv, seg, y, dyd, lse, B, T, H, KV, hd, drop_seed=seed, drop_p=p, bias_part=part,
                         rope=(cd, sd))
    unf = ops.attn_bwd(qkv, seg, y, dyd, lse, B, T, H, KV, hd, drop_seed=seed, drop_p=p)
    ops.rope_(unf, B, T, H, KV, hd, cd, sd, inverse=True)
    ff, uf = fused.float().cpu(), unf.float().cpu()

    def rel(a, b):
        return float((a.double() - b.double()).norm() / b.double().norm())
    for name, sl in (("dq", slice(0, H * hd)), ("dk", slice(H * hd, (H + KV) * hd)),
                     ("dv", slice((H + KV) * hd, N))):
        assert rel(ff[:, sl], pr.grad[:, sl]) <= 2e-2, (name, rel(ff[:, sl], pr.grad[:, sl]))
        assert rel(ff[:, sl], uf[:, sl]) <= 1e-2, (name, rel(ff[:, sl], uf[:, sl]))
    assert torch.equal(ff[:, (H + KV) * hd:], uf[:, (H + KV) * hd:])  # dV: same kernel, no rotation
    got = part.sum(0)
    colsum = fused.float().sum(0)
    assert torch.isfinite(got).all()
    assert float((got - colsum).abs().max() / colsum.abs().max()) <= 2e-3


def _mask_bits(words, T):
    """Unpack attn_drop_mask words -- tile-major [BH, nt, T, 2] (nt = ceil(T/64) key tiles), pair-split
    bit order -- into bool [BH, T(query), T(key)]."""
    nt = (T + 63) // 64
    w = words.cpu().numpy().view(np.uint32).reshape(-1, nt, T, 2)
    i = np.arange(T)
    bit = (i % 32 >> 1) + 16 * (i % 2)
    half = ((i % 64) // 32)[None, :, None]
    w0, w1 = w[..., 0], w[..., 1]                                      # [BH, nt, T]
    wk = np.where(half == 0, w0[:, i // 64, :], w1[:, i // 64, :])      # [BH, key, query]
    kb = ((wk >> bit.astype(np.uint32)[None, :, None]) & 1).astype(bool)
    return np.ascontiguousarray(np.transpose(kb, (0, 2, 1)))


@pytest.mark.parametrize("B,T,H", [(2, 200, 3), (1, 1024, 2), (1, 64, 1), (1, 129, 1)])
def test_attn_drop_mask_bits(B, T, H):
    """The precomputed attention keep bits equal the oracle's dropout_keep on every causal
    (query, key) pair."""
    ops = _ops()
    seed, p = 4242, 0.1
    mask = ops.attn_drop_mask(B, T, H, seed, p, DEV)
    torch.cuda.synchronize()
    wpr = 2 * ((T + 63) // 64)
    assert mask.numel() == B * H * T * wpr
    qm = _mask_bits(mask, T)        # [bh, q, key]
    keep = O.dropout_keep(seed, np.arange(B * H * T)[:, None], np.arange(T)[None, :], p).reshape(B * H, T, T)
    causal = np.tril(np.ones((T, T), dtype=bool))[None]
    assert np.array_equal(qm & causal, keep & causal)
    assert 0.85 < keep[causal.repeat(B * H, 0)].mean() < 0.95


@pytest.mark.parametrize("B,T,H,KV,hd", [(2, 1024, 8, 8, 64), (2, 512, 8, 4, 48), (1, 200, 4, 2, 32),
                                         (1, 129, 2, 1, 64)])
def test_attention_drop_mask_path_matches_hash_path(B, T, H, KV, hd):
    """bf16 MFMA attention with precomputed keep bits vs the in-kernel hash: identical keep
    decisions, so the forward is bitwise equal; the backward differs only by fma contraction
    (rel-L2 <= 1e-3)."""
    ops = _ops()
    g = torch.Generator().manual_seed(hd + T)
    N = (H + 2 * KV) * hd
    qkv = _bf(torch.randn(B * T, N, generator=g)).to(DEV, torch.bfloat16)
    idx = torch.randint(4, 68, (B, T), generator=g)
    idx[0, T // 3] = 3
    seg = ops.segment_starts(idx.to(DEV), 3)
    seed, p = 31337, 0.1
    mask = ops.attn_drop_mask(B, T, H, seed, p, DEV)
    y0, l0 = ops.attn_fwd(qkv, seg, B, T, H, KV, hd, drop_seed=seed, drop_p=p)
    y1, l1 = ops.attn_fwd(qkv, seg, B, T, H, KV, hd, drop_seed=seed, drop_p=p, drop_mask=mask)
    assert torch.equal(y0, y1) and torch.equal(l0, l1)
    dy = _bf(torch.randn(B * T, H * hd, generator=g)).to(DEV, torch.bfloat16)
    d0 = ops.attn_bwd(qkv, seg, y0, dy, l0, B, T, H, KV, hd, drop_seed=seed, drop_p=p).float()
    d1 = ops.attn_bwd(qkv, seg, y0, dy, l0, B, T, H, KV, hd, drop_seed=seed, drop_p=p, drop_mask=mask).float()
    assert float((d1 - d0).norm() / d0.norm()) <= 1e-3


@pytest.mark.parametrize("B,T,H,KV,hd,window,sep", [(2, 1024, 8, 8, 64, 0, True), (2, 512, 8, 4, 48, 0, True),
                                                    (1, 200, 4, 2, 32, 0, False), (1, 129, 2, 1, 64, 0, True),
                                                    (1, 300, 2, 2, 64, 70, False)])
def test_attention_fused_keep_forward(B, T, H, KV, hd, window, sep):
    """cg_attn_fwd_keep: the forward that hashes its own keep decisions writes, for every (query, key)
    pair a query sees, exactly attn_drop_mask's bit, and its y / lse equal the forward that reads
    attn_drop_mask's words (bitwise); the backward reading the fused words equals the one reading
    the mask kernel's."""
    ops = _ops()
    g = torch.Generator().manual_seed(7 * hd + T)
    N = (H + 2 * KV) * hd
    qkv = _bf(torch.randn(B * T, N, generator=g)).to(DEV, torch.bfloat16)
    idx = torch.randint(4, 68, (B, T), generator=g)
    if sep:
        idx[0, T // 3] = 3
        idx[-1, (2 * T) // 3] = 3
    seg = ops.segment_starts(idx.to(DEV), 3 if sep else -1)
    seed, p = 2024, 0.1
    ref = ops.attn_drop_mask(B, T, H, seed, p, DEV)
    y0, l0 = ops.attn_fwd(qkv, seg, B, T, H, KV, hd, window=window, drop_seed=seed, drop_p=p, drop_mask=ref)
    y1, l1, mk = ops.attn_fwd_keep(qkv, seg, B, T, H, KV, hd, seed, p, window=window)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1) and torch.equal(l0, l1)
    wpr = 2 * ((T + 63) // 64)
    a = _mask_bits(ref, T)
    b = _mask_bits(mk, T)
    # visible pairs: causal, same SEP segment (key >= segment start), inside the window
    q = np.arange(T)[:, None]
    k = np.arange(T)[None, :]
    st = seg.view(B, T).cpu().numpy().astype(np.int64)
    vis = (k <= q)[None] & (k >= st[:, :, None])
    if window:
        vis = vis & (k > q - window)[None]
    vis = np.repeat(vis, H, axis=0).reshape(B * H, T, T)
    assert np.array_equal(a & vis, b & vis)
    dy = _bf(torch.randn(B * T, H * hd, generator=g)).to(DEV, torch.bfloat16)
    d0 = ops.attn_bwd(qkv, seg, y0, dy, l0, B, T, H, KV, hd, window=window, drop_seed=seed, drop_p=p, drop_mask=ref)
    d1 = ops.attn_bwd(qkv, seg, y1, dy, l1, B, T, H, KV, hd, window=window, drop_seed=seed, drop_p=p, drop_mask=mk)
    assert torch.equal(d0, d1)


@pytest.mark.parametrize("V,d,p,acc", [(68, 512, 0.1, 0), (68, 256, 0.0, 1), (80, 384, 0.1, 0), (150, 256, 0.1, 1),
                                    (150, 128, 0.0, 0)])
def test_embed_bwd_token_rows(V, d, p, acc):
    """cg_embed_bwd's token-embedding gradient -- the float2 kernel (V <= 80) and the 64-column one --
    against an fp64 index_add of the dropout-kept rows (the oracle's keep hash), plain and accumulating."""
    from codonlm_amd import _lib as L
    B, T = 3, 217  # ragged: 651 rows, not a multiple of either kernel's row chunking
    M = B * T
    g = torch.Generator().manual_seed(V + d)
    idx = torch.randint(0, V, (B, T), generator=g)
    idx[0, :40] = 5  # one token on many consecutive rows (the serial per-lane add chain)
    gr = torch.randn(M, d, generator=g)
    seed = 77
    keep = O.dropout_keep(seed, np.arange(M)[:, None], np.arange(d)[None, :], p) if p > 0 else np.ones((M, d), bool)
    scale = 1.0 / (1.0 - p) if p > 0 else 1.0
    base = torch.randn(V, d, generator=g)
    ref = (base.double() if acc else torch.zeros(V, d, dtype=torch.float64)).index_add_(
        0, idx.view(-1), gr.double() * torch.from_numpy(keep).double() * scale)
    idx_d, gr_d = idx.to(DEV), gr.to(DEV)
    dtok = base.to(DEV) if acc else torch.full((V, d), float("nan"), device=DEV)
    need = int(L.lib.cg_embed_bwd_workspace(B, T, V, d))
    ws = torch.empty(need // 4 + 1, dtype=torch.float32, device=DEV)
    assert L.lib.cg_embed_bwd(idx_d.data_ptr(), gr_d.data_ptr(), dtok.data_ptr(), None, B, T, V, d, seed, p, acc,
                              ws.data_ptr(), need, L.stream_ptr(DEV)) == 0
    torch.cuda.synchronize()
    assert torch.allclose(dtok.cpu().double(), ref, atol=2e-4, rtol=1e-5)
    # the position rows: sum over the batch of the same kept rows (float4 kernel when d % 4 == 0)
    pbase = torch.randn(T, d, generator=g)
    kept = gr.double() * torch.from_numpy(keep).double() * scale
    pref = kept.view(B, T, d).sum(0) + (pbase.double() if acc else 0.0)
    dpos = pbase.to(DEV) if acc else torch.full((T, d), float("nan"), device=DEV)
    assert L.lib.cg_embed_bwd(idx_d.data_ptr(), gr_d.data_ptr(), None, dpos.data_ptr(), B, T, V, d, seed, p, acc,
                              None, 0, L.stream_ptr(DEV)) == 0
    torch.cuda.synchronize()
    assert torch.allclose(dpos.cpu().double(), pref, atol=2e-5, rtol=1e-5)


@pytest.mark.parametrize("eps,weighted", [(0.0, False), (0.05, False), (0.1, True)])
def test_cross_entropy(eps, weighted):
    ops = _ops()
    rows, V = 517, 68
    g = torch.Generator().manual_seed(11)
    z = torch.randn(rows, V, generator=g) * 5
    t = torch.randint(0, V, (rows,), generator=g)
    t[:50] = 0
    w = torch.rand(V, generator=g) + 0.5 if weighted else None
    zr = z.clone().requires_grad_(True)
    ref = F.cross_entropy(zr, t, ignore_index=0, label_smoothing=eps, weight=w)
    ref.backward()
    loss, dl = ops.cross_entropy(z.to(DEV), t.to(DEV), eps=eps, weight=w.to(DEV) if w is not None else None,
                                 pad_to=80)
    assert abs(loss.item() - ref.item()) < 1e-5 * max(1, abs(ref.item()))
    assert (dl[:, :V].cpu() - zr.grad).abs().max() < 1e-6
    assert torch.all(dl[:, V:] == 0)


def test_cross_entropy_all_pad_is_nan():
    ops = _ops()
    z = torch.randn(8, 68, device=DEV)
    t = torch.zeros(8, dtype=torch.long, device=DEV)
    loss, _ = ops.cross_entropy(z, t)
    assert math.isnan(loss.item())


def test_adamw_matches_torch():
    ops = _ops()
    n = 10000
    g = torch.Generator().manual_seed(5)
    p0 = torch.randn(n, generator=g)
    ps = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ps], lr=1e-3, weight_decay=0.05)
    pd = p0.clone().to(DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    shadow = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    for step in range(1, 4):
        grad = torch.randn(n, generator=g)
        ps.grad = grad.clone()
        opt.step()
        ops.adamw_(pd, (grad * 4).to(DEV), m, v, step, [(0, n, 1e-3, 0.05)], shadow=shadow, grad_scale=0.25)
    assert (pd.cpu() - ps.detach()).abs().max() < 1e-6
    assert (shadow.float().cpu() - ps.detach()).abs().max() < 1e-2


@pytest.mark.parametrize("shift", [1, 2, 3])
def test_adamw_offset_views(shift):
    """Offset views through the C ABI (bases not 16-B / 8-B aligned) take the elementwise path
    and give the aligned result bit for bit (the float4 interior needs aligned bases)."""
    ops = _ops()
    n = 5001
    g = torch.Generator().manual_seed(50 + shift)
    p0, grad = torch.randn(n, generator=g), torch.randn(n, generator=g)
    outs = []
    for off in (0, shift):
        bufs = [torch.zeros(n + 8, device=DEV) for _ in range(4)]
        pd, gd, m, v = (b[off:off + n] for b in bufs)
        pd.copy_(p0.to(DEV))
        gd.copy_(grad.to(DEV))
        sh = torch.zeros(n + 8, dtype=torch.bfloat16, device=DEV)[off:off + n]
        for step in (1, 2):
            ops.adamw_(pd, gd, m, v, step, [(0, 1000, 1e-3, 0.05), (1000, n, 2e-3, 0.0)], shadow=sh, grad_scale=0.5)
        torch.cuda.synchronize()
        outs.append((pd.cpu().clone(), m.cpu().clone(), v.cpu().clone(), sh.float().cpu().clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("ak,bk", [(1, 1), (1, 0), (0, 0), (0, 1)])
@pytest.mark.parametrize("M,N,K", [(512, 256, 512), (1000, 200, 192), (256, 136, 1024)])
def test_gemm_wide_tile(mode, ak, bk, M, N, K):
    """The 256x128 LDS-DMA tile (mode 1: CG_TILE_WIDE) and the 128x128 register-staged tile (mode 0:
    CG_TILE_VEC) against fp32, incl. partial M/N tiles and split-K, every operand layout."""
    ops = _ops()
    L = __import__("codonlm_amd._lib", fromlist=["x"])
    g = torch.Generator().manual_seed(M + N + K + 10 * ak + bk)
    Am = torch.randn(M, K, generator=g)
    Bn = torch.randn(N, K, generator=g)
    bias = torch.randn(N, generator=g)
    a = (Am if ak else Am.t().contiguous()).to(DEV, torch.bfloat16)
    b = (Bn if bk else Bn.t().contiguous()).to(DEV, torch.bfloat16)
    ref = _bf(Am) @ _bf(Bn).t()
    t = L.TILE_WIDE if mode else L.TILE_VEC
    out = ops.gemm(a, b, a_kcontig=bool(ak), b_kcontig=bool(bk), M=M, N=N, K=K, out_dtype=torch.float32, tile=t)
    outb = ops.gemm(a, b, a_kcontig=bool(ak), b_kcontig=bool(bk), M=M, N=N, K=K, out_dtype=torch.bfloat16,
                    bias=bias.to(DEV), epilogue=L.EPI_BIAS, tile=t)
    outs = ops.gemm(a, b, a_kcontig=bool(ak), b_kcontig=bool(bk), M=M, N=N, K=K, out_dtype=torch.float32,
                    split_k=2, tile=t)
    torch.cuda.synchronize()
    tol = 2e-2 * math.sqrt(K)
    assert (out.cpu() - ref).abs().max().item() <= tol
    assert (outs.cpu() - ref).abs().max().item() <= tol
    assert (outb.float().cpu() - (ref + bias)).abs().max().item() <= tol + 0.05 * (ref + bias).abs().max().item()


def test_gemm_forced_tile_errors():
    """A forced tile is a bf16 kernel: an unknown code is CG_EINVAL and a forced tile on fp32 operands
    is CG_EUNSUPPORTED (both ValueError), never a silent run of the f32-MFMA kernel."""
    ops = _ops()
    L = __import__("codonlm_amd._lib", fromlist=["x"])
    a = torch.randn(256, 256, device=DEV)
    for t in (-1, 5, 7):
        with pytest.raises(ValueError):
            ops.gemm(a.to(torch.bfloat16), a.to(torch.bfloat16), tile=t)
    for t in (L.TILE_VEC, L.TILE_WIDE, L.TILE_PERS, L.TILE_PERS_LW):
        with pytest.raises(ValueError):
            ops.gemm(a, a, tile=t)
    ops.gemm(a, a, tile=L.TILE_AUTO)  # fp32 on the automatic choice still runs


def test_transpose16_batch():
    ops = _ops()
    g = torch.Generator().manual_seed(5)
    mats = [torch.randn(r, c, generator=g).to(DEV, torch.bfloat16) for r, c in [(1536, 512), (72, 200), (8, 8), (520, 64)]]
    mats.append(torch.randn(64, 1408, generator=g).to(DEV, torch.bfloat16)[:, :1368])  # strided view
    outs = ops.transpose16(mats)
    for m, o in zip(mats, outs):
        assert torch.equal(o.cpu(), m.cpu().t())


@pytest.mark.parametrize("lw", [0, 1, 2])
@pytest.mark.parametrize("cap", [1, 3])
@pytest.mark.parametrize("M,N,K", [(600, 200, 192), (1000, 264, 128), (512, 384, 256), (600, 200, 320),
                                   (520, 264, 512)])
def test_gemm_persistent_tile_epilogues(cap, M, N, K, lw):
    """Persistent 256x128 tile (K-contiguous operands): every compile-time epilogue, partial
    M/N tiles, and (cap=3) a grid of 3 workgroups that each walk many tiles, so the LDS-DMA ring
    and the counted waits carry across tile boundaries with epilogue stores in flight.  K = 128 /
    192 issue the epilogue loads in the last k-step; K = 256 / 320 / 512 spread them over the
    tile's last 1 / 2 / 4 k-steps.  CG_EPI_GELU_DERIV: the forward stores gelu'(pre) and the
    backward multiplies by it.  lw=0: the eight-wave kernel (CG_TILE_PERS) for every epilogue;
    lw=1: automatic (each epilogue on the kernel the engine uses); lw=2: the loader-wave variant
    (gemm_lw.h, CG_TILE_PERS_LW) for every epilogue it implements."""
    ops = _ops()
    L = __import__("codonlm_amd._lib", fromlist=["x"])
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) * 0.1
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    xd, wd = x.to(DEV, torch.bfloat16), w.to(DEV, torch.bfloat16)
    base = _bf(x) @ _bf(w).t()
    tol = 3e-2 * 4
    gemm = functools.partial(ops.gemm, tile=(L.TILE_PERS, L.TILE_AUTO, L.TILE_PERS_LW)[lw],
                             max_wg=cap if cap > 1 else 0)
    y0 = gemm(xd, wd, out_dtype=torch.float32)
    y0b = gemm(xd, wd, out_dtype=torch.bfloat16)
    yb = gemm(xd, wd, out_dtype=torch.bfloat16, bias=bias.to(DEV), epilogue=L.EPI_BIAS)
    yr = gemm(xd, wd, out_dtype=torch.float32, bias=bias.to(DEV), resid=res.to(DEV),
                  epilogue=L.EPI_BIAS | L.EPI_RESID)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    yg = gemm(xd, wd, out_dtype=torch.bfloat16, bias=bias.to(DEV), epilogue=L.EPI_BIAS | L.EPI_GELU,
                  aux_out=aux)
    ydg = gemm(xd, wd, out_dtype=torch.bfloat16, epilogue=L.EPI_DGELU, aux=aux)
    p, seed = 0.25, 777
    ydr = gemm(xd, wd, out_dtype=torch.float32, bias=bias.to(DEV), resid=res.to(DEV),
                   epilogue=L.EPI_BIAS | L.EPI_DROPOUT | L.EPI_RESID, drop_seed=seed, drop_p=p)
    acc0 = torch.randn(M, N, generator=g)
    yac = acc0.clone().to(DEV)
    gemm(xd, wd, out=yac, epilogue=L.EPI_ACCUM, alpha=0.5)
    cs = torch.empty(N, device=DEV)
    ydc = gemm(xd, wd, out_dtype=torch.bfloat16, epilogue=L.EPI_DGELU, aux=aux, colsum_out=cs)
    auxd = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ygd = gemm(xd, wd, out_dtype=torch.bfloat16, bias=bias.to(DEV),
                   epilogue=L.EPI_BIAS | L.EPI_GELU | L.EPI_GELU_DERIV, aux_out=auxd)
    ydgd = gemm(xd, wd, out_dtype=torch.bfloat16, epilogue=L.EPI_DGELU | L.EPI_GELU_DERIV, aux=auxd)
    csd = torch.empty(N, device=DEV)
    ydcd = gemm(xd, wd, out_dtype=torch.bfloat16, epilogue=L.EPI_DGELU | L.EPI_GELU_DERIV, aux=auxd,
                    colsum_out=csd)
    torch.cuda.synchronize()
    pre = base + bias
    assert (y0.cpu() - base).abs().max() < tol
    assert (y0b.float().cpu() - base).abs().max() < tol + 0.01 * base.abs().max()
    assert (yb.float().cpu() - pre).abs().max() < tol + 0.01 * pre.abs().max()
    assert (yr.cpu() - (pre + res)).abs().max() < tol
    assert (aux.float().cpu() - pre).abs().max() < tol + 0.01 * pre.abs().max()
    assert (yg.float().cpu() - F.gelu(pre)).abs().max() < tol + 0.01 * pre.abs().max()
    xa = aux.float().cpu().requires_grad_(True)
    F.gelu(xa).sum().backward()
    assert (ydg.float().cpu() - base * xa.grad).abs().max() < tol + 0.01 * base.abs().max()
    keep = torch.from_numpy(O.dropout_keep(seed, np.arange(M)[:, None], np.arange(N)[None, :], p))
    ref = res + torch.where(keep, pre / (1 - p), torch.zeros(()))
    assert (ydr.cpu() - ref).abs().max() < tol
    assert (yac.cpu() - (acc0 + 0.5 * base)).abs().max() < tol
    ref_dg = base * xa.grad
    assert (ydc.float().cpu() - ref_dg).abs().max() < tol + 0.01 * base.abs().max()
    assert (cs.cpu() - ref_dg.sum(0)).abs().max() < 1e-2 * (1 + ref_dg.abs().sum(0).max())
    # derivative-storing GELU pair
    xp = pre.clone().requires_grad_(True)
    F.gelu(xp).sum().backward()
    assert (auxd.float().cpu() - xp.grad).abs().max() < 0.01 + 0.01 * tol
    assert (ygd.float().cpu() - F.gelu(pre)).abs().max() < tol + 0.01 * pre.abs().max()
    ref_dgd = base * auxd.float().cpu()
    assert (ydgd.float().cpu() - ref_dgd).abs().max() < tol + 0.01 * base.abs().max()
    assert torch.equal(ydcd.cpu(), ydgd.cpu())
    assert (csd.cpu() - ref_dgd.sum(0)).abs().max() < 1e-2 * (1 + ref_dgd.abs().sum(0).max())


@pytest.mark.parametrize("dtype,pers", [(torch.float32, 1), (torch.bfloat16, 0), (torch.bfloat16, 1)])
def test_gemm_colsum_epilogue(dtype, pers):
    """CG_EPI_COLSUM (fused bias-gradient column sums) on the persistent tile and on the
    unfused fallback (fp32 kernel / persistent tile disabled) against torch."""
    ops = _ops()
    L = __import__("codonlm_amd._lib", fromlist=["x"])
    M, N, K = 700, 264, 192
    g = torch.Generator().manual_seed(11)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) * 0.1
    base = (_bf(x) @ _bf(w).t()) if dtype == torch.bfloat16 else x @ w.t()
    cs = torch.empty(N, device=DEV)
    y = ops.gemm(x.to(DEV, dtype), w.to(DEV, dtype), out_dtype=dtype, colsum_out=cs,
                 tile=L.TILE_AUTO if pers else L.TILE_VEC)
    torch.cuda.synchronize()
    tol = 1e-3 if dtype == torch.float32 else 2e-2
    assert (y.float().cpu() - base).abs().max() < tol * 4 * (1 + base.abs().max())
    assert (cs.cpu() - base.sum(0)).abs().max() < tol * (1 + base.abs().sum(0).max())


@pytest.mark.parametrize("max_wg", [0, 4, 7, 12, 16])
@pytest.mark.parametrize("tile", ["pers", "lw"])
def test_gemm_colsum_multi_tile_walk(max_wg, tile):
    """Column sums carried across a persistent block's tiles (the 8-wave kernel sums consecutive
    tiles of one column block in registers and writes zero partials for the others): grid caps
    that divide the 4 column tiles (4, 12, 16: every block walks one column block), that do not
    (7: the column block changes along the walk) and the full grid, with the dGELU epilogue of
    the fc2 dX product; M = 2000 leaves a ragged last row tile."""
    ops = _ops()
    L = __import__("codonlm_amd._lib", fromlist=["x"])
    M, N, K = 2000, 512, 256
    g = torch.Generator().manual_seed(12)
    x, w = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.1
    aux = (torch.rand(M, N, generator=g) * 1.2).to(torch.bfloat16)
    base = (_bf(x) @ _bf(w).t()) * aux.float()
    cs = torch.empty(N, device=DEV)
    t = {"pers": L.TILE_PERS, "lw": L.TILE_PERS_LW}[tile]
    y = ops.gemm(x.to(DEV, torch.bfloat16), w.to(DEV, torch.bfloat16), out_dtype=torch.bfloat16, colsum_out=cs,
                 epilogue=L.EPI_DGELU | L.EPI_GELU_DERIV, aux=aux.to(DEV), tile=t, max_wg=max_wg)
    torch.cuda.synchronize()
    ref = y.float().cpu().sum(0)  # (the sums are of the fp32 values before the bf16 store)
    assert (y.float().cpu() - base).abs().max() < 2e-2 * (1 + base.abs().max())
    assert (cs.cpu() - base.sum(0)).abs().max() < 2e-2 * (1 + base.abs().sum(0).max())
    assert (cs.cpu() - ref).abs().max() < 1e-2 * (1 + base.abs().sum(0).max())


@pytest.mark.parametrize("cap", [1, 3])
@pytest.mark.parametrize("M,K,T,H,KV,hd,extra", [(16384, 384, 512, 8, 4, 48, 0), (700, 128, 77, 4, 2, 32, 0),
                                                 (513, 256, 513, 2, 1, 64, 64), (300, 128, 100, 1, 1, 48, 0),
                                                 (2048, 512, 1024, 8, 8, 64, 0)])
def test_gemm_rope_epilogue(cap, M, K, T, H, KV, hd, extra):
    """CG_EPI_ROPE (the qkv projection with RoPE fused into the loader-wave tile's epilogue,
    model_tiny_gpt.py:85-93): B rows fed in rotation-pair order so each lane holds dims i and
    i + hd/2 of one head, rotated after the bias at position m % T.  Against fp32 torch of the same
    bf16 operands (rel-L2 <= 4e-3: one bf16 rounding), against the bias-only GEMM + cg_rope_tab pass
    (<= 1e-2: that one rounds twice), and the V columns (and `extra` columns past them) against the
    bias-only GEMM (unrotated: within one bf16 ulp).  Shapes: C3 (hd48, N 768), hd32, hd64 with
    N % 64 != 0 rows of pair units, one head pair with N = 144 (a 64-column block half past N), C4
    geometry; cap = 3 workgroups each walk many tiles (the per-tile B-row order)."""
    ops = _ops()
    L = __import__("codonlm_amd._lib", fromlist=["x"])
    g = torch.Generator().manual_seed(M + hd + extra)
    N = (H + 2 * KV) * hd + extra
    x = _bf(torch.randn(M, K, generator=g))
    w = _bf(torch.randn(N, K, generator=g) * K ** -0.5)
    bias = torch.randn(N, generator=g)
    cos, sin = _rope_tabs(T, hd)
    ref = x @ w.t() + bias
    nq = (H + KV) * hd
    pos = torch.arange(M) % T
    rh = ref[:, :nq].view(M, H + KV, hd)
    a, b = rh[..., :hd // 2], rh[..., hd // 2:]
    c, s = cos[pos][:, None, :], sin[pos][:, None, :]
    ref_rot = torch.cat([torch.cat([a * c - b * s, b * c + a * s], -1).reshape(M, nq), ref[:, nq:]], 1)
    xd, wd, bd = x.to(DEV, torch.bfloat16), w.to(DEV, torch.bfloat16), bias.to(DEV)
    cd, sd = cos.to(DEV), sin.to(DEV)
    mw = cap if cap > 1 else 0
    fused = ops.gemm(xd, wd, out_dtype=torch.bfloat16, bias=bd, epilogue=L.EPI_BIAS, rope=(cd, sd, T, hd, H + KV),
                     max_wg=mw)
    plain = ops.gemm(xd, wd, out_dtype=torch.bfloat16, bias=bd, epilogue=L.EPI_BIAS, max_wg=mw)
    unf = plain.clone()
    if M % T == 0:
        ops.rope_(unf, M // T, T, H, KV, hd, cd, sd)
    torch.cuda.synchronize()
    ff = fused.float().cpu()

    def rel(u, v):
        return float((u.double() - v.double()).norm() / v.double().norm())
    assert rel(ff, ref_rot) <= 4e-3, rel(ff, ref_rot)
    assert rel(ff[:, :nq], ref_rot[:, :nq]) <= 4e-3
    if M % T == 0:
        assert rel(ff, unf.float().cpu()) <= 1e-2
    pv = plain.float().cpu()[:, nq:]
    assert torch.allclose(ff[:, nq:], pv, rtol=2 ** -7, atol=1e-6), (ff[:, nq:] - pv).abs().max()


def test_gemm_rope_epilogue_unsupported():
    """CG_EPI_ROPE outside the loader-wave tile is CG_EUNSUPPORTED (the engine then keeps the
    cg_rope_tab pass): fp32 operands, hd % 16 != 0, the eight-wave kernel forced."""
    ops = _ops()
    L = __import__("codonlm_amd._lib", fromlist=["x"])
    cos, sin = _rope_tabs(64, 40)
    x = torch.randn(256, 128, device=DEV)
    w = torch.randn(3 * 40 * 4, 128, device=DEV)
    with pytest.raises(ValueError, match="CG_EUNSUPPORTED"):
        ops.gemm(x, w, rope=(cos.to(DEV), sin.to(DEV), 64, 40, 8))
    xb, wb = x.bfloat16(), w.bfloat16()
    with pytest.raises(ValueError, match="CG_EUNSUPPORTED"):
        ops.gemm(xb, wb, rope=(cos.to(DEV), sin.to(DEV), 64, 40, 8))
    c2, s2 = _rope_tabs(64, 32)
    with pytest.raises(ValueError, match="CG_EUNSUPPORTED"):
        ops.gemm(xb, wb[:256], rope=(c2.to(DEV), s2.to(DEV), 64, 32, 4), tile=L.TILE_PERS)


@pytest.mark.parametrize("B,T,H,KV,hd,window,p", [(2, 1024, 8, 8, 64, 0, 0.1), (2, 512, 8, 4, 48, 0, 0.0),
                                                   (2, 300, 4, 2, 32, 0, 0.1), (1, 257, 4, 1, 24, 37, 0.2),
                                                   (2, 130, 2, 2, 8, 0, 0.0)])
def test_attention_bwd_f32mfma_vs_fp64(B, T, H, KV, hd, window, p):
    """The fp32 attention backward on v_mfma_f32_32x32x2_f32 (attention_f32.h; the reference's own
    fp32 GPU training, loop.py:498; the vector kernels where the head dim is not 32 / 48 / 64)
    against fp64 autograd of the same masked, dropped-out attention (the oracle's mask and keep
    bits): dQ / dK / dV agree to rel <= 2e-5 of each block's scale.  Covers C4 / C3 geometry, GQA,
    a local window, odd head dims (24, 8), ragged T and dropout keep bits."""
    ops = _ops()
    g = torch.Generator().manual_seed(T * 7 + hd)
    N = (H + 2 * KV) * hd
    qkv = torch.randn(B * T, N, generator=g)
    idx = torch.randint(4, 68, (B, T), generator=g)
    idx[0, T // 3] = 3
    idx[-1, T // 2] = 3
    drop = None
    if p > 0:
        keep = O.dropout_keep(31, np.arange(B * H * T)[:, None], np.arange(T)[None, :], p)
        drop = torch.from_numpy(keep.astype(np.float64) / (1 - p)).view(B, H, T, T)
    seg = ops.segment_starts(idx.to(DEV), 3)
    qd = qkv.to(DEV)
    y, lse = ops.attn_fwd(qd, seg, B, T, H, KV, hd, window=window, drop_seed=31, drop_p=p)
    dy = torch.randn(B * T, H * hd, generator=g)
    got = ops.attn_bwd(qd, seg, y, dy.to(DEV), lse, B, T, H, KV, hd, window=window, drop_seed=31, drop_p=p).cpu()
    qr = qkv.double().requires_grad_(True)
    _attn_ref(qr, idx, B, T, H, KV, hd, 3, window or None, drop).backward(dy.double())
    ref = qr.grad
    for name, sl in (("dq", slice(0, H * hd)), ("dk", slice(H * hd, (H + KV) * hd)),
                     ("dv", slice((H + KV) * hd, N))):
        a, r = got[:, sl].double(), ref[:, sl]
        err = float((a - r).abs().max() / r.abs().max())
        assert err <= 2e-5, (name, err)
