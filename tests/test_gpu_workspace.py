"""Workspace contract of the C-ABI (`void* workspace, size_t ws_bytes`).

Every entry point that takes scratch memory also takes its size and returns CG_EINVAL
(-> ValueError) when it is short, instead of writing past it (the round-2 embedding-backward
fault: a kernel variant wrote more row chunks than its caller had allocated).  Here each
op runs with EXACTLY the queried number of bytes followed by a sentinel guard region, at the
C1-C5 token geometries and at a ragged B*T, and the guard must come back untouched: the
cg_*_workspace queries cover what the kernels write.  One byte less must be refused.
The whole-model workspace (cg_model_workspace_bytes) gets the same guard check over a
training step with dropout at a ragged B*T.
"""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
GUARD = 4096  # bytes of sentinel after each workspace
SENT = 0x7FC0DEAD  # a NaN bit pattern no kernel writes

# (d, H, hidden, Nqkv) of C1..C5 and the (B, T) shapes: the config's own and a ragged one
GEOS = {"C1": (128, 2, 512, 384), "C2": (256, 4, 1024, 768), "C3": (384, 8, 2048, 768),
        "C4": (512, 8, 2048, 1536), "C5": (384, 8, 1536, 1152)}
SHAPES = {"C1": [(4, 512), (3, 170)], "C2": [(8, 512), (3, 170)], "C3": [(8, 512), (3, 170)],
          "C4": [(4, 1024), (3, 341)], "C5": [(8, 512), (5, 99)]}
CASES = [(n, B, T) for n in sorted(GEOS) for (B, T) in SHAPES[n]]


def _lib():
    from codonlm_amd import _lib as L
    return L


class Guarded:
    """`nbytes` of workspace followed by GUARD sentinel bytes."""

    def __init__(self, nbytes):
        self.n = int(nbytes)
        words = (self.n + 3) // 4 + GUARD // 4
        self.buf = torch.full((words,), SENT, dtype=torch.int32, device=DEV)
        self.ptr = self.buf.data_ptr()

    def intact(self):
        torch.cuda.synchronize()
        return bool((self.buf[(self.n + 3) // 4:] == SENT).all())


def _st():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("name,B,T", CASES)
def test_op_workspaces_cover_kernel_writes(name, B, T):
    L = _lib()
    lib = L.lib
    d, H, hid, Nqkv = GEOS[name]
    M = B * T
    V = 68
    g = torch.Generator(device=DEV).manual_seed(M)
    st = _st()

    # -- column sums (bias gradients): every column count the engine uses
    for cols in sorted({d, Nqkv, hid}):
        x = torch.randn(M, cols, device=DEV, generator=g).to(torch.bfloat16)
        need = int(lib.cg_colsum_workspace(M, cols))
        out = torch.empty(cols, device=DEV)
        ws = Guarded(need)
        assert lib.cg_colsum(L.CG_BF16, x.data_ptr(), cols, M, cols, out.data_ptr(), 0, ws.ptr, need, st) == 0
        assert ws.intact(), ("colsum", cols)
        torch.testing.assert_close(out, x.float().sum(0), rtol=1e-3, atol=1e-2)
        assert lib.cg_colsum(L.CG_BF16, x.data_ptr(), cols, M, cols, out.data_ptr(), 0, ws.ptr, need - 1, st) == -1
        npart = C.c_int(0)
        ws = Guarded(need)
        assert lib.cg_colsum_partials(L.CG_BF16, x.data_ptr(), cols, M, cols, ws.ptr, need, C.byref(npart), st) == 0
        assert ws.intact() and npart.value * cols * 4 <= need
        assert lib.cg_colsum_partials(L.CG_BF16, x.data_ptr(), cols, M, cols, ws.ptr, need - 1, C.byref(npart),
                                      st) == -1

    # -- LayerNorm backward partials (with and without the consumer column sums)
    x = torch.randn(M, d, device=DEV, generator=g)
    w = torch.randn(d, device=DEV, generator=g)
    mean, rstd = x.mean(1), torch.rsqrt(x.var(1, unbiased=False) + 1e-5)
    dy = torch.randn(M, d, device=DEV, generator=g).to(torch.bfloat16)
    gout = torch.empty(M, d, device=DEV)
    branch = torch.empty(M, d, dtype=torch.bfloat16, device=DEV)
    dg, db, dc = (torch.empty(d, device=DEV) for _ in range(3))
    for want in (0, 1):
        need = int(lib.cg_layernorm_bwd_workspace(M, d, want))
        ws = Guarded(need)
        rc = lib.cg_layernorm_bwd(L.CG_BF16, dy.data_ptr(), d, x.data_ptr(), d, mean.data_ptr(), rstd.data_ptr(),
                                  w.data_ptr(), None, gout.data_ptr(), L.CG_BF16, branch.data_ptr(), 7, 0.1,
                                  ws.ptr, need, dg.data_ptr(), db.data_ptr(), dc.data_ptr() if want else None, 0,
                                  M, d, 1e-5, st)
        assert rc == 0 and ws.intact(), ("layernorm_bwd", want)
        assert lib.cg_layernorm_bwd(L.CG_BF16, dy.data_ptr(), d, x.data_ptr(), d, mean.data_ptr(), rstd.data_ptr(),
                                    w.data_ptr(), None, gout.data_ptr(), L.CG_BF16, branch.data_ptr(), 7, 0.1,
                                    ws.ptr, need - 1, dg.data_ptr(), db.data_ptr(), dc.data_ptr() if want else None,
                                    0, M, d, 1e-5, st) == -1
        ws = Guarded(need)
        rc = lib.cg_layernorm_bwd_partials(L.CG_BF16, dy.data_ptr(), d, x.data_ptr(), d, mean.data_ptr(),
                                           rstd.data_ptr(), w.data_ptr(), gout.data_ptr(), gout.data_ptr(),
                                           L.CG_BF16, branch.data_ptr(), 7, 0.1, ws.ptr, need, want, M, d, st)
        assert rc == 0 and ws.intact(), ("layernorm_bwd_partials", want)

    # -- cross-entropy (split-bf16 dlogits, the engine's layout)
    Vp = 80
    logits = torch.randn(M, Vp, device=DEV, generator=g) * 4
    tg = torch.randint(0, V, (M,), device=DEV, generator=g)
    dl = torch.empty(M, 2 * Vp, dtype=torch.bfloat16, device=DEV)
    loss = torch.empty((), device=DEV)
    need = int(lib.cg_ce_workspace(M))
    ws = Guarded(need)
    assert lib.cg_cross_entropy(logits.data_ptr(), Vp, tg.data_ptr(), M, V, 0.05, None, 0, 1.0, L.CG_BF16X2,
                                dl.data_ptr(), 2 * Vp, loss.data_ptr(), ws.ptr, need, st) == 0
    assert ws.intact(), "cross_entropy"
    assert lib.cg_cross_entropy(logits.data_ptr(), Vp, tg.data_ptr(), M, V, 0.05, None, 0, 1.0, L.CG_BF16X2,
                                dl.data_ptr(), 2 * Vp, loss.data_ptr(), ws.ptr, need - 1, st) == -1

    # -- embedding backward (token and position rows)
    idx = torch.randint(0, V, (B, T), device=DEV, generator=g)
    gr = torch.randn(M, d, device=DEV, generator=g)
    dtok = torch.empty(V, d, device=DEV)
    need = int(lib.cg_embed_bwd_workspace(B, T, V, d))
    ws = Guarded(need)
    assert lib.cg_embed_bwd(idx.data_ptr(), gr.data_ptr(), dtok.data_ptr(), None, B, T, V, d, 3, 0.1, 0, ws.ptr,
                            need, st) == 0
    assert ws.intact(), "embed_bwd"
    assert lib.cg_embed_bwd(idx.data_ptr(), gr.data_ptr(), dtok.data_ptr(), None, B, T, V, d, 3, 0.1, 0, ws.ptr,
                            need - 1, st) == -1

    # -- attention backward (delta rows)
    hd = d // H
    qkv = (torch.randn(M, 3 * d, device=DEV, generator=g) * 0.5).to(torch.bfloat16)
    seg = torch.zeros(B, T, dtype=torch.int32, device=DEV)
    y = torch.empty(M, d, dtype=torch.bfloat16, device=DEV)
    lse = torch.empty(B * H * T, device=DEV)
    assert lib.cg_attn_fwd(L.CG_BF16, qkv.data_ptr(), 3 * d, seg.data_ptr(), y.data_ptr(), d, lse.data_ptr(), B, T,
                           H, H, hd, 0, 0, 0.0, None, st) == 0
    dyy = torch.randn(M, d, device=DEV, generator=g).to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    need = int(lib.cg_attn_bwd_workspace(B, T, H))
    ws = Guarded(need)
    assert lib.cg_attn_bwd(L.CG_BF16, qkv.data_ptr(), 3 * d, seg.data_ptr(), y.data_ptr(), d, dyy.data_ptr(), d,
                           lse.data_ptr(), dqkv.data_ptr(), 3 * d, B, T, H, H, hd, 0, 0, 0.0, None, None, 0, ws.ptr,
                           need, st) == 0
    assert ws.intact(), "attn_bwd"
    assert lib.cg_attn_bwd(L.CG_BF16, qkv.data_ptr(), 3 * d, seg.data_ptr(), y.data_ptr(), d, dyy.data_ptr(), d,
                           lse.data_ptr(), dqkv.data_ptr(), 3 * d, B, T, H, H, hd, 0, 0, 0.0, None, None, 0, ws.ptr,
                           need - 1, st) == -1


@pytest.mark.parametrize("name,B,T", CASES)
def test_gemm_workspaces_cover_kernel_writes(name, B, T):
    """Split-K slabs (split_k * M * N floats) and the fused bias-gradient column-sum partials
    (ceil(M/64) * N floats) of cg_gemm, sized by ws_bytes."""
    L = _lib()
    d, H, hid, Nqkv = GEOS[name]
    M = B * T
    g = torch.Generator(device=DEV).manual_seed(M + 1)
    a = torch.randn(M, hid, device=DEV, generator=g).to(torch.bfloat16)
    bmat = torch.randn(d, hid, device=DEV, generator=g).to(torch.bfloat16)
    # dX-shaped product with the COLSUM epilogue
    need = ((M + 63) // 64) * d * 4
    ws = Guarded(need)
    out = torch.empty(M, d, dtype=torch.bfloat16, device=DEV)
    dsc = L.GemmDesc()
    dsc.in_dtype = dsc.c_dtype = L.CG_BF16
    dsc.M, dsc.N, dsc.K = M, d, hid
    dsc.A, dsc.lda, dsc.a_kcontig = a.data_ptr(), hid, 1
    dsc.B, dsc.ldb, dsc.b_kcontig = bmat.data_ptr(), hid, 1
    dsc.C, dsc.ldc = out.data_ptr(), d
    dsc.epilogue, dsc.alpha, dsc.split_k = L.EPI_COLSUM, 1.0, 1
    dsc.workspace, dsc.ws_bytes = ws.ptr, need
    assert L.lib.cg_gemm(C.byref(dsc), _st()) == 0
    assert ws.intact(), "gemm colsum"
    dsc.ws_bytes = need - 1
    assert L.lib.cg_gemm(C.byref(dsc), _st()) == -1
    # dW-shaped split-K product (fp32 out, MN-contiguous operands, K = M tokens)
    split = 4
    need = split * d * hid * 4
    ws = Guarded(need)
    dw = torch.empty(d, hid, device=DEV)
    dy = torch.randn(M, d, device=DEV, generator=g).to(torch.bfloat16)
    dsc = L.GemmDesc()
    dsc.in_dtype, dsc.c_dtype = L.CG_BF16, L.CG_F32
    dsc.M, dsc.N, dsc.K = d, hid, M
    dsc.A, dsc.lda, dsc.a_kcontig = dy.data_ptr(), d, 0
    dsc.B, dsc.ldb, dsc.b_kcontig = a.data_ptr(), hid, 0
    dsc.C, dsc.ldc = dw.data_ptr(), hid
    dsc.alpha, dsc.split_k = 1.0, split
    dsc.workspace, dsc.ws_bytes = ws.ptr, need
    assert L.lib.cg_gemm(C.byref(dsc), _st()) == 0
    assert ws.intact(), "gemm split-K"
    torch.testing.assert_close(dw, dy.float().t() @ a.float(), rtol=2e-3, atol=2e-2 * (M ** 0.5))
    dsc.ws_bytes = need - 1
    assert L.lib.cg_gemm(C.byref(dsc), _st()) == -1


@pytest.mark.parametrize("name,B,T", [("C4", 3, 341), ("C3", 3, 170), ("C5", 5, 99)])
def test_model_workspace_covers_training_step(name, B, T):
    """cg_model_workspace_bytes covers every write of a bf16 training step with dropout (keep-bit
    arrays, grouped-dW slots, aux heads) at a ragged B*T: the engine's workspace is handed over
    with a sentinel guard behind the queried size."""
    from codonlm_amd import TinyGPT
    L = _lib()
    d, H, _, _ = GEOS[name]
    kw = dict(n_layer={"C3": 10, "C4": 12, "C5": 10}[name], n_head=H, n_embd=d, dropout=0.1,
              compute_dtype="bf16", device=DEV)
    if name == "C3":
        kw.update(n_kv_head=4, use_rope=True, use_swiglu=True)
    if name == "C5":
        kw.update(termination_aux=True, multi_offset_targets=[2, 4, 8, 16, 32])
    torch.manual_seed(0)
    m = TinyGPT(68, {"C3": 512, "C4": 1024, "C5": 512}[name], **kw)
    m.train()
    eng = m.engine
    need = int(L.lib.cg_model_workspace_bytes(C.byref(eng.model.cfg), B, T))
    buf = torch.full((need + GUARD,), 0xA5, dtype=torch.uint8, device=DEV)
    eng.workspace, eng._ws_key = buf, None
    x = torch.randint(4, 68, (B, T), device=DEV)
    y = torch.randint(4, 68, (B, T), device=DEV)
    if name == "C5":
        from codonlm_amd.training import objectives as obj
        logits, loss, aux = m(x, y, return_aux=True)
        off, _ = obj.multi_offset_lm_loss(aux["offset_logits"], y, {k: 0.2 for k in (2, 4, 8, 16, 32)})
        lab = obj.termination_distance_bucket_labels(y, stop_ids=(2,))
        total = loss + off + 0.1 * obj.termination_aux_loss(aux["termination_logits"], lab)
    else:
        logits, total = m(x, y)
    total.backward()
    torch.cuda.synchronize()
    assert eng.workspace.data_ptr() == buf.data_ptr(), "engine re-allocated its workspace"
    assert bool((buf[need:] == 0xA5).all()), name
    assert torch.isfinite(total).item()
