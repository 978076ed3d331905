"""Tensor-level wrappers over the op entry points of libcodonlm_hip.so.

Each wrapper validates shapes, allocates outputs with torch on the tensor's device and
launches on the current HIP stream.  These are the building blocks the engine uses
natively; they are exposed for op-level parity tests and for callers that compose
their own step (e.g. the auxiliary heads).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L

_DT = {torch.float32: L.CG_F32, torch.bfloat16: L.CG_BF16}


def _dt(t: torch.Tensor) -> int:
    if t.dtype not in _DT:
        raise ValueError(f"unsupported dtype {t.dtype}")
    return _DT[t.dtype]


def _p(t):
    return None if t is None else t.data_ptr()


def gemm(a, b, *, a_kcontig=True, b_kcontig=True, M=None, N=None, K=None, out=None, out_dtype=None,
         bias=None, resid=None, epilogue=0, aux=None, aux_out=None, alpha=1.0, drop_seed=0, drop_p=0.0,
         split_k=1, colsum_out=None, n_valid=0, rope=None, tile=0, max_wg=0):
    """C[m,n] = epi(alpha * sum_k A(m,k) B(n,k)); A(m,k)=a[m,k] if a_kcontig else a[k,m]; same for B.
    colsum_out (fp32 [N]): also the column sums of C (CG_EPI_COLSUM partials + cg_colsum_reduce).
    rope = (cos, sin, T, hd, heads): CG_EPI_ROPE -- the first heads*hd columns rotated at position
    m % T after the bias (tables fp32 [>= T][hd/2]).  tile: L.TILE_* (0 = automatic); max_wg: cap
    on the persistent grid (0 = one workgroup per CU)."""
    for t in (a, b):
        L.require_device(t, "gemm")
    if a.dtype != b.dtype:
        raise ValueError("a and b must share a dtype")
    if M is None:
        M = a.shape[0] if a_kcontig else a.shape[1]
    if K is None:
        K = a.shape[1] if a_kcontig else a.shape[0]
    if N is None:
        N = b.shape[0] if b_kcontig else b.shape[1]
    out_dtype = out_dtype or (out.dtype if out is not None else a.dtype)
    if out is None:
        out = torch.empty(M, N, dtype=out_dtype, device=a.device)
    ws = None
    if split_k > 1:
        ws = torch.empty(split_k * M * N, dtype=torch.float32, device=a.device)
    if colsum_out is not None:
        if split_k > 1:
            raise ValueError("colsum_out needs split_k == 1")
        epilogue = int(epilogue) | L.EPI_COLSUM
        ws = torch.empty(((M + 63) // 64) * N, dtype=torch.float32, device=a.device)
    d = L.GemmDesc()
    d.in_dtype, d.c_dtype = _dt(a), _dt(out)
    d.M, d.N, d.K = M, N, K
    d.A, d.lda, d.a_kcontig = a.data_ptr(), a.stride(0), int(a_kcontig)
    d.B, d.ldb, d.b_kcontig = b.data_ptr(), b.stride(0), int(b_kcontig)
    d.C, d.ldc = out.data_ptr(), out.stride(0)
    d.epilogue = int(epilogue)
    d.alpha = float(alpha)
    d.bias = _p(bias)
    d.resid, d.ldr = _p(resid), (resid.stride(0) if resid is not None else 0)
    d.aux = _p(aux)
    d.aux_out = _p(aux_out)
    aux_t = aux if aux is not None else aux_out
    d.ld_aux = aux_t.stride(0) if aux_t is not None else 0
    d.drop_seed, d.drop_p = int(drop_seed) & 0xFFFFFFFF, float(drop_p)
    d.split_k, d.workspace = int(split_k), _p(ws)
    d.ws_bytes = 0 if ws is None else ws.numel() * ws.element_size()
    d.n_valid = int(n_valid)
    d.tile, d.max_wg = int(tile), int(max_wg)
    if rope is not None:
        cos, sin, rT, rhd, rheads = rope
        d.epilogue |= L.EPI_ROPE
        d.rope_cos, d.rope_sin = cos.data_ptr(), sin.data_ptr()
        d.rope_T, d.rope_hd, d.rope_heads = int(rT), int(rhd), int(rheads)
    L.check(L.lib.cg_gemm(C.byref(d), L.stream_ptr(a.device)), "cg_gemm")
    if colsum_out is not None:
        L.check(L.lib.cg_colsum_reduce(ws.data_ptr(), (M + 63) // 64, N, colsum_out.data_ptr(), 0,
                                       L.stream_ptr(a.device)), "cg_colsum_reduce")
    return out


def layernorm_fwd(x, weight, bias, out_dtype=torch.float32, eps=1e-5):
    L.require_device(x, "layernorm_fwd")
    rows, cols = x.shape
    y = torch.empty(rows, cols, dtype=out_dtype, device=x.device)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty_like(mean)
    L.check(L.lib.cg_layernorm_fwd(_dt(y), x.data_ptr(), x.stride(0), weight.data_ptr(), bias.data_ptr(),
                                   y.data_ptr(), y.stride(0), mean.data_ptr(), rstd.data_ptr(), rows, cols, eps,
                                   L.stream_ptr(x.device)), "cg_layernorm_fwd")
    return y, mean, rstd


def layernorm_fwd_mask(x, weight, bias, B, T, H, drop_seed, drop_p, out_dtype=torch.bfloat16, eps=1e-5):
    """cg_layernorm_fwd_mask: layernorm_fwd and the attention-dropout keep words (attn_drop_mask) in one
    launch -> (y, mean, rstd, mask)."""
    L.require_device(x, "layernorm_fwd_mask")
    rows, cols = x.shape
    y = torch.empty(rows, cols, dtype=out_dtype, device=x.device)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty_like(mean)
    n = int(L.lib.cg_attn_drop_mask_bytes(B, T, H))
    mask = torch.zeros(max(n, 4) // 4, dtype=torch.int32, device=x.device)
    L.check(L.lib.cg_layernorm_fwd_mask(_dt(y), x.data_ptr(), x.stride(0), weight.data_ptr(), bias.data_ptr(),
                                        y.data_ptr(), y.stride(0), mean.data_ptr(), rstd.data_ptr(), rows, cols, eps,
                                        B, T, H, int(drop_seed) & 0xFFFFFFFF, float(drop_p), mask.data_ptr(),
                                        L.stream_ptr(x.device)), "cg_layernorm_fwd_mask")
    return y, mean, rstd, mask


def layernorm_bwd(dy, x, mean, rstd, weight, g_in=None, eps=1e-5, branch_dtype=None, drop_seed=0, drop_p=0.0):
    """LayerNorm backward.  With `branch_dtype`, also returns the consumer-branch copy of g_out
    (dropout-masked with (drop_seed, drop_p)) and its column sums (the producing Linear's bias grad):
    (g_out, dgamma, dbeta, g_branch, colsum); else (g_out, dgamma, dbeta)."""
    rows, cols = x.shape
    g_out = torch.empty(rows, cols, dtype=torch.float32, device=x.device)
    part_bytes = int(L.lib.cg_layernorm_bwd_workspace(rows, cols, 1))
    part = torch.empty(max(1, part_bytes // 4), dtype=torch.float32, device=x.device)
    dgamma = torch.empty(cols, dtype=torch.float32, device=x.device)
    dbeta = torch.empty_like(dgamma)
    branch = colsum = None
    if branch_dtype is not None:
        branch = torch.empty(rows, cols, dtype=branch_dtype, device=x.device)
        colsum = torch.empty_like(dgamma)
    L.check(L.lib.cg_layernorm_bwd(_dt(dy), dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), mean.data_ptr(),
                                   rstd.data_ptr(), weight.data_ptr(), _p(g_in), g_out.data_ptr(),
                                   _dt(branch) if branch is not None else L.CG_F32, _p(branch), drop_seed, drop_p,
                                   part.data_ptr(), part_bytes, dgamma.data_ptr(), dbeta.data_ptr(), _p(colsum), 0,
                                   rows, cols,
                                   eps, L.stream_ptr(x.device)), "cg_layernorm_bwd")
    if branch_dtype is not None:
        return g_out, dgamma, dbeta, branch, colsum
    return g_out, dgamma, dbeta


def layernorm_bwd_partials(dy, x, mean, rstd, weight, g_in=None, branch_dtype=None, drop_seed=0, drop_p=0.0):
    """LayerNorm backward row pass without the parameter reduction (cg_layernorm_bwd_partials):
    returns (g_out, partials [nblk][(2 + want_col) * cols], branch or None)."""
    rows, cols = x.shape
    g_out = torch.empty(rows, cols, dtype=torch.float32, device=x.device)
    nblk = L.lib.cg_layernorm_bwd_blocks(rows)
    nw = 3 if branch_dtype is not None else 2
    part = torch.empty(nblk, nw * cols, dtype=torch.float32, device=x.device)
    branch = torch.empty(rows, cols, dtype=branch_dtype, device=x.device) if branch_dtype is not None else None
    L.check(L.lib.cg_layernorm_bwd_partials(_dt(dy), dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0),
                                            mean.data_ptr(), rstd.data_ptr(), weight.data_ptr(), _p(g_in),
                                            g_out.data_ptr(), _dt(branch) if branch is not None else L.CG_F32,
                                            _p(branch), drop_seed, drop_p, part.data_ptr(),
                                            part.numel() * 4, int(nw == 3), rows, cols,
                                            L.stream_ptr(x.device)), "cg_layernorm_bwd_partials")
    return g_out, part, branch


def reduce_columns(jobs):
    """One cg_reduce_columns launch over jobs = [(part 2-D fp32 view, dst fp32 [cols], accumulate)]:
    dst (+)= part.sum(0) in the kernel's fixed order."""
    bt = L.ReduceBatch()
    bt.n = len(jobs)
    dev = None
    for i, (part, dst, acc) in enumerate(jobs):
        j = bt.j[i]
        j.part = part.data_ptr(); j.ld = part.stride(0); j.nrows = part.shape[0]; j.cols = part.shape[1]
        j.dst = dst.data_ptr(); j.accumulate = int(acc)
        dev = part.device
    L.check(L.lib.cg_reduce_columns(C.byref(bt), L.stream_ptr(dev) if dev is not None else None),
            "cg_reduce_columns")


def swiglu_fwd(gu, H):
    """s[:, j] = silu(gu[:, j]) * gu[:, Hp + j] for j < H (0 for H <= j < Hp), Hp = gu.shape[1] // 2."""
    rows, Hp = gu.shape[0], gu.shape[1] // 2
    s = torch.empty(rows, Hp, dtype=gu.dtype, device=gu.device)
    L.check(L.lib.cg_swiglu_fwd(_dt(gu), gu.data_ptr(), gu.stride(0), Hp, s.data_ptr(), s.stride(0), rows, H,
                                L.stream_ptr(gu.device)), "cg_swiglu_fwd")
    return s


def swiglu_bwd(gu, ds, H):
    """d(gate | up) of swiglu_fwd for the upstream gradient ds [rows][Hp]."""
    rows, Hp = gu.shape[0], gu.shape[1] // 2
    dgu = torch.empty_like(gu)
    L.check(L.lib.cg_swiglu_bwd(_dt(gu), gu.data_ptr(), gu.stride(0), Hp, ds.data_ptr(), ds.stride(0),
                                dgu.data_ptr(), dgu.stride(0), rows, H, L.stream_ptr(gu.device)), "cg_swiglu_bwd")
    return dgu


def rope_(qkv, B, T, H, KV, hd, cos_tab, sin_tab, inverse=False):
    """In-place rotate-half RoPE of the q and k heads of qkv [B*T][ld] (cos/sin fp32 [T][hd/2])."""
    L.check(L.lib.cg_rope_tab(_dt(qkv), qkv.data_ptr(), qkv.stride(0), B, T, H, KV, hd, cos_tab.data_ptr(),
                              sin_tab.data_ptr(), int(inverse), L.stream_ptr(qkv.device)), "cg_rope_tab")
    return qkv


def segment_starts(idx, sep_id):
    B, T = idx.shape
    out = torch.empty(B, T, dtype=torch.int32, device=idx.device)
    L.check(L.lib.cg_segment_starts(idx.contiguous().data_ptr(), out.data_ptr(), B, T,
                                    -1 if sep_id is None else int(sep_id), L.stream_ptr(idx.device)),
            "cg_segment_starts")
    return out


def attn_drop_mask(B, T, H, drop_seed, drop_p, device):
    """Attention-dropout keep bits (query-major + key-major words) for cg_attn_fwd / cg_attn_bwd."""
    n = int(L.lib.cg_attn_drop_mask_bytes(B, T, H))
    mask = torch.empty(max(n, 4) // 4, dtype=torch.int32, device=device)
    L.check(L.lib.cg_attn_drop_mask(B, T, H, int(drop_seed) & 0xFFFFFFFF, float(drop_p), mask.data_ptr(),
                                    L.stream_ptr(device)), "cg_attn_drop_mask")
    return mask


def attn_fwd(qkv, segstart, B, T, H, KV, hd, window=0, drop_seed=0, drop_p=0.0, drop_mask=None):
    y = torch.empty(B * T, H * hd, dtype=qkv.dtype, device=qkv.device)
    lse = torch.empty(B * H * T, dtype=torch.float32, device=qkv.device)
    L.check(L.lib.cg_attn_fwd(_dt(qkv), qkv.data_ptr(), qkv.stride(0), _p(segstart), y.data_ptr(), y.stride(0),
                              lse.data_ptr(), B, T, H, KV, hd, int(window or 0), int(drop_seed) & 0xFFFFFFFF,
                              float(drop_p), _p(drop_mask), L.stream_ptr(qkv.device)), "cg_attn_fwd")
    return y, lse


def attn_fwd_keep(qkv, segstart, B, T, H, KV, hd, drop_seed, drop_p, window=0, mask=None):
    """Dropout forward that also writes the keep bits for the backward (cg_attn_fwd_keep): (y, lse, mask).
    `mask` (optional): the cg_attn_drop_mask_bytes buffer to write into."""
    if mask is None:
        n = int(L.lib.cg_attn_drop_mask_bytes(B, T, H))
        mask = torch.zeros(max(n, 4) // 4, dtype=torch.int32, device=qkv.device)
    y = torch.empty(B * T, H * hd, dtype=qkv.dtype, device=qkv.device)
    lse = torch.empty(B * H * T, dtype=torch.float32, device=qkv.device)
    L.check(L.lib.cg_attn_fwd_keep(_dt(qkv), qkv.data_ptr(), qkv.stride(0), _p(segstart), y.data_ptr(), y.stride(0),
                                   lse.data_ptr(), B, T, H, KV, hd, int(window or 0), int(drop_seed) & 0xFFFFFFFF,
                                   float(drop_p), mask.data_ptr(), L.stream_ptr(qkv.device)), "cg_attn_fwd_keep")
    return y, lse, mask


ATTN_BWD_ALGO = {None: 0, "auto": 0, "split": 1, "fused": 2}


def attn_bwd(qkv, segstart, y, dy, lse, B, T, H, KV, hd, window=0, drop_seed=0, drop_p=0.0, drop_mask=None,
             bias_part=None, rope=None, algo=None):
    """dqkv; with bias_part (fp32 [B*ceil(T/128)][ld >= (H+2KV) hd], bf16 MFMA path) also the per-tile
    column sums of dqkv that cg_colsum_reduce turns into the q/k/v bias gradients.  rope = (cos, sin)
    fp32 [T][hd/2] tables: qkv holds rotated q / k and dQ / dK come back w.r.t. the un-rotated ones
    (cg_attn_bwd_rope, bf16 MFMA path).  algo: None / "auto", "split" (dQ kernel + dK/dV kernel) or
    "fused" (one pass, cg_attn_bwd_algo) for the bf16 MFMA backward."""
    dqkv = torch.zeros_like(qkv)
    ws = torch.empty(int(L.lib.cg_attn_bwd_workspace(B, T, H)) // 4 + 1, dtype=torch.float32, device=qkv.device)
    args = [_dt(qkv), qkv.data_ptr(), qkv.stride(0), _p(segstart), y.data_ptr(), y.stride(0), dy.data_ptr(),
            dy.stride(0), lse.data_ptr(), dqkv.data_ptr(), dqkv.stride(0), B, T, H, KV, hd, int(window or 0),
            int(drop_seed) & 0xFFFFFFFF, float(drop_p), _p(drop_mask), _p(bias_part),
            0 if bias_part is None else bias_part.stride(0)]
    tail = [ws.data_ptr(), ws.numel() * 4, L.stream_ptr(qkv.device)]
    if algo is not None:
        rp = [None, None] if rope is None else [rope[0].data_ptr(), rope[1].data_ptr()]
        L.check(L.lib.cg_attn_bwd_algo(ATTN_BWD_ALGO[algo], *args, *rp, *tail), "cg_attn_bwd_algo")
    elif rope is None:
        L.check(L.lib.cg_attn_bwd(*args, *tail), "cg_attn_bwd")
    else:
        L.check(L.lib.cg_attn_bwd_rope(*args, rope[0].data_ptr(), rope[1].data_ptr(), *tail), "cg_attn_bwd_rope")
    return dqkv


def cross_entropy(logits, targets, eps=0.0, weight=None, ignore_index=0, grad_dtype=torch.float32, pad_to=None):
    rows, V = logits.shape
    ldd = pad_to or V
    dl = torch.empty(rows, ldd, dtype=grad_dtype, device=logits.device)
    loss = torch.empty((), dtype=torch.float32, device=logits.device)
    ws = torch.empty(int(L.lib.cg_ce_workspace(rows)) // 4 + 1, dtype=torch.float32, device=logits.device)
    L.check(L.lib.cg_cross_entropy(logits.data_ptr(), logits.stride(0), targets.contiguous().data_ptr(), rows, V,
                                   float(eps), _p(weight), int(ignore_index), 1.0, _dt(dl), dl.data_ptr(), ldd,
                                   loss.data_ptr(), ws.data_ptr(), ws.numel() * 4, L.stream_ptr(logits.device)),
            "cg_cross_entropy")
    return loss, dl


def adamw_(param, grad, exp_avg, exp_avg_sq, step, segments, shadow=None, beta1=0.9, beta2=0.999, eps=1e-8,
           grad_scale=1.0):
    """In-place AdamW over flat fp32 buffers; segments: [(begin, end, lr, wd)]."""
    n = len(segments)
    segs = (L.AdamwSegment * n)()
    for i, (b, e, lr, wd) in enumerate(segments):
        segs[i].begin, segs[i].end, segs[i].lr, segs[i].wd = int(b), int(e), float(lr), float(wd)
    L.check(L.lib.cg_adamw(param.data_ptr(), grad.data_ptr(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(),
                           _p(shadow), segs, n, beta1, beta2, eps, int(step), float(grad_scale),
                           L.stream_ptr(param.device)), "cg_adamw")


def cast_to_bf16(x):
    out = torch.empty(x.numel(), dtype=torch.bfloat16, device=x.device)
    L.check(L.lib.cg_cast_f32_to_bf16(x.data_ptr(), out.data_ptr(), x.numel(), L.stream_ptr(x.device)),
            "cg_cast_f32_to_bf16")
    return out.view(x.shape)


def cast_pad_2d(src, dcols, dtype=torch.bfloat16):
    """fp32 [rows][cols] -> dtype [rows][dcols], pad columns zero."""
    L.require_device(src, "cast_pad_2d")
    rows, cols = src.shape
    out = torch.empty(rows, dcols, dtype=dtype, device=src.device)
    L.check(L.lib.cg_cast_pad_2d(src.data_ptr(), src.stride(0), rows, cols, _dt(out), out.data_ptr(), out.stride(0),
                                 dcols, L.stream_ptr(src.device)), "cg_cast_pad_2d")
    return out


def _ids(values):
    vals = [int(v) for v in values]
    return (C.c_int * max(1, len(vals)))(*vals), len(vals)


def offset_targets(y, offset, boundary_ids=(2, 3), count=True):
    """(targets, n_valid): y[:, t+k-1] where offset_target_mask is true, else PAD (0).
    n_valid is a device int32 scalar (None with count=False)."""
    L.require_device(y, "offset_targets")
    y = y.to(torch.int64).contiguous()
    B, T = y.shape
    out = torch.empty_like(y)
    nv = torch.zeros((), dtype=torch.int32, device=y.device) if count else None
    ids, n = _ids(boundary_ids)
    L.check(L.lib.cg_offset_targets(y.data_ptr(), B, T, int(offset), ids, n, out.data_ptr(), _p(nv),
                                    L.stream_ptr(y.device)), "cg_offset_targets")
    return out, nv


def termination_labels(y, stop_ids, bucket_edges=(0, 3, 10, 30), ignore_index=-100):
    L.require_device(y, "termination_labels")
    y = y.to(torch.int64).contiguous()
    B, T = y.shape
    out = torch.empty_like(y)
    st, ns = _ids(stop_ids)
    ed, ne = _ids(bucket_edges)
    L.check(L.lib.cg_termination_labels(y.data_ptr(), B, T, st, ns, ed, ne, int(ignore_index), out.data_ptr(),
                                        L.stream_ptr(y.device)), "cg_termination_labels")
    return out


POOL_MODES = {"mean_nonpad": 0, "mean_content": 1, "eos": 2}


def pool_hidden(hidden, idx, mode, content_ids=(), pad_id=0):
    """_pool_state (extract_embeddings.py:94-114) of hidden (B, T, d) -> fp32 (B, d)."""
    L.require_device(hidden, "pool_hidden")
    B, T, d = hidden.shape
    if hidden.stride(2) != 1 or hidden.stride(0) != T * hidden.stride(1):
        hidden = hidden.contiguous()
    idx = idx.to(device=hidden.device, dtype=torch.int64).contiguous()
    words = [0] * 8
    for t in content_ids:
        t = int(t)
        if not 0 <= t < 256:
            raise ValueError("content ids must be in [0, 256)")
        words[t >> 5] |= 1 << (t & 31)
    mask = (C.c_uint32 * 8)(*words)
    out = torch.empty(B, d, dtype=torch.float32, device=hidden.device)
    L.check(L.lib.cg_pool_hidden(_dt(hidden), hidden.data_ptr(), hidden.stride(1), idx.data_ptr(), B, T, d,
                                 int(pad_id), POOL_MODES[mode], mask, out.data_ptr(),
                                 L.stream_ptr(hidden.device)), "cg_pool_hidden")
    return out


def colsum(x, out=None, accumulate=False):
    """out[n] (+)= sum_m x[m, n] (fp32 out)."""
    L.require_device(x, "colsum")
    rows, cols = x.shape
    if out is None:
        out = torch.empty(cols, dtype=torch.float32, device=x.device)
    ws = torch.empty(int(L.lib.cg_colsum_workspace(rows, cols)) // 4 + 1, dtype=torch.float32, device=x.device)
    L.check(L.lib.cg_colsum(_dt(x), x.data_ptr(), x.stride(0), rows, cols, out.data_ptr(), int(bool(accumulate)),
                            ws.data_ptr(), ws.numel() * 4, L.stream_ptr(x.device)), "cg_colsum")
    return out


def transpose16(mats):
    """Batched transpose of 2-byte 2-D tensors (one launch); returns the contiguous transposes."""
    if len(mats) > L.TRANSPOSE_MAX:
        raise ValueError("too many matrices")
    tb = L.TransposeBatch()
    tb.n = len(mats)
    outs = []
    for i, m in enumerate(mats):
        if m.element_size() != 2 or m.dim() != 2 or m.stride(1) != 1:
            raise ValueError("transpose16 takes row-major 2-byte matrices")
        L.require_device(m, "transpose16")
        o = torch.empty(m.shape[1], m.shape[0], dtype=m.dtype, device=m.device)
        tb.items[i] = L.TransposeItem(m.data_ptr(), o.data_ptr(), m.stride(0), o.stride(0), m.shape[0], m.shape[1])
        outs.append(o)
    if mats:
        L.check(L.lib.cg_transpose16_batch(C.byref(tb), L.stream_ptr(mats[0].device)), "cg_transpose16_batch")
    return outs


def gemm_dw_grouped(products, *, tile_m=0, ksplit=1):
    """Grouped weight gradients: for each (dy [K, N_out] bf16, x [K, K_out] bf16, out fp32
    [N_out, K_out], alpha, accumulate[, col_sum]) -> out (+)= alpha * dy^T x, one persistent launch
    (cg_gemm_dw_grouped).  Row strides are taken from the tensors.  ksplit > 1: each tile's K rows
    split over that many workgroups (fp32 slabs + one in-order reduction).  col_sum (fp32 [N_out],
    optional): (+)= alpha * the column sums of dy (the bias gradient), ksplit 1 only."""
    if not products:
        return
    if len(products) > L.DW_MAX:
        raise ValueError(f"at most {L.DW_MAX} products per group")
    g = L.DwGroup()
    g.n, g.tile_m = len(products), int(tile_m)
    K = None
    for i, (dy, x, out, alpha, acc, *cs) in enumerate(products):
        for t in (dy, x, out):
            L.require_device(t, "gemm_dw_grouped")
        if dy.dtype != torch.bfloat16 or x.dtype != torch.bfloat16 or out.dtype != torch.float32:
            raise ValueError("gemm_dw_grouped: bf16 operands, fp32 output")
        if K is None:
            K = dy.shape[0]
        if dy.shape[0] != K or x.shape[0] != K:
            raise ValueError("gemm_dw_grouped: every product reduces over the same K rows")
        p = g.p[i]
        p.A, p.lda, p.B, p.ldb = dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0)
        p.C, p.ldc = out.data_ptr(), out.stride(0)
        p.N_out, p.K_out = dy.shape[1], x.shape[1]
        if tuple(out.shape) != (p.N_out, p.K_out):
            raise ValueError("gemm_dw_grouped: out must be [N_out, K_out]")
        p.alpha, p.accumulate = float(alpha), int(bool(acc))
        if cs and cs[0] is not None:
            L.require_device(cs[0], "gemm_dw_grouped")
            if cs[0].dtype != torch.float32 or cs[0].numel() != p.N_out or not cs[0].is_contiguous():
                raise ValueError("gemm_dw_grouped: col_sum must be a contiguous fp32 [N_out]")
            p.col_sum = cs[0].data_ptr()
    g.K = int(K)
    ws = None
    if ksplit > 1:
        g.ksplit = int(ksplit)
        nbytes = int(L.lib.cg_gemm_dw_grouped_workspace(C.byref(g)))
        ws = torch.empty(max(nbytes, 16) // 4, dtype=torch.float32, device=products[0][0].device)
        g.workspace, g.ws_bytes = ws.data_ptr(), ws.numel() * 4
    L.check(L.lib.cg_gemm_dw_grouped(C.byref(g), L.stream_ptr(products[0][0].device)), "cg_gemm_dw_grouped")
    return ws
