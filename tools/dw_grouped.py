"""Grouped dW GEMM (cg_gemm_dw_grouped) vs the split-K dW path on the C4/C5 block products:
correctness against torch fp32 of the same bf16 operands, then device time per layer."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "genomics-lm_amd"))
import torch
from codonlm_amd import ops, _lib as L

dev = "cuda"
torch.manual_seed(0)


def layer_products(M, d, nqkv, hid):
    # (dY cols N_out, X cols K_out): qkv, proj, fc1, fc2
    shapes = [(nqkv, d), (d, d), (hid, d), (d, hid)]
    out = []
    for n, k in shapes:
        dy = (torch.randn(M, n, device=dev) * 0.5).to(torch.bfloat16)
        x = torch.randn(M, k, device=dev).to(torch.bfloat16)
        out.append((dy, x, torch.empty(n, k, device=dev), 1.0, False))
    return out


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


for name, (M, d, nqkv, hid) in {"c4": (16384, 512, 1536, 2048), "c5": (16384, 384, 1152, 1536)}.items():
    prods = layer_products(M, d, nqkv, hid)
    # correctness (one product of each shape, both tiles)
    for bm in (128, 256, 512):
        ops.gemm_dw_grouped(prods, tile_m=bm)
        torch.cuda.synchronize()
        for dy, x, out, _, _ in prods:
            ref = dy.float().t() @ x.float()
            err = ((out - ref).abs().max() / ref.abs().max()).item()
            assert err < 1e-4, (name, bm, tuple(out.shape), err)
    flops = sum(2.0 * M * p[0].shape[1] * p[1].shape[1] for p in prods)
    for bm in (128, 129, 256, 512):
        t1 = timeit(lambda: ops.gemm_dw_grouped(prods, tile_m=bm))
        print(f"{name} layer group  BM={bm}: {t1:8.1f} us  {flops / t1 / 1e6:7.1f} TF/s")
        for p in prods[:1]:
            f = 2.0 * M * p[0].shape[1] * p[1].shape[1]
            t = timeit(lambda: ops.gemm_dw_grouped([p], tile_m=bm))
            print(f"   single {tuple(p[2].shape)} BM={bm}: {t:8.1f} us  {f / t / 1e6:7.1f} TF/s")
    for G in (2, 4, 5):
        many = prods * G  # same operands G times (L2/MALL-warm upper bound for a G-layer group)
        outs = [(a, b, torch.empty_like(c), al, ac) for a, b, c, al, ac in many]
        for bm in (256, 512):
            t = timeit(lambda: ops.gemm_dw_grouped(outs, tile_m=bm))
            print(f"{name} {G}-layer group BM={bm}: {t:8.1f} us  {G * flops / t / 1e6:7.1f} TF/s  ({t / G:.1f} us/layer)")
    # the split-K path this replaces (dW = dY^T X via cg_gemm with MN-contiguous operands)
    def old():
        for dy, x, out, _, _ in prods:
            n, k = out.shape
            ops.gemm(dy, x, a_kcontig=False, b_kcontig=False, M=n, N=k, K=M, out=out,
                     split_k=max(1, min(16, 512 // (((n + 127) // 128) * ((k + 127) // 128)))))
    t = timeit(old)
    print(f"{name} split-K path (4 launches + reduces): {t:8.1f} us  {flops / t / 1e6:7.1f} TF/s")
