"""Known-good references on the same hardware: hipBLASLt (torch.mm) and torch SDPA vs our kernels
at the C4 step shapes.  Device time via HIP events; bf16 operands, random data."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "genomics-lm_amd"))
import torch
import torch.nn.functional as F
from codonlm_amd import _lib as L, ops

dev = "cuda"


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / it * 1e-3


M = 16384
g = torch.Generator().manual_seed(0)
print(f"{'shape':28s} {'ours_us':>8s} {'ours_TF':>8s} {'blas_us':>8s} {'blas_TF':>8s}")
for name, N, K in [("qkv", 1536, 512), ("proj", 512, 512), ("fc1", 2048, 512), ("fc2", 512, 2048)]:
    x = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(dev, torch.bfloat16)
    dy = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    dx = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
    dw = torch.empty(N, K, dtype=torch.float32, device=dev)
    fl = 2.0 * M * N * K
    rows = [
        ("fwd " + name, lambda: ops.gemm(x, w, out=out), lambda: torch.mm(x, w.t(), out=out)),
        ("dX  " + name, lambda: ops.gemm(dy, w, b_kcontig=False, M=M, N=K, K=N, out=dx),
         lambda: torch.mm(dy, w, out=dx)),
    ]
    for sp in (4, 8, 16):
        rows.append((f"dW  {name} s{sp}", lambda sp=sp: ops.gemm(dy, x, a_kcontig=False, b_kcontig=False, M=N, N=K,
                                                               K=M, out=dw, split_k=sp),
                     lambda: torch.mm(dy.t(), x)))
    for lbl, ours, blas in rows:
        a, b = t(ours), t(blas)
        print(f"{lbl:28s} {a*1e6:8.1f} {fl/a/1e12:8.1f} {b*1e6:8.1f} {fl/b/1e12:8.1f}", flush=True)

# attention: B=16 H=8 T=1024 hd=64, causal
B, H, T, hd = 16, 8, 1024, 64
qkv = (torch.randn(B * T, 3 * H * hd, generator=g) * 0.5).to(dev, torch.bfloat16)
q = qkv[:, :H * hd].view(B, T, H, hd).transpose(1, 2).contiguous()
k = qkv[:, H * hd:2 * H * hd].view(B, T, H, hd).transpose(1, 2).contiguous()
v = qkv[:, 2 * H * hd:].view(B, T, H, hd).transpose(1, 2).contiguous()
tri = 2.0 * B * H * hd * T * (T + 1) / 2
seg = torch.zeros(B, T, dtype=torch.int32, device=dev)
y = torch.empty(B * T, H * hd, dtype=torch.bfloat16, device=dev)
lse = torch.empty(B * H * T, dtype=torch.float32, device=dev)


def ours_fwd():
    L.check(L.lib.cg_attn_fwd(L.CG_BF16, qkv.data_ptr(), qkv.stride(0), None, y.data_ptr(), y.stride(0),
                              lse.data_ptr(), B, T, H, H, hd, 0, 0, 0.0, None, L.stream_ptr(qkv.device)), "fwd")


def sdpa_fwd():
    return F.scaled_dot_product_attention(q, k, v, is_causal=True)


a, b = t(ours_fwd), t(sdpa_fwd)
print(f"{'attn fwd causal':28s} {a*1e6:8.1f} {2*tri/a/1e12:8.1f} {b*1e6:8.1f} {2*tri/b/1e12:8.1f}")
qr, kr, vr = (z.clone().requires_grad_(True) for z in (q, k, v))
o = F.scaled_dot_product_attention(qr, kr, vr, is_causal=True)
go = torch.randn_like(o)


def sdpa_bwd():
    torch.autograd.grad(o, (qr, kr, vr), go, retain_graph=True)


b = t(sdpa_bwd)
print(f"{'attn bwd causal (sdpa)':28s} {'':8s} {'':8s} {b*1e6:8.1f} {5*tri/b/1e12:8.1f}")
print("backend flags:", torch.backends.cuda.flash_sdp_enabled(), torch.backends.cuda.mem_efficient_sdp_enabled())
