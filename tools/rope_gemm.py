"""Time the C3 qkv projection with RoPE (M = 64 x 512 rows, N = (8 + 2 x 4) x 48, K = 384):
bias-only GEMM, the fused CG_EPI_ROPE epilogue, and bias GEMM + the cg_rope_tab pass.
Interleaved rounds of HIP-event-timed loops; min and median per variant.

    python tools/rope_gemm.py [M N_heads KV hd K T]
"""
import statistics
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "genomics-lm_amd"))
import torch  # noqa: E402
from codonlm_amd import _lib as L, ops  # noqa: E402

a = [int(v) for v in sys.argv[1:]]
M, H, KV, hd, K, T = a if len(a) == 6 else (32768, 8, 4, 48, 384, 512)
N = (H + 2 * KV) * hd
g = torch.Generator().manual_seed(0)
x = torch.randn(M, K, generator=g).to("cuda", torch.bfloat16)
w = (torch.randn(N, K, generator=g) * K ** -0.5).to("cuda", torch.bfloat16)
bias = torch.randn(N, generator=g).to("cuda")
half = hd // 2
inv = 1.0 / (10000 ** (torch.arange(half, dtype=torch.float64) / half))
ang = torch.arange(T, dtype=torch.float64)[:, None] * inv[None, :]
cos, sin = torch.cos(ang).float().cuda(), torch.sin(ang).float().cuda()
out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")


def v_bias():
    ops.gemm(x, w, out=out, bias=bias, epilogue=L.EPI_BIAS)


def v_fused():
    ops.gemm(x, w, out=out, bias=bias, epilogue=L.EPI_BIAS, rope=(cos, sin, T, hd, H + KV))


def v_table():
    ops.gemm(x, w, out=out, bias=bias, epilogue=L.EPI_BIAS)
    ops.rope_(out, M // T, T, H, KV, hd, cos, sin)


variants = {"bias": v_bias, "fused": v_fused, "bias+table": v_table}
times = {k: [] for k in variants}
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for fn in variants.values():
    for _ in range(3):
        fn()
torch.cuda.synchronize()
for _ in range(5):
    for k, fn in variants.items():
        s.record()
        for _ in range(20):
            fn()
        e.record()
        e.synchronize()
        times[k].append(s.elapsed_time(e) / 20 * 1e3)
for k, t in times.items():
    print(f"{k:12s} min {min(t):7.2f} us  median {statistics.median(t):7.2f} us", flush=True)
