"""cg_gemm vs torch/hipBLASLt on the C4 step shapes (device time, HIP events)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "genomics-lm_amd"))
import torch  # noqa: E402
from codonlm_amd import _lib as L, ops  # noqa: E402

dev = "cuda"
M = 16384


def t(fn, it=30):
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


def main():
    g = torch.Generator().manual_seed(0)
    for name, N, K in [("qkv", 1536, 512), ("proj", 512, 512), ("fc1", 2048, 512), ("fc2", 512, 2048)]:
        x = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
        w = (torch.randn(N, K, generator=g) * 0.05).to(dev, torch.bfloat16)
        wT = w.t().contiguous()
        dy = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        bias = torch.zeros(N, device=dev)
        dx = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
        dw = torch.empty(N, K, dtype=torch.float32, device=dev)
        fl = 2.0 * M * N * K
        rows = [
            ("fwd ours", lambda: ops.gemm(x, w, out=out)),
            ("fwd ours bias", lambda: ops.gemm(x, w, out=out, bias=bias, epilogue=L.EPI_BIAS)),
            ("fwd ours gelu", lambda: ops.gemm(x, w, out=out, bias=bias, epilogue=L.EPI_BIAS | L.EPI_GELU, aux_out=aux)),
            ("fwd blas", lambda: torch.mm(x, w.t(), out=out)),
            ("dX ours(wT)", lambda: ops.gemm(dy, wT, M=M, N=K, K=N, out=dx)),
            ("dX ours dgelu", lambda: ops.gemm(dy, wT, M=M, N=K, K=N, out=dx, epilogue=L.EPI_DGELU, aux=x)),
            ("dX blas", lambda: torch.mm(dy, w, out=dx)),
            ("dW ours s4", lambda: ops.gemm(dy, x, a_kcontig=False, b_kcontig=False, M=N, N=K, K=M, out=dw, split_k=4)),
            ("dW ours s8", lambda: ops.gemm(dy, x, a_kcontig=False, b_kcontig=False, M=N, N=K, K=M, out=dw, split_k=8)),
            ("dW blas bf16", lambda: torch.mm(dy.t(), x)),
            ("dW blas f32out", lambda: torch.mm(dy.t(), x, out_dtype=torch.float32) if hasattr(torch, "mm") else None),
        ]
        for rn, fn in rows:
            try:
                dt = t(fn)
                print(f"{name:5s} {rn:16s} {dt*1e6:8.1f} us {fl/dt/1e12:7.1f} TF/s", flush=True)
            except Exception as ex:  # noqa: BLE001
                print(f"{name:5s} {rn:16s} n/a ({type(ex).__name__}: {str(ex)[:60]})", flush=True)


if __name__ == "__main__":
    main()
