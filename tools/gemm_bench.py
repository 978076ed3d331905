"""Micro-benchmark of cg_gemm at the C4 step shapes (device time via HIP events)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "genomics-lm_amd"))
import torch  # noqa: E402
from codonlm_amd import _lib as L, ops  # noqa: E402

dev = "cuda"
M = 16384


def t(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / it * 1e-3


def run():
    g = torch.Generator().manual_seed(0)
    res = []
    for name, N, K in [("qkv", 1536, 512), ("proj", 512, 512), ("fc1", 2048, 512), ("fc2", 512, 2048)]:
        x = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
        w = (torch.randn(N, K, generator=g) * 0.05).to(dev, torch.bfloat16)
        bias = torch.zeros(N, device=dev)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        outf = torch.empty(M, N, dtype=torch.float32, device=dev)
        aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        fl = 2.0 * M * N * K
        for ename, fn in [
            ("none_bf16", lambda: ops.gemm(x, w, out=out)),
            ("none_f32", lambda: ops.gemm(x, w, out=outf)),
            ("bias", lambda: ops.gemm(x, w, out=out, bias=bias, epilogue=L.EPI_BIAS)),
            ("bias_gelu", lambda: ops.gemm(x, w, out=out, bias=bias, epilogue=L.EPI_BIAS | L.EPI_GELU, aux_out=aux)),
            ("resid_f32", lambda: ops.gemm(x, w, out=outf, bias=bias, resid=outf, epilogue=L.EPI_BIAS | L.EPI_RESID)),
        ]:
            dt = t(fn)
            res.append(f"fwd  {name:5s} {ename:10s} {dt*1e6:8.1f} us {fl/dt/1e12:7.1f} TF/s")
        # dX layout (B n-contig) and dW layout (both mn-contig)
        wt = w  # [N][K] as W: dx = dy[M,N] . W[N,K] -> gemm(A=dy kc, B(n=k, k=n) = W[n*K + k] mn-contig)
        dy = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
        dx = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
        dt = t(lambda: ops.gemm(dy, wt, b_kcontig=False, M=M, N=K, K=N, out=dx))
        res.append(f"dX   {name:5s} {'none_bf16':10s} {dt*1e6:8.1f} us {fl/dt/1e12:7.1f} TF/s")
        dw = torch.empty(N, K, dtype=torch.float32, device=dev)
        for sk in (1, 4, 8):
            dt = t(lambda: ops.gemm(dy, x, a_kcontig=False, b_kcontig=False, M=N, N=K, K=M, out=dw, split_k=sk))
            res.append(f"dW   {name:5s} split{sk:<5d} {dt*1e6:8.1f} us {fl/dt/1e12:7.1f} TF/s")
    print("\n".join(res))


if __name__ == "__main__":
    run()
