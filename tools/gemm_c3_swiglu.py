"""C3 SwiGLU products (M = 64 x 512 tokens, d 384, hidden 1024): the gate|up forward with the
SwiGLU epilogue and the dL/ds product with the SwiGLU backward epilogue, min over reps of the
per-launch time by HIP events (CG_LIB_PATH selects a variant build for same-box A/B)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "genomics-lm_amd"))
import torch  # noqa: E402
from codonlm_amd import _lib as L, ops  # noqa: E402

M, D, H = 32768, 384, 1024
dev = "cuda"
g = torch.Generator().manual_seed(0)
x = torch.randn(M, D, generator=g).to(dev, torch.bfloat16)
wgu = (torch.randn(2 * H, D, generator=g) * D ** -0.5).to(dev, torch.bfloat16)
gin = torch.randn(M, D, generator=g).to(dev, torch.bfloat16)
wdT = (torch.randn(H, D, generator=g) * D ** -0.5).to(dev, torch.bfloat16)
gu = torch.empty(M, 2 * H, device=dev, dtype=torch.bfloat16)
s = torch.empty(M, H, device=dev, dtype=torch.bfloat16)
dgu = torch.empty(M, 2 * H, device=dev, dtype=torch.bfloat16)
rows = [("swiglu fwd", lambda: ops.gemm(x, wgu, N=H, out=s, epilogue=L.EPI_SWIGLU, aux_out=gu, n_valid=H)),
        ("swiglu bwd", lambda: ops.gemm(gin, wdT, N=H, out=dgu, epilogue=L.EPI_DSWIGLU, aux=gu, n_valid=H))]
for _, f in rows:
    f()
torch.cuda.synchronize()
best = {}
for _ in range(6):
    for name, f in rows:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            f()
        e1.record()
        torch.cuda.synchronize()
        best[name] = min(best.get(name, 1e9), e0.elapsed_time(e1) * 100.0)
for name, _ in rows:
    print(f"{name:12s} {best[name]:7.1f} us")
