"""fc1-forward-shaped persistent GEMM (M=16384, N=2048, K=512) with epilogue 0 / bias / bias+GELU,
for rocprofv3 counter passes (one kernel name per epilogue)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "genomics-lm_amd"))
import torch  # noqa: E402
from codonlm_amd import _lib as L, ops  # noqa: E402
M, N, K = 16384, 2048, 512
g = torch.Generator().manual_seed(0)
x = torch.randn(M, K, generator=g).to("cuda", torch.bfloat16)
w = (torch.randn(N, K, generator=g) * 0.05).to("cuda", torch.bfloat16)
bias = torch.zeros(N, device="cuda")
out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
aux = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
for _ in range(5):
    ops.gemm(x, w, out=out)
    ops.gemm(x, w, out=out, bias=bias, epilogue=L.EPI_BIAS)
    ops.gemm(x, w, out=out, bias=bias, epilogue=L.EPI_BIAS | L.EPI_GELU, aux_out=aux)
torch.cuda.synchronize()
print("ok")
