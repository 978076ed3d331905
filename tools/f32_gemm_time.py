"""fp32 GEMM timing on the C4 step shapes (forward, dX, dW layouts), HIP events, one library per
process (CG_LIB_PATH).  Prints us and TF/s per product."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "genomics-lm_amd"))
import torch  # noqa: E402
from codonlm_amd import ops  # noqa: E402

M, D = 16384, 512
dev = "cuda"
g = torch.Generator().manual_seed(0)


def t(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / it * 1e3


for name, N, K in [("qkv", 3 * D, D), ("fc1", 4 * D, D), ("fc2", D, 4 * D)]:
    x = torch.randn(M, K, generator=g).to(dev)
    w = torch.randn(N, K, generator=g).to(dev)
    dy = torch.randn(M, N, generator=g).to(dev)
    fl = 2.0 * M * N * K
    us = t(lambda: ops.gemm(x, w))
    print(f"{name:4s} fwd  {us:8.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)
    us = t(lambda: ops.gemm(dy, w, b_kcontig=False, M=M, N=K, K=N))
    print(f"{name:4s} dX   {us:8.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)
    ws = torch.empty(8 * N * K, device=dev)
    us = t(lambda: ops.gemm(dy, x, a_kcontig=False, b_kcontig=False, M=N, N=K, K=M, split_k=8))
    print(f"{name:4s} dW   {us:8.1f} us {fl / us / 1e6:7.1f} TF/s  (split 8)", flush=True)
