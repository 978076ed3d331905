"""dW GEMM sweep at the C4 shapes: 128x128 register-staged vs 256x128 LDS-DMA tile, split-K."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "genomics-lm_amd"))
import torch  # noqa: E402
from codonlm_amd import _lib as L, ops  # noqa: E402

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


g = torch.Generator().manual_seed(0)
for name, N, K in [("qkv", 1536, 512), ("proj", 512, 512), ("fc1", 2048, 512), ("fc2", 512, 2048)]:
    x = torch.randn(M, K, generator=g).to("cuda", torch.bfloat16)
    dy = torch.randn(M, N, generator=g).to("cuda", torch.bfloat16)
    dw = torch.empty(N, K, dtype=torch.float32, device="cuda")
    ref = (dy.float().t() @ x.float())
    fl = 2.0 * M * N * K
    for wide in (0, 1):
        L.lib.cg_gemm_set_wide(wide)
        for sk in (2, 4, 8, 16, 32):
            fn = lambda: ops.gemm(dy, x, a_kcontig=False, b_kcontig=False, M=N, N=K, K=M, out=dw, split_k=sk)
            dt = t(fn)
            err = float((dw - ref).abs().max() / ref.abs().max())
            print(f"{name:5s} wide={wide} split={sk:2d} {dt*1e6:8.1f} us {fl/dt/1e12:7.1f} TF/s err={err:.1e}", flush=True)
    L.lib.cg_gemm_set_wide(-1)
