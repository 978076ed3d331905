"""Plain persistent-GEMM products of the C4 step (no epilogue), min device time over rounds.
Run once per library build (CG_LIB_PATH=ab/<variant>/libcodonlm_hip.so) to compare diagnostic
variants (gemm_pers.h CG_PERS_DIAG: 1 = no operand DMA in the k-loop, 2 = no MFMA)."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "genomics-lm_amd"))
import torch  # noqa: E402
from codonlm_amd import ops  # noqa: E402

M = 16384
SHAPES = [("fc1 dX", 512, 2048), ("qkv dX", 512, 1536), ("proj dX", 512, 512), ("qkv fwd", 1536, 512),
          ("fc1 fwd", 2048, 512)]


def main():
    g = torch.Generator().manual_seed(0)
    ops_ = []
    for name, N, K in SHAPES:
        a = torch.randn(M, K, generator=g).to("cuda", torch.bfloat16)
        b = (torch.randn(N, K, generator=g) * 0.05).to("cuda", torch.bfloat16)
        o = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        ops_.append((name, N, K, lambda a=a, b=b, o=o: ops.gemm(a, b, out=o)))
    best = {}
    for _ in range(6):
        for name, N, K, f in ops_:
            f()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                f()
            e.record()
            e.synchronize()
            best[name] = min(best.get(name, 1e9), s.elapsed_time(e) / 10 * 1e3)
    tag = os.environ.get("CG_LIB_PATH", "default")
    for name, N, K, _ in ops_:
        t = best[name]
        print(f"{tag[-40:]:40s} {name:8s} N={N:5d} K={K:5d} {t:7.1f} us {2.0 * M * N * K / t / 1e6:7.1f} TF/s")


if __name__ == "__main__":
    main()
