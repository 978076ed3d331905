"""The C4 step's forward / dX persistent GEMMs with the engine's own epilogues, timed in
interleaved rounds (min over rounds; DVFS drifts within a long single-variant loop).

Each row: the epilogue the engine uses, and the same product with no epilogue (bf16 out), so
the epilogue's cost is the difference.  Device time by HIP events.
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "genomics-lm_amd"))
import torch  # noqa: E402
from codonlm_amd import _lib as L, ops  # noqa: E402

dev = "cuda"
import os  # noqa: E402
M, D = int(os.environ.get("GEMM_M", 16384)), 512  # GEMM_M=32768: the B=32 bench step


def timer(fn, it=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / it * 1e3  # us


def probe_bytes(fn):
    """algorithmic (FLOPs, HBM bytes) of one call, from the library's probe (persistent class)"""
    import ctypes as C
    L.lib.cg_probe_sample(1)
    L.lib.cg_probe_enable(L.PROBE_GEMM_PERS)
    fn()
    torch.cuda.synchronize()
    w, ms, k, b = C.c_double(0), C.c_double(0), C.c_longlong(0), C.c_double(0)
    L.lib.cg_probe_read(C.byref(w), C.byref(ms), C.byref(k))
    L.lib.cg_probe_bytes(C.byref(b))
    L.lib.cg_probe_enable(0)
    return w.value, b.value


def main():
    g = torch.Generator().manual_seed(0)
    bf = lambda *s: torch.randn(*s, generator=g).to(dev, torch.bfloat16)  # noqa: E731
    x512, x2048, x1536 = bf(M, D), bf(M, 4 * D), bf(M, 3 * D)
    w = {n: (torch.randn(*s, generator=g) * 0.05).to(dev, torch.bfloat16)
         for n, s in [("qkv", (3 * D, D)), ("proj", (D, D)), ("fc1", (4 * D, D)), ("fc2", (D, 4 * D)),
                      ("qkvT", (D, 3 * D)), ("projT", (D, D)), ("fc1T", (D, 4 * D)), ("fc2T", (4 * D, D))]}
    bias = {n: torch.zeros(n, device=dev) for n in (D, 3 * D, 4 * D)}
    resid = torch.randn(M, D, generator=g).to(dev)
    o512f = torch.empty(M, D, device=dev)
    o512 = torch.empty(M, D, dtype=torch.bfloat16, device=dev)
    o1536 = torch.empty(M, 3 * D, dtype=torch.bfloat16, device=dev)
    o2048 = torch.empty(M, 4 * D, dtype=torch.bfloat16, device=dev)
    aux2048 = torch.empty(M, 4 * D, dtype=torch.bfloat16, device=dev)
    cs = torch.empty(4 * D, device=dev)
    E = L
    rows = [
        ("qkv fwd   bias", 3 * D, D, lambda: ops.gemm(x512, w["qkv"], out=o1536, bias=bias[3 * D], epilogue=E.EPI_BIAS),
         lambda: ops.gemm(x512, w["qkv"], out=o1536)),
        ("proj fwd  bias+resid f32", D, D,
         lambda: ops.gemm(x512, w["proj"], out=o512f, bias=bias[D], resid=o512f, epilogue=E.EPI_BIAS | E.EPI_RESID),
         lambda: ops.gemm(x512, w["proj"], out=o512)),
        ("fc1 fwd   bias+gelu", 4 * D, D,
         lambda: ops.gemm(x512, w["fc1"], out=o2048, bias=bias[4 * D], aux_out=aux2048,
                          epilogue=E.EPI_BIAS | E.EPI_GELU | E.EPI_GELU_DERIV),
         lambda: ops.gemm(x512, w["fc1"], out=o2048)),
        ("fc2 fwd   bias+drop+resid f32", D, 4 * D,
         lambda: ops.gemm(x2048, w["fc2"], out=o512f, bias=bias[D], resid=o512f, drop_seed=5, drop_p=0.1,
                          epilogue=E.EPI_BIAS | E.EPI_RESID | E.EPI_DROPOUT),
         lambda: ops.gemm(x2048, w["fc2"], out=o512)),
        ("qkv dX", D, 3 * D, lambda: ops.gemm(x1536, w["qkvT"], out=o512), None),
        ("proj dX", D, D, lambda: ops.gemm(x512, w["projT"], out=o512), None),
        ("fc1 dX", D, 4 * D, lambda: ops.gemm(x2048, w["fc1T"], out=o512), None),
        ("fc2 dX    dgelu+colsum", 4 * D, D,
         lambda: ops.gemm(x512, w["fc2T"], out=o2048, aux=aux2048, colsum_out=cs,
                          epilogue=E.EPI_DGELU | E.EPI_GELU_DERIV),
         lambda: ops.gemm(x512, w["fc2T"], out=o2048)),
        ("fc2 dX    dgelu only", 4 * D, D,
         lambda: ops.gemm(x512, w["fc2T"], out=o2048, aux=aux2048, epilogue=E.EPI_DGELU | E.EPI_GELU_DERIV), None),
        ("fc2 dX    dgelu(pre-act) only", 4 * D, D,
         lambda: ops.gemm(x512, w["fc2T"], out=o2048, aux=aux2048, epilogue=E.EPI_DGELU), None),
        ("fc1 fwd   bias+gelu(pre-act) only", 4 * D, D,
         lambda: ops.gemm(x512, w["fc1"], out=o2048, bias=bias[4 * D], aux_out=aux2048,
                          epilogue=E.EPI_BIAS | E.EPI_GELU), None),
        ("fc2 dX    colsum only", 4 * D, D,
         lambda: ops.gemm(x512, w["fc2T"], out=o2048, colsum_out=cs), None),
        ("colsum reduce", 4 * D, D,
         lambda: L.lib.cg_colsum_reduce(csw.data_ptr(), M // 64, 4 * D, cs.data_ptr(), 0, L.stream_ptr(cs.device)), None),
    ]
    csw = torch.zeros(M // 64 * 4 * D, device=dev)
    for _, _, _, f, f0 in rows:
        f()
        if f0:
            f0()
    torch.cuda.synchronize()
    only = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] else None  # e.g. "fc2 dX": time only matching rows
    rows = [r for r in rows if only is None or r[0].startswith(only)]
    # GEMM_VARIANTS="auto,pers,lw": the persistent-tile kernels to interleave (cg_gemm_desc.tile:
    # automatic, the eight-wave kernel, the loader-wave kernel)
    import functools
    gemm0 = ops.gemm

    def set_variant(v):
        ops.gemm = functools.partial(gemm0, tile={"auto": L.TILE_AUTO, "pers": L.TILE_PERS,
                                                  "lw": L.TILE_PERS_LW}[v])

    modes = [v for v in os.environ.get("GEMM_VARIANTS", "").split(",") if v] or [None]
    bests = {m: {} for m in modes}
    for _ in range(8):
        for mode in modes:
            if mode is not None:
                set_variant(mode)
            best = bests[mode]
            for name, _, _, f, f0 in rows:
                for tag, fn in (("epi", f), ("plain", f0)):
                    if fn is None:
                        continue
                    t = timer(fn)
                    best[(name, tag)] = min(best.get((name, tag), 1e9), t)
    for mode in modes:
        if mode is not None:
            set_variant(mode)
            print(f"== persistent variant: {mode}")
        report(rows, bests[mode], only)


def report(rows, best, only):
    tot = 0.0
    for name, N, K, f, f0 in rows:
        fl = 2.0 * M * N * K
        te = best[(name, "epi")]
        pw, pb = probe_bytes(f)
        # roofline time of the product: max(FLOPs at 2.5 PF, algorithmic bytes at 8 TB/s)
        bound = max(pw / 2.5e15, pb / 8e12) * 1e6 if pw else 0.0
        if not name.endswith(" only") and name != "colsum reduce":  # the step's own products
            tot += te
        tp = best.get((name, "plain"))
        extra = f"  plain {tp:6.1f} us {fl / tp / 1e6:6.1f} TF/s" if tp else ""
        print(f"{name:32s} N={N:5d} K={K:5d} {te:6.1f} us {fl / te / 1e6:6.1f} TF/s  {pb / 1e6:6.1f} MB "
              f"{pb / te / 1e6:5.2f} TB/s  roof {bound:5.1f} us ({bound / te:4.2f}){extra}", flush=True)
    if only is None:
        print(f"sum per layer {tot:.1f} us  (x12 = {tot * 12 / 1e3:.2f} ms)")


if __name__ == "__main__":
    main()
