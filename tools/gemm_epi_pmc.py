"""The C4 step's persistent forward / dX products with their epilogues and the same products plain,
one call each in a fixed order, for rocprofv3 --pmc passes (tools/gpu.sh pmc).  M = 32768 (the B=32
bench step).  With --summarize <dir>: join the counter rows of every pass (dispatch order) to the
product names and print per-product counters next to the plain product.

    python tools/gemm_epi_pmc.py                       (the workload, under rocprofv3)
    python tools/gemm_epi_pmc.py --summarize gpurun_out/pmc_epi
"""
import argparse
import csv
import glob
import os
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

# (name, N, K) in call order; each is called plain right after its epilogue version
PRODUCTS = [("proj fwd bias+resid", 512, 512), ("fc1 fwd bias+gelu", 2048, 512),
            ("fc2 fwd bias+drop+resid", 512, 2048), ("fc2 dX dgelu+colsum", 2048, 512)]
M = int(os.environ.get("GEMM_M", 32768))


def workload():
    sys.path.insert(0, str(ROOT / "genomics-lm_amd"))
    import torch
    from codonlm_amd import _lib as E, ops
    dev = "cuda"
    D = 512
    g = torch.Generator().manual_seed(0)
    bf = lambda *s: torch.randn(*s, generator=g).to(dev, torch.bfloat16)  # noqa: E731
    x512, x2048 = bf(M, D), bf(M, 4 * D)
    w = {n: (torch.randn(*s, generator=g) * 0.05).to(dev, torch.bfloat16)
         for n, s in [("proj", (D, D)), ("fc1", (4 * D, D)), ("fc2", (D, 4 * D)), ("fc2T", (4 * D, D))]}
    bias = {n: torch.zeros(n, device=dev) for n in (D, 4 * D)}
    o512f = torch.randn(M, D, generator=g).to(dev)
    o512 = torch.empty(M, D, dtype=torch.bfloat16, device=dev)
    o2048 = torch.empty(M, 4 * D, dtype=torch.bfloat16, device=dev)
    aux2048 = bf(M, 4 * D)
    cs = torch.empty(4 * D, device=dev)
    calls = [
        (lambda: ops.gemm(x512, w["proj"], out=o512f, bias=bias[D], resid=o512f, epilogue=E.EPI_BIAS | E.EPI_RESID),
         lambda: ops.gemm(x512, w["proj"], out=o512)),
        (lambda: ops.gemm(x512, w["fc1"], out=o2048, bias=bias[4 * D], aux_out=aux2048,
                          epilogue=E.EPI_BIAS | E.EPI_GELU | E.EPI_GELU_DERIV),
         lambda: ops.gemm(x512, w["fc1"], out=o2048)),
        (lambda: ops.gemm(x2048, w["fc2"], out=o512f, bias=bias[D], resid=o512f, drop_seed=5, drop_p=0.1,
                          epilogue=E.EPI_BIAS | E.EPI_RESID | E.EPI_DROPOUT),
         lambda: ops.gemm(x2048, w["fc2"], out=o512)),
        (lambda: ops.gemm(x512, w["fc2T"], out=o2048, aux=aux2048, colsum_out=cs,
                          epilogue=E.EPI_DGELU | E.EPI_GELU_DERIV),
         lambda: ops.gemm(x512, w["fc2T"], out=o2048)),
    ]
    for epi, plain in calls:  # warm-up (allocations, attributes) outside the counted order
        epi(); plain()
    torch.cuda.synchronize()
    print("MARK", flush=True)
    for epi, plain in calls:
        epi()
        torch.cuda.synchronize()
        plain()
        torch.cuda.synchronize()
    print("done")


def summarize(root):
    rows = defaultdict(dict)  # (pass, dispatch) -> counters; kernel name
    per_pass = defaultdict(list)
    for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        p = Path(f).parent.name
        disp = defaultdict(dict)
        names = {}
        for r in csv.DictReader(open(f)):
            if "gemm_bf16" not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            disp[d][r["Counter_Name"]] = disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[d] = r["Kernel_Name"].split("(")[0]
        ids = sorted(disp)[-2 * len(PRODUCTS):]  # the counted order: the last 2 x 4 GEMM dispatches
        per_pass[p] = [(names[d], disp[d]) for d in ids]
    order = [(n, tag) for n, _, _ in PRODUCTS for tag in ("epi", "plain")]
    table = defaultdict(dict)
    kname = {}
    for p, lst in per_pass.items():
        for (key, (kn, cs)) in zip(order, lst):
            table[key].update(cs)
            kname[key] = kn
    ctrs = sorted({c for v in table.values() for c in v})
    for n, N, K in PRODUCTS:
        print(f"== {n}  (M {M}, N {N}, K {K})")
        for tag in ("epi", "plain"):
            v = table[(n, tag)]
            print(f"   {tag:5s} {kname.get((n, tag), '?')}")
            print("         " + "  ".join(f"{c}={v[c]:.4g}" for c in ctrs if c in v))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--summarize")
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize)
    else:
        workload()
