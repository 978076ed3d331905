"""Sensitivity of the C4 training step to CUs held by another kernel.

In a data-parallel run RCCL's all-reduce kernels run on some CUs beside the backward; every
persistent launch (forward / dX tiles, grouped dW) assumes one workgroup per CU.  Here a
stand-in kernel (cg_diag_occupy: whole-CU workgroups that sleep) holds N CUs for the backward's
duration, on a side stream started right after the forward, and the step time is measured for
N in {0, 8, 16, 32} with the persistent grids using all CUs (reserve 0) or leaving the N CUs
free (cg_set_cu_reserve(N)).  Interleaved rounds, min and median over rounds.

    python tools/cu_busy.py
"""
import ctypes as C
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "genomics-lm_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from codonlm_amd import TinyGPT, _lib as L  # noqa: E402
from codonlm_amd.optim import FusedAdamW  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = TinyGPT(68, 1024, n_layer=12, n_head=8, n_embd=512, dropout=0.1, label_smoothing=0.05,
                compute_dtype="bf16", device=dev)
    m.train()
    opt = FusedAdamW(m, lr=3e-4, weight_decay=0.05)
    rng = np.random.default_rng(0)
    tok = torch.from_numpy(rng.integers(4, 68, size=(16, 1025))).to(dev)
    x, y = tok[:, :-1].contiguous(), tok[:, 1:].contiguous()
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)

    def step(n_busy, bwd_us):
        opt.zero_grad(set_to_none=True)
        _, loss = m(x, y)
        if n_busy:
            ev = torch.cuda.Event()
            ev.record(main_s)
            side.wait_event(ev)
            L.check(L.lib.cg_diag_occupy(n_busy, int(bwd_us), side.cuda_stream), "cg_diag_occupy")
        loss.backward()
        opt.step()

    for _ in range(5):
        step(0, 0)
    torch.cuda.synchronize()
    # backward duration, to size the occupier
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    _, loss = m(x, y)
    s.record()
    loss.backward()
    e.record()
    e.synchronize()
    bwd_us = s.elapsed_time(e) * 1e3
    print(f"backward {bwd_us:.0f} us", flush=True)
    cases = [(n, r) for n in (0, 8, 16, 32) for r in sorted({0, n})]
    times = {c: [] for c in cases}
    for _ in range(5):
        for n, r in cases:
            L.lib.cg_set_cu_reserve(r)
            step(n, bwd_us)  # warm (re-plans the dW grouping for the reserve)
            torch.cuda.synchronize()
            s.record()
            for _ in range(5):
                step(n, bwd_us)
            e.record()
            e.synchronize()
            times[(n, r)].append(s.elapsed_time(e) / 5)
    L.lib.cg_set_cu_reserve(0)
    for (n, r), t in times.items():
        print(f"busy CUs {n:2d}  reserve {r:2d}:  step {min(t):6.3f} ms (median {statistics.median(t):6.3f})",
              flush=True)


if __name__ == "__main__":
    main()
