"""Step time of the C4 training step (fwd + bwd + AdamW, no communication) under forced grouped-dW
plans (cg_model_opts dw_group / dw_ksplit), interleaved rounds, min and median -- the check of the
dW planner's choice at a batch size.

    BR_B=32 python tools/dw_plans.py "G:KS G:KS ..."      (0 = the planner's choice)
"""
import os
import statistics
import sys
import ctypes as C
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "genomics-lm_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from codonlm_amd import TinyGPT, _lib as L  # noqa: E402
from codonlm_amd.optim import FusedAdamW  # noqa: E402

B = int(os.environ.get("BR_B", "32"))
plans = [tuple(int(v) for v in p.split(":")) for p in (sys.argv[1] if len(sys.argv) > 1 else "0:0 5:0").split()]
dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
tok = torch.from_numpy(rng.integers(4, 68, size=(B, 1025))).to(dev)
x, y = tok[:, :-1].contiguous(), tok[:, 1:].contiguous()
models = {}
G, tm, ks = C.c_int(0), C.c_int(0), C.c_int(0)
for g, k in plans:
    torch.manual_seed(0)
    m = TinyGPT(68, 1024, n_layer=12, n_head=8, n_embd=512, dropout=0.1, label_smoothing=0.05, compute_dtype="bf16",
                device=dev, engine_opts={"dw_group": g, "dw_ksplit": k})
    m.train()
    L.check(L.lib.cg_model_dw_plan(C.byref(m.engine.model.cfg), B, 1024, C.byref(G), C.byref(tm), C.byref(ks)), "plan")
    models[(g, k)] = (m, FusedAdamW(m, lr=3e-4, weight_decay=0.05), (G.value, tm.value, ks.value))


def step(m, opt):
    opt.zero_grad(set_to_none=True)
    _, loss = m(x, y)
    loss.backward()
    opt.step()


times = {p: [] for p in models}
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(4):
    for p, (m, opt, _) in models.items():
        step(m, opt)
        torch.cuda.synchronize()
        s.record()
        for _ in range(5):
            step(m, opt)
        e.record()
        e.synchronize()
        times[p].append(s.elapsed_time(e) / 5)
for p, t in times.items():
    print(f"B={B} forced {p} -> plan (G, tile, ks) {models[p][2]}: step {min(t):6.3f} ms (median {statistics.median(t):6.3f})",
          flush=True)
