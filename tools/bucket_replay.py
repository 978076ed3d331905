"""Price the grouped-dW bucket order of the C4 data-parallel backward on one GPU.

A data-parallel step all-reduces each block's fp32 gradient bucket (12.6 MB at C4) once its dW
group's grouped launch is enqueued (training/ddp.py); RCCL's kernels then hold some CUs beside
the backward's persistent launches, and the buckets whose all-reduce can only start after the
last dW launch are exposed.  Here that is replayed on one GPU: at every bucket hook of the
engine's backward a stand-in kernel (cg_diag_occupy: whole-CU workgroups that sleep) is queued
on a side stream behind an event of the compute stream, holding NCH CUs (RCCL's channels) for the
bucket's modelled ring time over xGMI,

    t = 2 (n - 1) / n * bytes / busbw,   n = 8 GPUs,

and the step time (fwd + bwd + the side stream + AdamW, synchronised) is measured for each dW
group plan -- the planner's own choice, 5/5/2, 4/4/4, 3/3/3/3, 6/6 (remainder group last) --
and each (NCH, busbw) pair.  Interleaved rounds, min and median.

    BR_B=32 python tools/bucket_replay.py [busbw_GBs ...]     (BR_B: sequences per GPU, default 32)

BR_PLANS=planner limits the plans; BR_RESERVE=8,16 adds the planner's plan with every persistent
launch capped at cg_pers_cus() - R workgroups (cg_model_opts.pers_max_wg), the CUs a data-parallel
run would leave to RCCL's kernels.
"""
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "genomics-lm_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from codonlm_amd import TinyGPT, _lib as L  # noqa: E402
from codonlm_amd.optim import FusedAdamW  # noqa: E402
from codonlm_amd.training.ddp import bucket_ranges  # noqa: E402

# (name, engine_opts): the dW group plans (cg_model_opts dw_remainder_first / dw_group)
PLANS = [("planner", {}), ("5/5/2", {"dw_group": 5}), ("4/4/4", {"dw_group": 4}), ("3/3/3/3", {"dw_group": 3}),
         ("6/6", {"dw_group": 6})]
B = int(os.environ.get("BR_B", "32"))


def main():
    busbws = [float(a) for a in sys.argv[1:]] or [300.0, 600.0]
    dev = torch.device("cuda", 0)
    models = {}
    plans = [p for p in PLANS if p[0] in os.environ.get("BR_PLANS", ",".join(n for n, _ in PLANS)).split(",")]
    cus = int(L.lib.cg_pers_cus())
    for r in [int(v) for v in os.environ.get("BR_RESERVE", "").split(",") if v]:
        plans.append((f"res{r}", {"pers_max_wg": cus - r}))
    PLANS[:] = plans
    for name, opts in PLANS:  # one model per plan (the plan is part of the model's configuration)
        torch.manual_seed(0)
        m = TinyGPT(68, 1024, n_layer=12, n_head=8, n_embd=512, dropout=0.1, label_smoothing=0.05,
                    compute_dtype="bf16", device=dev, engine_opts=opts)
        m.train()
        models[name] = (m, FusedAdamW(m, lr=3e-4, weight_decay=0.05))
    rng = np.random.default_rng(0)
    tok = torch.from_numpy(rng.integers(4, 68, size=(B, 1025))).to(dev)
    G, tm, ks = L.C.c_int(0), L.C.c_int(0), L.C.c_int(0)
    for name, (m, _) in models.items():
        L.check(L.lib.cg_model_dw_plan(L.C.byref(m.engine.model.cfg), B, 1024, L.C.byref(G), L.C.byref(tm),
                                       L.C.byref(ks)), "cg_model_dw_plan")
        print(f"plan {name}: groups of {G.value} blocks, tile {tm.value}, token split {ks.value}", flush=True)
    x, y = tok[:, :-1].contiguous(), tok[:, 1:].contiguous()
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)
    nbytes = {k: 4 * (e - b) for k, (b, e) in bucket_ranges(models["planner"][0]).items()}

    def step(m, opt, nch, busbw):
        opt.zero_grad(set_to_none=True)
        _, loss = m(x, y)
        if nch:
            def hook(name):
                t_us = 2 * 7 / 8 * nbytes[name] / (busbw * 1e9) * 1e6
                ev = torch.cuda.Event()
                ev.record(main_s)
                side.wait_event(ev)
                L.check(L.lib.cg_diag_occupy(nch, max(1, int(t_us)), side.cuda_stream), "cg_diag_occupy")
            m._bucket_hook = hook
        loss.backward()
        if nch:  # the optimizer waits for every all-reduce
            ev = torch.cuda.Event()
            ev.record(side)
            main_s.wait_event(ev)
        opt.step()

    cases = [(p, nch, bw) for p, _ in PLANS for nch, bw in [(0, 0.0)] + [(n, b) for n in (8, 16) for b in busbws]]
    times = {c: [] for c in cases}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(4):
        for plan, nch, bw in cases:
            m, opt = models[plan]
            step(m, opt, nch, bw)  # warm
            torch.cuda.synchronize()
            s.record()
            for _ in range(5):
                step(m, opt, nch, bw)
            e.record()
            e.synchronize()
            times[(plan, nch, bw)].append(s.elapsed_time(e) / 5)
    for (plan, nch, bw), t in times.items():
        tag = "no comm" if not nch else f"{nch:2d} CUs, busbw {bw:4.0f} GB/s"
        print(f"plan {plan:7s} {tag:28s} step {min(t):6.3f} ms (median {statistics.median(t):6.3f})", flush=True)


if __name__ == "__main__":
    main()
