#!/usr/bin/env python3
"""Throughput of the MI355X codon-LM training step (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c2|c3|c5] [--path engine|trainer]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Workload = BASELINE config C4: TinyGPT 12L8H d512 (hd 64), T=1024, V=68 codons, GELU MLP,
SEP-segment causal mask, dropout 0.1, label smoothing 0.05, bf16 compute with fp32
master weights / AdamW, per-GPU microbatch B=32 (weak scaling) -- the 32 sequences of one
optimizer step of the reference's 12L8H d512 run (batch_size 2 x grad_accum_steps 16,
runs/2025-11-05_tiny_12L8H_d512_e5/log.txt:30-31,80), taken as one microbatch per GPU --
synthetic random codon batches already resident in HBM.  One step = fwd + CE + bwd + (RCCL all-reduce) + AdamW.
Rank 0 prints ONE JSON line.

--path engine (default): the DataParallelStep sequence (native engine calls, bucketed
RCCL all-reduce during the backward).  --path trainer: the per-microbatch sequence of
codonlm_amd.training.loop (model(xb, yb) through the nn.Module API, loss.backward()
through autograd, the stats read behind an event, the rank-consistent group control,
FusedAdamW + LambdaLR), i.e. what `python -m codonlm_amd.train_codon_lm` runs per step.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "genomics-lm_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CONFIGS = {
    # BASELINE.json configs[3] (the metric's config); the others are the remaining GPU configs
    "c4": dict(n_layer=12, n_head=8, n_embd=512, block_size=1024, batch=32, swiglu=False, rope=False, kv=None),
    # per-GPU microbatch of every config = the sequences of one optimizer step of the reference's
    # own config for that shape (batch_size x grad_accum_steps): C4 2 x 16 (runs/2025-11-05_tiny_
    # 12L8H_d512_e5/log.txt:30-31), C2 4 x 64 (configs/stage2.5_master.yaml:25-26), C3 8 x 32
    # (configs/bench_b8_gqa4.yaml:1,6), C5 4 x 32 (configs/stage2.6_large_scaling.yaml:25-26)
    "c2": dict(n_layer=6, n_head=4, n_embd=256, block_size=512, batch=256, swiglu=False, rope=False, kv=None),
    "c3": dict(n_layer=10, n_head=8, n_embd=384, block_size=512, batch=256, swiglu=True, rope=True, kv=4),
    # stage2.6_large_scaling + termination head + multi-offset heads: the trainer's
    # full objective (loop.py:1075-1112) on packed BOS..EOS,SEP segments
    "c5": dict(n_layer=10, n_head=8, n_embd=384, block_size=512, batch=128, swiglu=False, rope=False, kv=None,
               offsets=(2, 4, 8, 16, 32), term=True),
}
# CPU-baseline batch per BASELINE.md §3 (the reference's default per-device batch)
CPU_BATCH = {"c4": 2, "c2": 4, "c3": 4, "c5": 4}
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip table)
PEAK_HBM_GBS = 8000.0


def flops_per_token(c, V=68):
    d, L, T = c["n_embd"], c["n_layer"], c["block_size"]
    hd = d // c["n_head"]
    kvd = (c["kv"] or c["n_head"]) * hd
    hid = int(8 * d // 3) if c["swiglu"] else 4 * d
    mlp = 3 * d * hid if c["swiglu"] else 2 * d * hid
    n_mm = L * (d * (d + 2 * kvd) + d * d + mlp) + d * V
    n_mm += (5 * d if c.get("term") else 0) + len(c.get("offsets", ())) * (2 * d * d + d * V)  # aux heads
    # 6*N_mm + 6*L*d*T (causal-exact attention, no recompute)
    return 6 * n_mm + 6 * L * d * T


def probe_pass(kind, run, first, n):
    """Run n untimed steps with the live probe on `kind`; returns (work, ms, launches, bytes)."""
    import ctypes as C
    from codonlm_amd import _lib as L
    L.lib.cg_probe_enable(kind)
    for i in range(n):
        run(first + i)
    torch.cuda.synchronize()
    w, ms, k = C.c_double(0), C.c_double(0), C.c_longlong(0)
    L.check(L.lib.cg_probe_read(C.byref(w), C.byref(ms), C.byref(k)), "cg_probe_read")
    nbytes = C.c_double(0)
    L.check(L.lib.cg_probe_bytes(C.byref(nbytes)), "cg_probe_bytes")
    L.lib.cg_probe_enable(0)
    return w.value, ms.value, k.value, nbytes.value


def _cpu_share():
    """Host threads this process may use: its affinity set, capped by a cgroup CPU quota."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, math.floor(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


def _cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(cfg_name, c, budget_s=80.0):
    """The fp32 CPU restatement of the same training step (oracle.CpuTrainer: fwd + CE + bwd +
    AdamW, pinned to the reference), BASELINE.md §3 protocol: the reference's default per-device
    batch, synthetic codons from default_rng(1337), 20 warmup + 100 measured steps -- bounded by a
    time budget: warmup stops after 10% of it, and at least 20 steps are measured whenever a step
    takes under ~3.6 s (the counts run and the step-time spread are reported), on every host
    thread this process may use.  Rank 0 only."""
    from oracle import tinygpt_oracle as O
    threads = _cpu_share()
    torch.set_num_threads(threads)
    cfg = O.OracleConfig(vocab_size=68, block_size=c["block_size"], n_layer=c["n_layer"], n_head=c["n_head"],
                         n_embd=c["n_embd"], n_kv_head=c["kv"], use_swiglu=c["swiglu"], use_rope=c["rope"],
                         dropout=0.1, label_smoothing=0.05)
    tr = O.CpuTrainer(cfg, O.synthetic_params(cfg, seed=1), lr=3e-4, wd=0.05)
    Bc, T = CPU_BATCH[cfg_name], c["block_size"]
    rng = np.random.default_rng(1337)
    tok = rng.integers(4, 68, size=(Bc, T + 1))
    x, y = tok[:, :-1], tok[:, 1:]
    t0 = time.perf_counter()
    nw = 0
    while nw < 20 and (nw == 0 or time.perf_counter() - t0 < 0.1 * budget_s):
        tr.step(x, y, dropout_seed=nw)
        nw += 1
    times = []
    t1 = time.perf_counter()
    while len(times) < 100 and (len(times) < 2 or time.perf_counter() - t1 < 0.9 * budget_s):
        s = time.perf_counter()
        tr.step(x, y, dropout_seed=1000 + len(times))
        times.append(time.perf_counter() - s)
    step = float(np.mean(times))
    return {"value": Bc * T / step, "unit": "tokens/s", "cores": threads, "kind": "port", "batch": Bc,
            "cpu": _cpu_model(), "host_cpus": os.cpu_count(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "warmup": nw, "measured": len(times), "ms_per_step": round(step * 1e3, 1),
            "ms_per_step_std": round(float(np.std(times)) * 1e3, 1),
            "ms_per_step_min_max": [round(min(times) * 1e3, 1), round(max(times) * 1e3, 1)],
            "sample": f"{len(times)} timed fp32 steps (after {nw} warmup) of the same model at B={Bc}, T={T} "
                      f"(the reference's default per-device batch, BASELINE.md §3), {threads} threads"}


def _head():
    try:
        return subprocess.run(["git", "-C", str(ROOT), "rev-parse", "--short=12", "HEAD"], capture_output=True,
                              text=True, timeout=10).stdout.strip() or None
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--path", default="engine", choices=["engine", "trainer", "forward"],
                    help="engine: the DP training step; trainer: the trainer's per-microbatch sequence; "
                         "forward: the eval-mode batched forward of extract_embeddings / query_model")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-roofline", action="store_true")
    ap.add_argument("--attn-bwd", default="auto", choices=["auto", "split", "fused"],
                    help="bf16 attention backward (cg_model_opts.attn_bwd_algo; A/B runs, default automatic)")
    ap.add_argument("--engine-opt", action="append", default=[], metavar="NAME=VALUE",
                    help="a cg_model_opts field for A/B runs (repeatable; all zero = the measured defaults)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from codonlm_amd import TinyGPT
    from codonlm_amd.optim import FusedAdamW
    from codonlm_amd.training.ddp import DataParallelStep

    engine_opts = {"attn_bwd_algo": {"auto": 0, "split": 1, "fused": 2}[args.attn_bwd]}
    for kv in args.engine_opt:
        k, v = kv.split("=", 1)
        engine_opts[k] = int(v)
    c = dict(CONFIGS[args.config])
    B = args.batch or c["batch"]
    T = c["block_size"]
    torch.manual_seed(1337)
    aux = bool(c.get("offsets") or c.get("term"))
    model = TinyGPT(68, T, n_layer=c["n_layer"], n_head=c["n_head"], n_embd=c["n_embd"], dropout=0.1,
                    label_smoothing=0.05, n_kv_head=c["kv"], use_swiglu=c["swiglu"], use_rope=c["rope"],
                    termination_aux=bool(c.get("term")), multi_offset_targets=list(c.get("offsets", ())) or None,
                    compute_dtype=args.dtype, device=dev,
                    engine_opts=engine_opts)
    if world > 1:  # identical replicas
        dist.broadcast(model.flat_parameters(), 0)
    model.train()
    model._seed_rank = rank
    opt = FusedAdamW(model, lr=3e-4, weight_decay=0.05)
    stepper = DataParallelStep(model, opt)

    rng = np.random.default_rng(1337 + rank)
    nbuf = 4
    batches = []
    for j in range(nbuf):
        tok = rng.integers(4, 68, size=(B, T + 1))
        if aux:  # packed segments: BOS ... EOS, SEP every ~330 tokens
            tok[:, 0] = 1
            for p0 in range(330 + j, T + 1, 330):
                tok[:, p0 - 1], tok[:, p0] = 2, 3
                if p0 + 1 <= T:
                    tok[:, p0 + 1] = 1
        batches.append((torch.from_numpy(tok[:, :-1].copy()).to(dev), torch.from_numpy(tok[:, 1:].copy()).to(dev)))

    from codonlm_amd.training import objectives as obj
    offw = {k: 1.0 / len(c["offsets"]) for k in c.get("offsets", ())}

    def objective(xb, yb):
        """The trainer's objective (loop.py:1075-1112) through the model API."""
        if not aux:
            _, loss = model(xb, yb)
            return loss
        _, loss, auxo = model(xb, yb, return_aux=True)
        total = loss
        if offw:
            off_total, _, _ = obj.multi_offset_lm_loss(auxo["offset_logits"], yb, offw, label_smoothing=0.05,
                                                       return_counts=True)
            total = total + off_total
        if c.get("term"):
            labels = obj.termination_distance_bucket_labels(yb, stop_ids=(2,))
            total = total + 0.1 * obj.termination_aux_loss(auxo["termination_logits"], labels)
        return total

    fwd_only = args.path == "forward"
    if fwd_only:
        model.eval()

        def run(i):
            xb, _ = batches[i % nbuf]
            with torch.no_grad():
                logits, _ = model(xb)
            return logits[:1, :1].float().sum()
    elif args.path == "engine" and not aux:
        def run(i):
            xb, yb = batches[i % nbuf]
            return stepper.step(xb, yb, seed=1000 + i)
    else:
        # the trainer's per-microbatch sequence (training/loop.py one_pass, gacc = 1)
        from codonlm_amd.training.loop import AccumulationHealth, cosine_lr_lambda
        from codonlm_amd.training.stepper import GroupController, control_group
        health = AccumulationHealth()
        ctl = GroupController(gacc=1, health=health, world=world, group=control_group(world))
        sched = torch.optim.lr_scheduler.LambdaLR(opt, cosine_lr_lambda(10, 10 ** 6, 3e-4, 3e-5))
        host = torch.empty(2, dtype=torch.float32, pin_memory=True)

        def run(i):
            xb, yb = batches[i % nbuf]
            opt.zero_grad(set_to_none=True)
            loss = objective(xb, yb)
            host.copy_(torch.stack([loss.detach().float(), yb.ne(0).sum().float()]), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            handles = []
            if world > 1:
                model._bucket_hook = stepper.bucket_hook(handles)
            loss.backward()
            ev.synchronize()
            v = host.tolist()
            abort, _ = ctl.agree(not math.isfinite(v[0]))
            for h in handles:
                h.wait()
            if abort:
                health.abort_group(opt)
                return loss
            health.record_finite_microbatch()
            opt.step(grad_scale=1.0 / world)
            health.complete_group()
            sched.step()
            return loss

    for i in range(args.warmup):
        loss = run(i)
    torch.cuda.synchronize()
    # find the dominant MFMA kernel with short untimed probe passes (rank-local, no comms)
    from codonlm_amd import _lib as L
    probes = {}
    dominant = 0
    if not args.no_kernel_roofline and args.dtype == "bf16":
        nxt = args.warmup
        for kind in (L.PROBE_GEMM_PERS, L.PROBE_GEMM_DW_GROUPED, L.PROBE_GEMM_DW, L.PROBE_GEMM_FWD, L.PROBE_GEMM_DX,
                     L.PROBE_ATTN_FWD, L.PROBE_ATTN_DQ, L.PROBE_ATTN_DKDV, L.PROBE_ATTN_BWD, L.PROBE_DW_SLAB):
            probes[kind] = probe_pass(kind, run, nxt, 2)
            nxt += 2
        # the roofline kernel is the MFMA kernel class with the most device time per step (a class =
        # one kernel template: the persistent fwd/dX GEMM with all its epilogue instantiations, the
        # grouped dW with its tile variants, each attention kernel)
        dominant = max(tuple(L.PROBE_KERNELS), key=lambda k: probes[k][1])
        if world > 1:  # all ranks probe the same kernel in the probe window
            t = torch.tensor([dominant], device=dev)
            dist.broadcast(t, 0)
            dominant = int(t.item())
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = run(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # The timed region above carries no probe.  The roofline kernel is then timed live in a
    # separate window of `probe_steps` further steps: HIP events on the launch stream around 1
    # launch in `every` of that class -- the smallest every >= 4 coprime to the class's launches
    # per step, so the sampled launches cycle through every product of the step (a class spans
    # several shapes).
    live = None
    per_step = max(1, probes[dominant][2] // 2) if dominant else 1
    every = next(e for e in range(4, 64) if math.gcd(e, per_step) == 1)
    probe_steps = max(8, 2 * every)
    if dominant:
        import ctypes as C
        L.lib.cg_probe_sample(every)
        L.lib.cg_probe_enable(dominant)
        for i in range(probe_steps):
            run(args.warmup + args.steps + i)
        torch.cuda.synchronize()
        w, ms, k = C.c_double(0), C.c_double(0), C.c_longlong(0)
        L.check(L.lib.cg_probe_read(C.byref(w), C.byref(ms), C.byref(k)), "cg_probe_read")
        nbytes = C.c_double(0)
        L.check(L.lib.cg_probe_bytes(C.byref(nbytes)), "cg_probe_bytes")
        L.lib.cg_probe_enable(0)
        live = (w.value, ms.value, k.value, nbytes.value)
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.item())

    tokens = world * B * T * args.steps
    value = tokens / elapsed
    ftok = flops_per_token(c) // (3 if fwd_only else 1)  # a forward is one third of a training step
    if fwd_only:
        metric = f"codon tokens/sec batched forward (eval, {args.config})"
    elif args.config == "c4":
        metric = "codon tokens/sec training step, 12L8H d512 seq1024"
    else:
        metric = f"codon tokens/sec training step ({args.config})"
    result = {
        "metric": metric,
        "value": round(value, 1),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (uniform random codons 4..67, pre-staged in HBM: the trainer's one per-batch gather "
                "launch, cg_gather_windows, is not in the timed step; random-init weights)",
        "config": {"workload": f"TinyGPT {c['n_layer']}L{c['n_head']}H d{c['n_embd']} T{T} V68 "
                               + ("eval forward" if fwd_only else "train step")
                               + (" + 5 offset heads + termination head (trainer objective)" if aux and not fwd_only
                                  else ""),
                   "model": "TinyGPT (genomics-lm src/codonlm)", "global_batch": world * B, "seq_len": T,
                   "micro_batch_per_gpu": B, "parallelism": f"dp{world}", "dropout": 0.1,
                   "label_smoothing": 0.05, "sep_mask": True,
                   "path": args.path if (not aux or fwd_only) else "trainer",
                   **({"attn_bwd": args.attn_bwd} if args.attn_bwd != "auto" else {}),
                   **({"engine_opts": {k: v for k, v in engine_opts.items() if v}}
                      if any(v for v in engine_opts.values()) else {})},
        "final_loss": round(final_loss, 4),
        "model_flops_per_token": ftok,
        "step_mfma_frac": round(value / world * ftok / (PEAK_BF16_TFLOPS * 1e12), 4),
    }
    if rank == 0 and live is not None and live[1] > 0:
        work, ms, k, abytes = live
        ach = work / (ms * 1e-3) / 1e12
        result["roofline"] = {"kernel": L.PROBE_NAMES[dominant],
                              "rocprof_kernels": [p + "*" for p in L.PROBE_KERNELS[dominant]],
                              "bound": "mfma", "achieved": round(ach, 2),
                              "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / PEAK_BF16_TFLOPS, 4),
                              "traffic": None, "launches": k, "avg_launch_us": round(ms / k * 1e3, 2),
                              "ms_per_step_probe": round(probes[dominant][1] / 2, 3),
                              "algorithmic_bytes_per_launch": round(abytes / k) if k else None,
                              "launches_per_step": per_step,
                              "measured": f"HIP events on the launch stream around 1 in {every} launches of the "
                                          f"kernel class ({per_step} launches per step) over {probe_steps} steps run "
                                          "after the timed region (the timed region carries no probe); achieved = "
                                          "sum of their algorithmic FLOPs (2MNK) / sum of their device time"}
        # HBM bytes per launch of the same kernel class from the committed rocprofv3 PMC passes
        # (FETCH_SIZE x2 + WRITE_SIZE, gfx950 corrections; tools/pmc_traffic.py); attached only for
        # the same config, batch and kernel class, newest round first, with the commit the counters
        # were collected at
        name = L.PROBE_NAMES[dominant]
        cands = sorted(ROOT.glob(f"profiles/round*/pmc_traffic_{args.config}_{name}.json"), reverse=True)
        cands += [ROOT / "profiles" / "round2" / f"pmc_traffic_{args.config}.json"]
        for tr in cands:
            if not tr.exists():
                continue
            t = json.loads(tr.read_text())
            if t.get("probe") != name or t.get("micro_batch", 16) != B:  # (files before round 5: B=16)
                continue
            if args.path != "engine":  # the passes ran the engine's training step (tools/prof_round3.sh)
                continue
            result["roofline"]["traffic"] = t["hbm_bytes_per_launch"]
            result["roofline"]["traffic_unit"] = "HBM bytes/launch (PMC)"
            result["roofline"]["traffic_source"] = (f"{tr.relative_to(ROOT)} "
                                                    f"(collected at {t.get('commit')}; this run {_head()})")
            result["roofline"]["traffic_algorithmic"] = t.get("algorithmic_bytes_per_launch")
            break
        # MFMA classes priced in TFLOP/s against the bf16 peak; the HBM-bound slab reduce of a k-split
        # grouped dW in GB/s against the HBM peak
        result["kernels"] = {}
        for kk, v in probes.items():
            if not v[2]:
                continue
            ent = {"ms_per_step": round(v[1] / 2, 3), "launches_per_step": v[2] // 2}
            if kk == L.PROBE_DW_SLAB:
                gbs = v[3] / (v[1] * 1e-3) / 1e9 if v[1] > 0 else None
                ent.update({"gbps": round(gbs, 1) if gbs else None,
                            "frac_hbm": round(gbs / PEAK_HBM_GBS, 4) if gbs else None})
            else:
                ent.update({"tflops": round(v[0] / (v[1] * 1e-3) / 1e12, 1) if v[1] > 0 else None,
                            "frac": round(v[0] / (v[1] * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4) if v[1] > 0 else None})
            result["kernels"][L.PROBE_NAMES[kk]] = ent
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.config, c)
        # the two sides run different batches (the CPU at the reference's default per-device batch, the
        # GPU at one optimizer step's sequences as one microbatch): both stated, so the ratio is read
        # with its batch-size effect in view
        result["cpu_baseline"]["gpu_batch"] = B
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
