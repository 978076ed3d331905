"""world_size-2 data parallelism on the REAL engine (marker ``gpu``).

tests/test_ddp_cpu.py checks the bucket host logic with a stand-in engine; here two ranks run the
native engine and its bucket hooks for real: both processes share the one MI355X of the box and
talk over gloo (CUDA tensors; RCCL needs a GPU per rank, the driver's 8-GPU scaling run covers
it).  After one synchronised microbatch every rank must hold the rank-SUM of the gradients over
the whole flat buffer -- every bucket all-reduced, including the tied head's contribution that
phase 0 writes into the embedding rows and the grouped-dW blocks whose hooks fire per group --
equal to one process accumulating both shards (loop.py:1233-1238 semantics, 1/world in AdamW).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = dict(n_layer=3, n_head=4, n_embd=128, dropout=0.0, label_smoothing=0.05, compute_dtype="bf16")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shards(world):
    rng = np.random.default_rng(100)
    out = []
    for _ in range(world):
        t = torch.from_numpy(rng.integers(4, 68, size=(4, 129)))
        t[:, 40] = 3  # a SEP boundary in every row
        out.append((t[:, :-1].contiguous(), t[:, 1:].contiguous()))
    return out


def _model(TinyGPT):
    torch.manual_seed(7)
    m = TinyGPT(68, 128, device="cuda:0", **CFG)
    m.train()
    return m


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from codonlm_amd import TinyGPT
        from codonlm_amd.optim import FusedAdamW
        from codonlm_amd.training.ddp import DataParallelStep, bucket_ranges
        shards = _shards(world)
        m = _model(TinyGPT)
        step = DataParallelStep(m, FusedAdamW(m, lr=1e-3))
        x, y = (t.cuda() for t in shards[rank])
        _, handles = step.microbatch(x, y, seed=3, accumulate=False, sync=True)
        for h in handles:
            h.wait()
        torch.cuda.synchronize()
        res = {"grads": m.flat_grads().detach().cpu().clone(), "handles": len(handles),
               "buckets": sum(1 for b, e in bucket_ranges(m).values() if e > b)}
        if rank == 0:  # one process, both shards accumulated (no hooks)
            r = _model(TinyGPT)
            rs = DataParallelStep(r, FusedAdamW(r, lr=1e-3))
            for j, (xj, yj) in enumerate(shards):
                rs.microbatch(xj.cuda(), yj.cuda(), seed=3, accumulate=j > 0, sync=False)
            torch.cuda.synchronize()
            res["ref"] = r.flat_grads().detach().cpu().clone()
        dist.barrier()
        out[rank] = res
    finally:
        dist.destroy_process_group()


def test_ddp_two_ranks_real_engine_gloo():
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    g0, g1, ref = out[0]["grads"], out[1]["grads"], out[0]["ref"]
    assert out[0]["handles"] == out[0]["buckets"] >= 3, (out[0]["handles"], out[0]["buckets"])
    assert torch.equal(g0, g1), "ranks disagree after the bucket all-reduces"
    # the rank-sum of per-shard gradients equals one process accumulating both shards
    scale = ref.abs().max().item()
    err = (g0 - ref).abs().max().item()
    assert err <= 1e-5 * scale, (err, scale)
    assert ref.abs().sum() > 0
