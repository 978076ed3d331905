"""world_size-2 gloo test of the data-parallel step's host logic on CPU.

DataParallelStep's buckets must tile the flat gradient buffer exactly (each backward phase
of the native engine completes one contiguous range), every bucket must be all-reduced
once per optimizer step right after its phase is enqueued, and the optimizer must see the
rank-average (grad_scale = 1/world).  The native engine is replaced by a CPU
stand-in that writes rank-dependent gradients phase by phase.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeEngine:
    def __init__(self, model, rank, log):
        self.model, self.rank, self.log = model, rank, log

    def forward(self, idx, targets, training, seed):
        return None, torch.tensor(1.0)

    def backward(self, accumulate=False, bucket_hook=None):
        from codonlm_amd.training.ddp import bucket_ranges
        rng = bucket_ranges(self.model)
        g = self.model.flat_grads()
        order = ["head"] + list(range(self.model.n_layer - 1, -1, -1)) + ["embed"]
        for name in order:
            b, e = rng[name]
            g[b:e] = float(self.rank + 1) * (1 + torch.arange(b, e, dtype=torch.float32) % 7)
            self.log.append(name)
            if bucket_hook:
                bucket_hook(name)


class _FakeOpt:
    def __init__(self):
        self.scales = []

    def step(self, grad_scale=1.0):
        self.scales.append(grad_scale)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from codonlm_amd import TinyGPT
        from codonlm_amd.training.ddp import DataParallelStep, bucket_ranges
        m = TinyGPT(68, 32, n_layer=3, n_head=4, n_embd=64, device="cpu")
        log = []
        m._engine = _FakeEngine(m, rank, log)
        opt = _FakeOpt()
        step = DataParallelStep(m, opt)
        step.step(None, None, seed=0)
        # coverage: buckets tile [0, total) without overlap
        rng = bucket_ranges(m)
        spans = sorted(rng.values())
        cov = 0
        for b, e in spans:
            assert b == cov
            cov = e
        assert cov == m.flat_grads().numel()
        g = m.flat_grads()
        idx = torch.arange(g.numel(), dtype=torch.float32)
        expected = (1.0 + 2.0) * (1 + idx % 7)  # sum over ranks (the 1/world is in grad_scale)
        out[rank] = (bool(torch.allclose(g, expected)), opt.scales, log)
    finally:
        dist.destroy_process_group()


def test_ddp_buckets_allreduce_gloo():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        ok, scales, log = out[r]
        assert ok, f"rank {r}: gradients are not the rank-sum"
        assert scales == [pytest.approx(1.0 / world)]
        assert log[0] == "head" and log[-1] == "embed" and log[1:-1] == [2, 1, 0]
