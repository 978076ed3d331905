"""Host logic of the MI355X trainer on CPU: rank-consistent group control under gloo
(world_size 2), data-parallel batch sharding, the primary-config contract, the
vocabulary-remapping transfer load, and the optimizer-state interchange with
torch.optim.AdamW (the reference trainer's optimizer)."""
import os
import socket

import numpy as np
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


# --------------------------------------------------------------------------- group control
def _ctl_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from codonlm_amd.training.loop import AccumulationHealth
        from codonlm_amd.training.stepper import GroupController, control_group
        grp = control_group(world)
        health = AccumulationHealth()
        # skewed clocks: rank 0 passes the wall-time limit at microbatch 7, rank 1 never does
        tick = {"i": 0}
        clock = (lambda: 100.0 if tick["i"] >= 7 else 0.0) if rank == 0 else (lambda: 0.0)
        ctl = GroupController(gacc=3, health=health, world=world, group=grp, wall_limit_s=10.0, clock=clock, t0=0.0)
        log, scales, consumed = [], [], 0
        pending = 0
        for i in range(12):
            tick["i"] = i
            sync = ctl.completes_group(i == 11)
            nonfinite = rank == 1 and i == 4  # only rank 1 sees a NaN loss
            abort, stop = ctl.agree(nonfinite)
            log.append((i, sync, abort, stop))
            if abort:
                health.abort_group(type("O", (), {"zero_grad": lambda self, set_to_none=True: None})())
                pending = 0
                continue
            pending += 10 + rank  # this rank's non-PAD tokens
            health.record_finite_microbatch()
            if health.active_microbatches == 3:
                scales.append(1.0 / (health.active_microbatches * world))
                consumed += int(ctl.sum([pending])[0])
                pending = 0
                health.complete_group()
            if stop:
                break
        out[rank] = (log, scales, consumed, health.aborted_groups)
    finally:
        dist.destroy_process_group()


def test_group_control_is_rank_consistent_gloo():
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_ctl_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    (log0, sc0, cons0, ab0), (log1, sc1, cons1, ab1) = out[0], out[1]
    # identical decisions on both ranks
    assert log0 == log1
    assert sc0 == sc1 == [pytest.approx(1 / 6)] * 2
    assert cons0 == cons1 == 2 * 3 * (10 + 11)  # two committed groups, tokens summed over ranks
    assert ab0 == ab1 == 1
    # rank 1's NaN at microbatch 4 aborted the group on BOTH ranks
    assert log0[4][2] is True and not any(a for i, _, a, _ in log0 if i != 4)
    # rank 0's wall-time limit (microbatch 7) stopped both ranks there
    assert log0[-1][0] == 7 and log0[-1][3] is True
    # the overlap decision: microbatch 2 closes group 1 (gacc 3); after the abort at 4 the
    # next group is 5, 6, 7
    syncs = [i for i, s, _, _ in log0 if s]
    assert 2 in syncs and 7 in syncs and 1 not in syncs


# --------------------------------------------------------------------------- sharding
class _FakeDS:
    def __init__(self, n):
        self.n, self.device, self.is_dynamic = n, "cpu", False

    def __len__(self):
        return self.n

    seq_lengths = None


def test_loader_shards_train_floor_eval_cover():
    from codonlm_amd.data_loading import DeviceBatchLoader
    ds = _FakeDS(23)  # 6 batches of 4
    for world in (1, 2, 4):
        train = [DeviceBatchLoader(ds, 4, rank=r, world=world).shard() for r in range(world)]
        assert all(len(t) == 6 // world for t in train)  # equal counts: matched collectives
        ev = [DeviceBatchLoader(ds, 4, rank=r, world=world, drop_remainder=False).shard() for r in range(world)]
        assert sorted(k for e in ev for k in e) == list(range(6))  # every val batch exactly once
        for r in range(world):
            assert all(k % world == r for k in ev[r])


# --------------------------------------------------------------------------- primary contract
def _primary_cfg():
    from codonlm_amd.training import primary_contract as P
    root = P.DATASETS["genome"]["root"]
    cfg = dict(P.COMMON_VALUES)
    cfg.update(primary_training_contract={"schema": P.SCHEMA_NAME, "version": P.SCHEMA_VERSION,
                                          "release": P.RELEASE, "dataset_freeze_id": P.DATASET_FREEZE_ID,
                                          "role": "primary", "protocol": "genome",
                                          "dataset_id": P.DATASETS["genome"]["dataset_id"]},
               dataset_manifest=f"{root}/manifest.json", itos_path=f"{root}/itos.txt",
               train_npz=f"{root}/train_bs512.npz", val_npz=f"{root}/val_bs512.npz",
               test_npz=f"{root}/test_bs512.npz", seed=2027, dataloader_seed=2027, epochs=10,
               max_time_minutes=None, run_id="corrected-codonlm-v1-genome-seed2027")
    return cfg


def test_primary_contract_validation():
    from codonlm_amd.training.primary_contract import validate_primary_training_config
    cfg = _primary_cfg()
    res = validate_primary_training_config(cfg)
    assert res["run_id"] == "corrected-codonlm-v1-genome-seed2027" and cfg["device"] == "mps"
    for key, bad in (("n_layer", 12), ("device", "cuda"), ("seed", 7), ("lr", 1e-3)):
        c = dict(cfg, **{key: bad})
        with pytest.raises(ValueError):
            validate_primary_training_config(c)
    with pytest.raises(ValueError, match="undeclared"):
        validate_primary_training_config(dict(cfg, compute_dtype="bf16"))


def test_resolve_device_contract(monkeypatch):
    from codonlm_amd.training import loop
    with pytest.raises(ValueError):
        loop.resolve_device({"device": "tpu"})
    with pytest.raises(RuntimeError, match="CPU"):
        loop.resolve_device({"device": "cpu"})
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError, match="no MI355X"):
            loop.resolve_device({"device": "mps"})


# --------------------------------------------------------------------------- transfer
def test_transfer_remaps_vocabulary_rows():
    from codonlm_amd import TinyGPT
    from codonlm_amd.training.checkpoint import load_transfer_state_dict
    torch.manual_seed(0)
    src = TinyGPT(70, 32, n_layer=1, n_head=2, n_embd=64, device="cpu")
    dst = TinyGPT(68, 64, n_layer=1, n_head=2, n_embd=64, device="cpu")
    src_itos = [f"t{i}" for i in range(70)]
    dst_itos = [f"t{i}" for i in range(68)]
    dst_itos[5], dst_itos[6] = "t6", "t5"  # two tokens swapped in the target vocabulary
    dst_itos[7] = "new"                    # one token the source does not have
    before = dst.state_dict()["tok_emb.weight"].clone()
    sd = {k: v.clone() for k, v in src.state_dict().items()}
    rep = load_transfer_state_dict(dst, sd, source_itos=src_itos, target_itos=dst_itos)
    emb = dst.state_dict()["tok_emb.weight"]
    assert torch.equal(emb[5], sd["tok_emb.weight"][6]) and torch.equal(emb[6], sd["tok_emb.weight"][5])
    assert torch.equal(emb[7], before[7])  # unknown token keeps its init
    assert torch.equal(emb[10], sd["tok_emb.weight"][10])
    assert "tok_emb.weight:67" in rep["loaded_rows"]
    # block_size 32 -> 64: position rows copied by the token map (the reference's behaviour for
    # any row-count mismatch when both itos lists are known), the rest kept
    assert any(r.startswith("pos_emb.weight:") for r in rep["loaded_rows"])
    assert "blocks.0.attn.query.weight" in rep["loaded_exact"]
    assert "blocks.0.attn.mask" in rep["skipped"]  # (1,1,32,32) vs (1,1,64,64)
    assert torch.equal(dst.state_dict()["blocks.0.attn.query.weight"], sd["blocks.0.attn.query.weight"])


# --------------------------------------------------------------------------- optimizer state
def _ref_adamw(model, lr, lr_emb, wd):
    """torch.optim.AdamW with the reference's param groups (loop.py:681-731)."""
    fast = [p for n, p in model.named_parameters() if "offset_projs" in n or "termination_head" in n]
    back = [p for n, p in model.named_parameters() if not ("offset_projs" in n or "termination_head" in n)]
    return torch.optim.AdamW([{"params": fast, "lr": lr_emb, "weight_decay": 0.0},
                              {"params": back, "lr": lr, "weight_decay": wd}])


def test_optimizer_state_interchanges_with_torch_adamw():
    from codonlm_amd import TinyGPT
    from codonlm_amd.optim import FusedAdamW
    torch.manual_seed(1)
    m = TinyGPT(68, 32, n_layer=2, n_head=2, n_embd=64, termination_aux=True, multi_offset_targets=[2],
                device="cpu")
    opt = FusedAdamW(m, lr=1e-3, weight_decay=0.05, lr_embedding=3e-3)
    opt.exp_avg.copy_(torch.randn_like(opt.exp_avg))
    opt.exp_avg_sq.copy_(torch.rand_like(opt.exp_avg_sq))
    opt.step_count = 7
    sd = opt.state_dict()
    # ours -> the reference trainer's optimizer
    ref = _ref_adamw(m, 1e-3, 3e-3, 0.05)
    ref.load_state_dict({"state": sd["state"], "param_groups": sd["param_groups"]})
    named = dict(m.named_parameters())
    for g in ref.param_groups:
        for p in g["params"]:
            st = ref.state[p]
            assert int(st["step"]) == 7
            assert torch.equal(st["exp_avg"], opt._moment_view(opt.exp_avg, p))
    assert len(ref.state) == len(named)
    # the reference trainer's optimizer state -> ours (no flat_state in its checkpoints)
    opt2 = FusedAdamW(m, lr=1e-3, weight_decay=0.05, lr_embedding=3e-3)
    rsd = ref.state_dict()
    assert "flat_state" not in rsd
    opt2.load_state_dict(rsd)
    assert opt2.step_count == 7
    for p in named.values():  # (alignment / pad gaps of the flat buffer carry no state)
        assert torch.equal(opt2._moment_view(opt2.exp_avg, p), opt._moment_view(opt.exp_avg, p))
        assert torch.equal(opt2._moment_view(opt2.exp_avg_sq, p), opt._moment_view(opt.exp_avg_sq, p))
