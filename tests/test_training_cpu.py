"""Host-side trainer logic vs the reference (no GPU): batch order, accumulation counters,
warmup / offset-weight resolution and the LR schedule (loop.py, data_loading.py)."""
import numpy as np
import pytest

from conftest import load_golden


def _dl():
    from codonlm_amd import data_loading
    return data_loading


def _loop():
    from codonlm_amd.training import loop
    return loop


def test_fixed_window_order_matches_reference_dataloader():
    D = _dl()
    _, g = load_golden("data_order")
    X = np.arange(23 * 5, dtype=np.int32).reshape(23, 5) % 60 + 4
    X[:, 0] = np.arange(23) + 4
    for seed in (11, 12):
        order, bounds = D.epoch_batches(23, 4, shuffle=True, seed=seed)
        assert np.array_equal(X[order], g[f"fixed_seed{seed}_x"])
        assert np.array_equal(np.diff(bounds), g[f"fixed_seed{seed}_sizes"])
    order, _ = D.epoch_batches(23, 4, shuffle=False)
    assert np.array_equal(X[order], g["fixed_val_x"])


def _collate(flat, starts, lens, rows):
    """dynamic_lm_collate_fn (data_loading.py:380-393) on host arrays."""
    Tout = int(lens[rows].max()) - 1
    x = np.zeros((len(rows), Tout), np.int64)
    y = np.zeros_like(x)
    for i, r in enumerate(rows):
        s = flat[starts[r]: starts[r] + lens[r]]
        x[i, : len(s) - 1] = s[:-1]
        y[i, : len(s) - 1] = s[1:]
    return x, y


def test_bucket_batches_match_reference_sampler():
    D = _dl()
    _, g = load_golden("data_order")
    flat, lens = g["dyn_flat"], g["dyn_lengths"]
    starts = np.concatenate([[0], np.cumsum(lens[:-1])])
    order, bounds = D.epoch_batches(len(lens), 3, shuffle=True, seed=9, lengths=lens, n_buckets=4)
    assert len(bounds) - 1 == int(g["dyn_bucket_batches"])
    for i in range(len(bounds) - 1):
        rows = order[bounds[i]: bounds[i + 1]]
        x, y = _collate(flat, starts, lens, rows)
        assert np.array_equal(x, g[f"dyn_bucket_x_{i}"]) and np.array_equal(y, g[f"dyn_bucket_y_{i}"]), i
    order, bounds = D.epoch_batches(len(lens), 3)
    for i in range(int(g["dyn_val_batches"])):
        x, _ = _collate(flat, starts, lens, order[bounds[i]: bounds[i + 1]])
        assert np.array_equal(x, g[f"dyn_val_x_{i}"])


def test_accumulation_health_counters():
    loop = _loop()

    class Opt:
        zeroed = 0

        def zero_grad(self, set_to_none=True):
            Opt.zeroed += 1

    h = loop.AccumulationHealth()
    h.record_finite_microbatch()
    h.record_finite_microbatch()
    assert h.abort_group(Opt()) == 2 and Opt.zeroed == 1
    assert h.metrics_dict() == {"active_microbatches": 0, "nonfinite_microbatches": 1, "aborted_groups": 1,
                                "discarded_finite_microbatches": 2}
    assert h.exceeds_limit(0) and not h.exceeds_limit(1) and not h.exceeds_limit(-1)
    with pytest.raises(ValueError):
        h.complete_group()
    h.record_finite_microbatch()
    assert h.state_dict()["active_microbatches"] == 0
    h2 = loop.AccumulationHealth()
    h2.load_state_dict(h.state_dict())
    assert h2.aborted_groups == 1 and h2.active_microbatches == 0


def test_warmup_offsets_and_schedule():
    loop = _loop()
    assert loop.resolve_warmup_steps({}, 10) == 200
    assert loop.resolve_warmup_steps({"warmup_fraction": 0.1}, 55) == 6
    assert loop.resolve_warmup_steps({"warmup_fraction": 0.0}, 55) == 0
    with pytest.raises(ValueError):
        loop.resolve_warmup_steps({"warmup_fraction": 0.1, "warmup_steps": 3}, 10)
    with pytest.raises(ValueError):
        loop.resolve_warmup_steps({}, 0)
    assert loop.normalize_offset_weights([2, 4]) == {2: 0.5, 4: 0.5}
    assert loop.normalize_offset_weights([2, 4], {"2": 1.0}) == {2: 1.0, 4: 0.0}
    assert loop.normalize_offset_weights([2, 4], [0.3, 0.7]) == {2: 0.3, 4: 0.7}
    assert loop.normalize_offset_weights([2, 4], 0.2) == {2: 0.2, 4: 0.2}
    with pytest.raises(ValueError):
        loop.normalize_offset_weights([2, 4], [1.0])
    _, g = load_golden("objectives")
    lam = loop.cosine_lr_lambda(10, 50, 3e-4, 1e-5)
    np.testing.assert_allclose([3e-4 * lam(s) for s in range(len(g["lr_schedule"]))], g["lr_schedule"],
                               rtol=1e-12)


def test_build_model_kwargs_mapping():
    """cfg -> TinyGPT kwargs (loop.py:396-405,559-579) without touching a GPU."""
    loop = _loop()
    lw = [1.0] * 68
    for tok in ("<EOS_CDS>", "TAA", "TAG", "TGA"):
        lw[loop.STOI[tok]] = 3.0
    assert loop.STOI["<EOS_CDS>"] == 2 and loop.STOI["TAA"] == 52 and loop.STOI["TGA"] == 60
    assert len(loop.VOCAB) == 68
