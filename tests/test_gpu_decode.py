"""KV-cached incremental decoding vs the reference's full re-forward.

Teacher-forced: the prompt prefix is prefilled, then the golden sequence's next tokens are
decoded one at a time; every step's logits must equal the REFERENCE's logits at that
position (golden fixtures hold the reference TinyGPT's logits for the whole sequence, whose
causal mask makes position t depend on tokens 0..t only) -- SEP segments, RoPE + GQA +
SwiGLU, untied heads and a local window included.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from test_gpu_model import DEV, make_model, _idx

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", ["mha_gelu_sep", "gqa_rope_swiglu_w", "untied_causal", "hd48_gqa", "window8"])
def test_decode_matches_reference_logits(case):
    cfgd, g = load_golden(case)
    m, cfg, _ = make_model(cfgd, g)
    m.eval()
    x, _ = _idx(g)
    B, T = x.shape
    window = 8 if case == "window8" else None
    ref = g["logits"]
    scale = max(1.0, float(np.abs(ref).max()))
    p0 = 5
    cache = m.engine.new_kv_cache(B, cfg.block_size)
    logits = cache.prefill(x[:, :p0], window=window)
    assert float(np.abs(logits.cpu().numpy() - ref[:, :p0]).max()) <= 1e-4 * scale
    worst = 0.0
    for t in range(p0, T):
        step = cache.decode(x[:, t]).cpu().numpy()
        worst = max(worst, float(np.abs(step - ref[:, t]).max()))
    assert worst <= 1e-4 * scale, (worst, scale)
    with pytest.raises(ValueError):
        if T == cfg.block_size:
            cache.decode(x[:, 0])
        else:
            raise ValueError("cache not full for this case")


def test_decode_bf16_close_to_full_forward():
    cfgd, g = load_golden("mha_gelu_sep")
    m, cfg, _ = make_model(cfgd, g, dtype="bf16")
    m.eval()
    x, _ = _idx(g)
    B, T = x.shape
    with torch.no_grad():
        full, _ = m(x)
    full = full.float().cpu().numpy()
    cache = m.engine.new_kv_cache(B, cfg.block_size)
    cache.prefill(x[:, :3])
    worst = 0.0
    for t in range(3, T):
        worst = max(worst, float(np.abs(cache.decode(x[:, t]).cpu().numpy() - full[:, t]).max()))
    assert worst <= 3e-2 * max(1.0, float(np.abs(full).max())), worst


def test_cached_greedy_equals_recompute_greedy():
    """query_model.greedy_generate: cached path == re-forward path, across the block_size slide."""
    from codonlm_amd import query_model as Q
    cfgd, g = load_golden("mha_gelu_sep")
    m, cfg, _ = make_model(cfgd, g)
    m.eval()
    ctx = [1, 20, 33, 3, 1, 45]
    a = Q.greedy_generate(m, torch.device(DEV), ctx, max_new=80, kv_cache=True)
    b = Q.greedy_generate(m, torch.device(DEV), ctx, max_new=80, kv_cache=False)
    assert a == b


@pytest.mark.parametrize("topk", [0, 5])
def test_cached_sampling_equals_recompute_sampling(topk):
    """query_model.generate (the CLI's --mode generate): the KV-cached loop draws the same tokens
    as the reference's re-forward loop from the same device RNG state (fp32 engine: the two
    paths' logits agree to ~1e-6, far inside any multinomial bin), across the block_size slide,
    with temperature and top-k."""
    from codonlm_amd import query_model as Q
    cfgd, g = load_golden("mha_gelu_sep")
    m, cfg, _ = make_model(cfgd, g)
    m.eval()
    ctx = [1, 20, 33, 3, 1, 45]
    out = []
    for kv in (True, False):
        torch.manual_seed(1234)
        out.append(Q.generate(m, torch.device(DEV), ctx, max_new=80, temperature=0.8, topk=topk, kv_cache=kv))
    assert out[0] == out[1]
    assert len(out[0]) == min(len(ctx) + 80, cfg.block_size)
