"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports every
symbol include/codonlm_hip.h declares, and the host-only entry points (layout,
workspace sizing) give a reference-compatible module without touching a GPU."""
import re
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parent.parent


def _declared_functions():
    text = (ROOT / "include" / "codonlm_hip.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(cg_[a-z0-9_]+)\s*\(", text)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    from codonlm_amd import _lib
    declared = _declared_functions()
    assert len(declared) >= 25
    for name in declared:
        assert hasattr(_lib.lib, name), name
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature"
    assert _lib.lib.cg_version().decode().startswith("codonlm_hip")


def test_ctypes_struct_mirrors_match_the_library():
    """Every struct the ctypes binding mirrors has the size the loaded library was built with
    (cg_struct_bytes), so a field added on one side only fails here, not as a misread argument."""
    import ctypes
    from codonlm_amd import _lib as L
    mirrors = {"cg_gemm_desc": L.GemmDesc, "cg_dw_product": L.DwProduct, "cg_dw_group": L.DwGroup,
               "cg_reduce_job": L.ReduceJob, "cg_reduce_batch": L.ReduceBatch,
               "cg_transpose_item": L.TransposeItem, "cg_transpose_batch": L.TransposeBatch,
               "cg_adamw_segment": L.AdamwSegment, "cg_model_cfg": L.ModelCfg,
               "cg_param_entry": L.ParamEntry, "cg_model": L.Model, "cg_model_opts": L.ModelOpts}
    for name, cls in mirrors.items():
        assert L.lib.cg_struct_bytes(name.encode()) == ctypes.sizeof(cls), name
    assert L.lib.cg_struct_bytes(b"nope") == 0


def test_product_path_never_imports_oracle():
    pkg = ROOT / "genomics-lm_amd" / "codonlm_amd"
    for f in pkg.rglob("*.py"):
        src = f.read_text()
        assert "oracle" not in re.findall(r"^\s*(?:from|import)\s+(\S+)", src, flags=re.M), f
        assert "tinygpt_oracle" not in src, f


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    import importlib
    import codonlm_amd._lib as L
    monkeypatch.setattr(L, "LIB_PATH", tmp_path / "nope.so")
    with pytest.raises(L.LibraryError):
        L._load()
    importlib.reload(L)  # restore


@pytest.mark.parametrize("kw", [dict(), dict(n_kv_head=2, use_rope=True, use_swiglu=True),
                                dict(tie_embeddings=False, sep_id=None),
                                dict(termination_aux=True, multi_offset_targets=[2, 4])])
def test_state_dict_and_init_match_reference_layout(kw):
    """Same keys/shapes/order as the reference TinyGPT, and torch.manual_seed(s) gives the
    reference's initial weights (init drawn in the reference's module order)."""
    from codonlm_amd import TinyGPT
    from oracle import tinygpt_oracle as O
    cfg = O.OracleConfig(vocab_size=68, block_size=64, n_layer=2, n_head=4, n_embd=64,
                         n_kv_head=kw.get("n_kv_head"), use_rope=kw.get("use_rope", False),
                         use_swiglu=kw.get("use_swiglu", False), tie_embeddings=kw.get("tie_embeddings", True),
                         termination_aux=kw.get("termination_aux", False),
                         multi_offset_targets=kw.get("multi_offset_targets", []))
    torch.manual_seed(7)
    m = TinyGPT(68, 64, n_layer=2, n_head=4, n_embd=64, device="cpu", **kw)
    sd = m.state_dict()
    shapes = O.param_shapes(cfg)
    for k, shp in shapes.items():
        assert tuple(sd[k].shape) == tuple(shp), k
    extra = set(sd) - set(shapes)
    allowed = {"loss_weights", "head.weight"} | {f"blocks.{i}.attn.mask" for i in range(2)}
    assert extra <= allowed, extra
    assert tuple(sd["blocks.0.attn.mask"].shape) == (1, 1, 64, 64)
    # params are views into the flat buffer; grads view the flat grad buffer
    flat = m.flat_parameters()
    for name, p in m.named_parameters():
        assert p.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr(), name
        assert p.grad is not None and p.grad.shape == p.shape


def test_reference_init_bitwise(tmp_path):
    import sys
    ref = Path("/root/reference")
    if not ref.exists():
        pytest.skip("reference tree only present in the build container")
    sys.path.insert(0, str(ref))
    try:
        from src.codonlm.model_tiny_gpt import TinyGPT as Ref
    except Exception as e:  # pragma: no cover
        pytest.skip(f"reference not importable: {e}")
    finally:
        sys.path.remove(str(ref))
    from codonlm_amd import TinyGPT
    torch.manual_seed(11)
    r = Ref(68, 32, n_layer=2, n_head=4, n_embd=64, n_kv_head=2, use_swiglu=True, use_rope=True)
    torch.manual_seed(11)
    m = TinyGPT(68, 32, n_layer=2, n_head=4, n_embd=64, n_kv_head=2, use_swiglu=True, use_rope=True, device="cpu")
    for k, v in r.state_dict().items():
        assert torch.equal(v, m.state_dict()[k]), k


def test_workspace_and_layout_sizes():
    from codonlm_amd.engine import EngineConfig, param_layout
    import ctypes as C
    from codonlm_amd import _lib as L
    c4 = EngineConfig(vocab_size=68, block_size=1024, n_layer=12, n_head=8, n_embd=512, dtype="bf16")
    lay, total = param_layout(c4)
    n_real = sum((r * cc if cc else r) for _, _, _, r, cc, _ in lay)
    assert n_real == 38_388_736  # C4 parameter count (tied head counted once)
    assert total >= n_real
    offs = [o for _, _, o, _, _, _ in lay]
    assert offs == sorted(offs)
    ws = L.lib.cg_model_workspace_bytes(C.byref(c4.to_c()), 16, 1024)
    assert 1e9 < ws < 16e9
