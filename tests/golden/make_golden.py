#!/usr/bin/env python3
"""Generate golden parity vectors by running the REAL reference in the build container.

Run (build container only -- /root/reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports AvishaiBarnoy/genomics-lm read-only from /root/reference
(src/codonlm/model_tiny_gpt.py TinyGPT, src/codonlm/training/objectives.py,
torch.optim.AdamW as configured at src/codonlm/training/loop.py:681-731) and
writes small .npz fixtures (inputs + outputs only, never reference code) next
to this script.  Weights come from oracle.tinygpt_oracle.synthetic_params
(deterministic numpy generator) and are loaded into the reference TinyGPT via
load_state_dict, so the large-geometry fixture does not need to store them.
"""
from __future__ import annotations

import json
import math
import os
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
REF = os.environ.get("GENOMICS_LM_REFERENCE", "/root/reference")
sys.path.insert(0, REF)

from oracle.tinygpt_oracle import OracleConfig, synthetic_params  # noqa: E402
from src.codonlm.model_tiny_gpt import TinyGPT  # noqa: E402  (reference)
from src.codonlm.training import objectives as ref_obj  # noqa: E402  (reference)


def packed_tokens(rng, B, T, pad_tail=0, sep_every=0):
    """Random codons 4..67; optional BOS/EOS/SEP packing and a PAD tail."""
    t = rng.integers(4, 68, size=(B, T + 1)).astype(np.int64)
    if sep_every:
        for b in range(B):
            t[b, 0] = 1
            pos = sep_every + int(rng.integers(0, 5))
            while pos + 1 < T + 1:
                t[b, pos - 1] = 2
                t[b, pos] = 3
                if pos + 1 < T + 1:
                    t[b, pos + 1] = 1
                pos += sep_every + int(rng.integers(0, 7))
    if pad_tail:
        t[-1, T + 1 - pad_tail:] = 0
    return t[:, :-1].copy(), t[:, 1:].copy()


def build_ref(cfg: OracleConfig, params):
    m = TinyGPT(
        cfg.vocab_size, cfg.block_size, n_layer=cfg.n_layer, n_head=cfg.n_head,
        n_embd=cfg.n_embd, dropout=cfg.dropout, use_checkpoint=False,
        label_smoothing=cfg.label_smoothing, sep_id=cfg.sep_id,
        tie_embeddings=cfg.tie_embeddings, n_kv_head=cfg.n_kv_head, use_sdpa=False,
        loss_weights=cfg.loss_weights, termination_aux=cfg.termination_aux,
        termination_n_classes=cfg.termination_n_classes,
        multi_offset_targets=cfg.multi_offset_targets or None,
        use_swiglu=cfg.use_swiglu, use_rope=cfg.use_rope,
    )
    sd = {k: torch.from_numpy(v) for k, v in params.items()}
    if cfg.tie_embeddings:
        sd["head.weight"] = sd["tok_emb.weight"]
    missing, unexpected = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if not (k.endswith("attn.mask") or k == "loss_weights")]
    assert not missing and not unexpected, (missing, unexpected)
    m.eval()
    return m


def run_case(name, cfg: OracleConfig, B, T, *, seed=1234, pad_tail=0, sep_every=0,
             store_params=True, store_grads=True, adamw=False, window=None):
    rng = np.random.default_rng(seed + 7)
    params = synthetic_params(cfg, seed=seed)
    idx, tgt = packed_tokens(rng, B, T, pad_tail=pad_tail, sep_every=sep_every)
    model = build_ref(cfg, params)
    out = {"config": np.array(json.dumps(cfg.to_dict())), "param_seed": np.array(seed),
           "idx": idx, "targets": tgt}
    x = torch.from_numpy(idx)
    y = torch.from_numpy(tgt)
    need_aux = cfg.termination_aux or bool(cfg.multi_offset_targets)
    if need_aux:
        logits, loss, aux = model(x, y, return_aux=True, attention_window=window)
    else:
        logits, loss = model(x, y, attention_window=window)
        aux = {}
    out["logits"] = logits.detach().numpy()
    out["loss"] = np.array(loss.item(), dtype=np.float64)
    out["greedy"] = logits.detach().argmax(-1).numpy()
    top2 = torch.topk(logits.detach(), 2, dim=-1).values
    out["top2_margin"] = (top2[..., 0] - top2[..., 1]).numpy()
    if "termination_logits" in aux:
        out["termination_logits"] = aux["termination_logits"].detach().numpy()
    for k, v in aux.get("offset_logits", {}).items():
        out[f"offset_logits_{k}"] = v.detach().numpy()
    loss.backward()
    if store_grads:
        for k, p in model.named_parameters():
            g = p.grad if p.grad is not None else torch.zeros_like(p)
            out[f"grad/{k}"] = g.detach().numpy().copy()
    else:
        for k, p in model.named_parameters():
            g = p.grad if p.grad is not None else torch.zeros_like(p)
            out[f"gradsum/{k}"] = np.array([float(g.double().sum()), float(g.double().abs().sum()),
                                             float(g.double().pow(2).sum())])
    if store_params:
        for k, v in params.items():
            out[f"param/{k}"] = v
    # hidden states + pooling (iter_hidden_states, extract_embeddings._pool_state)
    with torch.no_grad():
        states = list(model.iter_hidden_states(x, attention_window=window))
    for layer, h in states:
        if store_params or layer == "final":
            out[f"hidden/{layer}"] = h.numpy()
    nonpad = x.ne(0)
    content = list(range(4, 68))
    for layer, h in states:
        for mode in ("mean_nonpad", "mean_content", "eos"):
            if mode == "mean_nonpad":
                mask = nonpad
            elif mode == "mean_content":
                mask = torch.zeros_like(nonpad)
                for tok in content:
                    mask |= x.eq(tok)
            if mode == "eos":
                pos = nonpad.long().sum(1).sub(1).clamp_min(0)
                pooled = h[torch.arange(h.size(0)), pos]
            else:
                w = mask.to(h.dtype).unsqueeze(-1)
                pooled = (h * w).sum(1) / w.sum(1).clamp_min(1.0)
            out[f"pooled/{layer}/{mode}"] = pooled.numpy()
    # attention mask (build_attention_mask)
    am = model.build_attention_mask(x, window)
    if am is not None:
        out["attn_mask"] = am[:, 0].numpy()
    if adamw:
        # one AdamW step exactly as loop.py builds it: every TinyGPT tensor lands in the
        # backbone group (lr=lr, weight_decay=0.05) because the fast-group name match
        # (loop.py:689) never hits tok_emb/pos_emb.
        lr, wd = 3e-4, 0.05
        opt = torch.optim.AdamW([{"params": [p for p in model.parameters()], "lr": lr,
                                  "weight_decay": wd}])
        opt.step()
        opt.zero_grad(set_to_none=True)
        logits2, loss2 = model(x, y)
        loss2.backward()
        opt.step()
        for k, p in model.named_parameters():
            out[f"adamw2/{k}"] = p.detach().numpy().copy()
        out["adamw_lr"] = np.array(lr)
        out["adamw_wd"] = np.array(wd)
    np.savez_compressed(HERE / f"{name}.npz", **out)
    print(f"[golden] {name}: loss={loss.item():.6f} keys={len(out)}")


def objectives_case():
    rng = np.random.default_rng(99)
    y = rng.integers(4, 68, size=(3, 40)).astype(np.int64)
    y[0, 10] = 2
    y[0, 11] = 3
    y[1, 5] = 50  # TAA? (id of stop codons is fine either way)
    y[1, 20] = 2
    y[2, 30:] = 0
    y[2, 7] = 3
    y = torch.from_numpy(y)
    out = {"y": y.numpy()}
    for k in (2, 3, 4, 8):
        out[f"offset_mask_{k}"] = ref_obj.offset_target_mask(y, k).numpy()
    stop_ids = (2, 52, 54, 60)
    out["stop_ids"] = np.array(stop_ids)
    out["term_labels"] = ref_obj.termination_distance_bucket_labels(y, stop_ids=stop_ids).numpy()
    torch.manual_seed(5)
    logits = torch.randn(3, 40, 68)
    out["mo_logits"] = logits.numpy()
    tot, losses = ref_obj.multi_offset_lm_loss(logits, y, {2: 0.5, 4: 0.25}, label_smoothing=0.05)
    out["mo_total"] = np.array(float(tot))
    for k, v in losses.items():
        out[f"mo_loss_{k}"] = np.array(float(v))
    tl = torch.randn(3, 40, 5)
    out["term_logits"] = tl.numpy()
    cw = torch.tensor([1.0, 2.0, 1.5, 1.0, 0.5])
    out["term_cw"] = cw.numpy()
    out["term_loss"] = np.array(float(ref_obj.termination_aux_loss(tl, torch.from_numpy(out["term_labels"]), cw)))
    # LambdaLR schedule as built in loop.py:770-779 (re-evaluated through LambdaLR itself)
    lrs = []
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.AdamW([p], lr=3e-4)
    W, S, min_lr, base = 10, 50, 1e-5, 3e-4

    def lam(s):
        if s < max(1, W):
            return float(s + 1) / max(1, W)
        prog = (s - max(1, W)) / max(1, S - max(1, W))
        return (min_lr / base) + (1 - min_lr / base) * 0.5 * (1.0 + math.cos(math.pi * prog))
    sch = torch.optim.lr_scheduler.LambdaLR(opt, lam)
    for _ in range(S + 3):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        sch.step()
    out["lr_schedule"] = np.array(lrs)
    np.savez_compressed(HERE / "objectives.npz", **out)
    print("[golden] objectives")


AUX_OBJECTIVE = dict(offset_weights={2: 0.5, 4: 0.25}, term_weight=0.1, stop_ids=(2, 52),
                     bucket_edges=(0, 3, 10, 30), term_class_weights=[1.0, 2.0, 1.5, 1.0, 0.5])


def aux_objective_case():
    """The codon trainer's full objective with aux heads (loop.py:1075-1112): next-codon CE +
    multi_offset_lm_loss + w_t * termination_aux_loss, backpropagated through the reference
    TinyGPT; all parameter grads (incl. offset_projs / termination_head) are stored."""
    cfg = OracleConfig(vocab_size=68, block_size=64, n_layer=1, n_head=4, n_embd=64, sep_id=3,
                       label_smoothing=0.05, termination_aux=True, multi_offset_targets=[2, 4],
                       loss_weights=[1.0, 1.0, 3.0] + [1.0] * 65)
    rng = np.random.default_rng(4321)
    params = synthetic_params(cfg, seed=77)
    idx, tgt = packed_tokens(rng, 2, 64, pad_tail=6, sep_every=14)
    tgt[0, 20] = 52  # a stop codon id inside a segment
    model = build_ref(cfg, params)
    model.train()  # dropout=0: train mode only matters for the trainer path
    x, y = torch.from_numpy(idx), torch.from_numpy(tgt)
    A = AUX_OBJECTIVE
    logits, loss, aux = model(x, y, return_aux=True)
    lw = model.loss_weights if not torch.all(model.loss_weights == 1.0).item() else None
    off_total, off_losses = ref_obj.multi_offset_lm_loss(aux["offset_logits"], y, A["offset_weights"],
                                                         label_smoothing=cfg.label_smoothing, loss_weights=lw)
    labels = ref_obj.termination_distance_bucket_labels(y, stop_ids=A["stop_ids"], bucket_edges=A["bucket_edges"])
    cw = torch.tensor(A["term_class_weights"])
    term_loss = ref_obj.termination_aux_loss(aux["termination_logits"], labels, class_weights=cw)
    total = loss + off_total + A["term_weight"] * term_loss
    total.backward()
    out = {"config": np.array(json.dumps(cfg.to_dict())), "objective": np.array(json.dumps(
        {k: (list(v) if isinstance(v, tuple) else ({str(a): b for a, b in v.items()} if isinstance(v, dict) else v))
         for k, v in A.items()})), "idx": idx, "targets": tgt,
        "loss": np.array(loss.item()), "total": np.array(total.item()), "term_loss": np.array(term_loss.item()),
        "term_labels": labels.numpy(), "termination_logits": aux["termination_logits"].detach().numpy()}
    for k, v in off_losses.items():
        out[f"offset_loss_{k}"] = np.array(v.item())
    for k, v in aux["offset_logits"].items():
        out[f"offset_logits_{k}"] = v.detach().numpy()
    for k, v in params.items():
        out[f"param/{k}"] = v
    for k, p in model.named_parameters():
        out[f"grad/{k}"] = (p.grad if p.grad is not None else torch.zeros_like(p)).detach().numpy().copy()
    np.savez_compressed(HERE / "aux_objective.npz", **out)
    print(f"[golden] aux_objective: total={total.item():.6f}")


def data_order_case():
    """Batch order of the reference loaders (data_loading.py:332-486): a fixed-window NPZ
    through build_codon_lm_dataloaders (seeded RandomSampler) and a dynamic NPZ through the
    BucketBatchSampler + dynamic collate; stored as the batches the reference yields."""
    import tempfile
    from src.codonlm.data_loading import PackedDataset, build_codon_lm_dataloaders  # noqa: E402 (reference)
    out = {}
    with tempfile.TemporaryDirectory() as td:
        n, T = 23, 5
        X = np.arange(n * T, dtype=np.int32).reshape(n, T) % 60 + 4
        X[:, 0] = np.arange(n) + 4
        Y = (X + 1).astype(np.int32)
        fx = os.path.join(td, "fixed.npz")
        np.savez_compressed(fx, X=X, Y=Y)
        ds = PackedDataset([fx])
        for seed in (11, 12):
            tl, vl, _, _ = build_codon_lm_dataloaders(ds, ds, {"batch_size": 4, "dataloader_seed": seed})
            out[f"fixed_seed{seed}_x"] = np.concatenate([xb.numpy() for xb, _ in tl])
            out[f"fixed_seed{seed}_sizes"] = np.array([xb.shape[0] for xb, _ in tl])
        out["fixed_val_x"] = np.concatenate([xb.numpy() for xb, _ in vl])
        rng = np.random.default_rng(5)
        lens = rng.integers(3, 20, size=37)
        flat = rng.integers(4, 68, size=int(lens.sum())).astype(np.int32)
        fd = os.path.join(td, "dyn.npz")
        np.savez_compressed(fd, X=flat, lengths=lens)
        dds = PackedDataset([fd])
        tl, vl, sampler, _ = build_codon_lm_dataloaders(dds, dds, {"batch_size": 3, "dataloader_seed": 9,
                                                                    "bucket_batching": True, "n_buckets": 4})
        xs, ys = [], []
        for xb, yb in tl:
            xs.append(xb.numpy())
            ys.append(yb.numpy())
        out["dyn_flat"], out["dyn_lengths"] = flat, lens
        out["dyn_bucket_batches"] = np.array(len(xs))
        for i, (xa, ya) in enumerate(zip(xs, ys)):
            out[f"dyn_bucket_x_{i}"], out[f"dyn_bucket_y_{i}"] = xa, ya
        vx = [xb.numpy() for xb, _ in vl]
        out["dyn_val_batches"] = np.array(len(vx))
        for i, xa in enumerate(vx):
            out[f"dyn_val_x_{i}"] = xa
    np.savez_compressed(HERE / "data_order.npz", **out)
    print("[golden] data_order")


def main():
    torch.set_num_threads(8)
    only = set(sys.argv[1:])
    if only:  # regenerate selected fixtures only, e.g. `make_golden.py aux_objective`
        if "aux_objective" in only:
            aux_objective_case()
        if "data_order" in only:
            data_order_case()
        if "objectives" in only:
            objectives_case()
        return
    c1 = OracleConfig(vocab_size=68, block_size=64, n_layer=2, n_head=4, n_embd=64,
                      label_smoothing=0.05, sep_id=3)
    run_case("mha_gelu_sep", c1, 2, 64, sep_every=20, pad_tail=9, adamw=True)
    c2 = OracleConfig(vocab_size=68, block_size=64, n_layer=2, n_head=4, n_embd=64, n_kv_head=2,
                      use_rope=True, use_swiglu=True, sep_id=3,
                      loss_weights=[1.0, 1.0, 3.0] + [1.0] * 45 + [3.0, 3.0, 1.0, 3.0] + [1.0] * 16)
    run_case("gqa_rope_swiglu_w", c2, 2, 64, sep_every=25, pad_tail=5)
    c3 = OracleConfig(vocab_size=69, block_size=48, n_layer=2, n_head=2, n_embd=64,
                      label_smoothing=0.1, sep_id=None, tie_embeddings=False)
    run_case("untied_causal", c3, 3, 48)
    c4 = OracleConfig(vocab_size=68, block_size=64, n_layer=1, n_head=4, n_embd=64, sep_id=3,
                      termination_aux=True, multi_offset_targets=[2, 4])
    run_case("aux_heads", c4, 2, 64, sep_every=18)
    c5 = OracleConfig(vocab_size=68, block_size=128, n_layer=1, n_head=4, n_embd=192, n_kv_head=2,
                      use_rope=True, use_swiglu=True, sep_id=3, label_smoothing=0.05)
    run_case("hd48_gqa", c5, 2, 128, sep_every=40)
    c6 = OracleConfig(vocab_size=68, block_size=64, n_layer=1, n_head=4, n_embd=64, sep_id=3)
    run_case("window8", c6, 2, 64, sep_every=30, window=8)
    # C4 layer geometry (d512, H8, hd64, T1024) -- weights regenerated from the seed
    c7 = OracleConfig(vocab_size=68, block_size=1024, n_layer=1, n_head=8, n_embd=512, sep_id=3,
                      label_smoothing=0.05)
    run_case("c4_layer", c7, 1, 1024, sep_every=330, store_params=False, store_grads=False)
    objectives_case()
    aux_objective_case()
    data_order_case()


if __name__ == "__main__":
    main()
