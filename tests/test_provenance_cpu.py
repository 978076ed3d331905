"""The frozen dataset-manifest contract used by ``extract_embeddings --manifest``
(reference: src/codonlm/dataset_manifest.py, src/codonlm/evaluation_provenance.py), on a
synthetic manifest built here: a valid manifest binds, and each tamper the reference rejects
is rejected."""
import copy
import json
from pathlib import Path

import numpy as np
import pytest

from codonlm_amd import provenance as P

SPECIAL = ["<PAD>", "<BOS_CDS>", "<EOS_CDS>", "<SEP>"]


def _write_dataset(root: Path):
    itos = SPECIAL + ["AAA", "AAC", "AAG", "AAT"]
    (root / "itos.txt").write_text("\n".join(itos) + "\n")
    files = {"vocabulary": root / "itos.txt"}
    rng = np.random.default_rng(0)
    for split in P.SPLITS:
        x = rng.integers(0, len(itos), size=(4, 16), dtype=np.int64)
        np.savez(root / f"{split}_bs16.npz", X=x, Y=x)
        files[f"{split}_tokens"] = root / f"{split}_bs16.npz"
    for name in ("source_metadata", "source_dna", "fragment_metadata", "leakage_audit", "train_packing_metadata",
                 "val_packing_metadata", "test_packing_metadata"):
        (root / f"{name}.json").write_text(json.dumps({"name": name}))
        files[name] = root / f"{name}.json"
    arts = {n: {"path": p.name, "role": n, "bytes": p.stat().st_size, "sha256": P.file_sha256(p)}
            for n, p in files.items()}
    manifest = {
        "schema": {"name": P.SCHEMA_NAME, "version": P.SCHEMA_VERSION},
        "dataset": {"source_record_count": 10, "scientific_valid": True},
        "split_policy": {"record_counts": {"train": 6, "val": 2, "test": 2},
                         "requested_fractions": {"val": 0.2, "test": 0.2}, "scientific_valid": True,
                         "effective_group_by": "genome"},
        "leakage_audit": {"status": "passed"},
        "vocabulary": {"size": len(itos), "sha256": P.file_sha256(files["vocabulary"]),
                       "special_tokens": {t: i for i, t in enumerate(SPECIAL)}},
        "sources": {}, "tokenization": {"ambiguous_codon_policy": "drop"},
        "packing": {"mode": "fixed", "transition_policy": "exactly_once"},
        "reproducibility": {"split_seed": 1, "packing_seed": 2},
        "artifacts": arts,
    }
    manifest["dataset"]["id"] = P.dataset_identity(manifest)
    return manifest


def _save(root, manifest):
    path = root / "manifest.json"
    path.write_text(json.dumps(manifest))
    return path


def test_manifest_binds_and_checkpoint_matches(tmp_path):
    m = _write_dataset(tmp_path)
    _, prov = P.bind_dataset_manifest(_save(tmp_path, m))
    assert prov["status"] == "frozen_manifest_verified" and prov["dataset_id"] == m["dataset"]["id"]
    cfg = {"dataset_manifest": {"dataset_id": m["dataset"]["id"]}, "vocabulary": {"sha256": m["vocabulary"]["sha256"]}}
    assert P.bind_checkpoint_dataset(cfg, prov)["status"] == "checkpoint_manifest_verified"
    assert P.bind_checkpoint_dataset({}, None)["status"] == "legacy_checkpoint_unverified"
    with pytest.raises(P.EvaluationProvenanceError, match="requires an explicit"):
        P.bind_checkpoint_dataset(cfg, None)
    with pytest.raises(P.EvaluationProvenanceError, match="identity mismatch"):
        P.bind_checkpoint_dataset({"dataset_manifest": {"dataset_id": "x"}}, prov)


@pytest.mark.parametrize("tamper", ["id", "counts", "leak", "vocab_hash", "token_range", "special"])
def test_manifest_tampering_is_rejected(tmp_path, tamper):
    m = _write_dataset(tmp_path)
    bad = copy.deepcopy(m)
    if tamper == "id":
        bad["dataset"]["id"] = "0" * 64
    elif tamper == "counts":
        bad["split_policy"]["record_counts"]["train"] = 7
    elif tamper == "leak":
        bad["leakage_audit"]["status"] = "failed"
    elif tamper == "vocab_hash":
        bad["vocabulary"]["sha256"] = "f" * 64
    elif tamper == "special":
        bad["vocabulary"]["special_tokens"]["<SEP>"] = 5
    elif tamper == "token_range":
        x = np.full((4, 16), 99, dtype=np.int64)
        np.savez(tmp_path / "val_bs16.npz", X=x, Y=x)
        p = tmp_path / "val_bs16.npz"
        bad["artifacts"]["val_tokens"].update(bytes=p.stat().st_size, sha256=P.file_sha256(p))
    if tamper != "id":
        bad["dataset"]["id"] = P.dataset_identity(bad)
    with pytest.raises(P.DatasetManifestError):
        P.bind_dataset_manifest(_save(tmp_path, bad))
