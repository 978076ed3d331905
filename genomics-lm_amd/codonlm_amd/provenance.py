"""Frozen dataset manifests and checkpoint provenance for embedding extraction.

Restates the reference's fail-closed contracts that ``scripts/extract_embeddings.py:227-230``
applies when ``--manifest`` is given:

* ``src/codonlm/dataset_manifest.py`` -- content-addressed manifest: schema, dataset identity
  (sha256 of the canonical JSON without path / compatibility keys, :45-64), split policy, leakage
  audit, vocabulary and required artifacts (:87-189), artifact / source sizes and sha256, special
  token ids and token-id bounds of every split (:147-189).
* ``src/codonlm/evaluation_provenance.py`` -- ``bind_dataset_manifest`` (:27-61, provenance record
  of the manifest, its vocabulary and any bound artifacts) and ``bind_checkpoint_dataset``
  (:64-111, a corrected checkpoint must name the same dataset and vocabulary).

Host-side file checks only; nothing here runs on the GPU.
"""
from __future__ import annotations

import copy
import hashlib
import json
from pathlib import Path
from typing import Any, Mapping

import numpy as np

SCHEMA_NAME = "codonlm_dataset_manifest"
SCHEMA_VERSION = 1
SPLITS = ("train", "val", "test")
REQUIRED_ARTIFACTS = ("train_tokens", "val_tokens", "test_tokens", "vocabulary", "source_metadata", "source_dna",
                      "fragment_metadata", "leakage_audit", "train_packing_metadata", "val_packing_metadata",
                      "test_packing_metadata")


class DatasetManifestError(ValueError):
    """An unsupported or inconsistent dataset manifest (dataset_manifest.py:17)."""


class EvaluationProvenanceError(ValueError):
    """Inputs that cannot be bound to one frozen dataset (evaluation_provenance.py:12)."""


def file_sha256(path: Path) -> str:
    h = hashlib.sha256()
    with Path(path).open("rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def dataset_identity(manifest: Mapping[str, Any]) -> str:
    """sha256 of the manifest without its id, compatibility keys and paths (:45-64)."""
    payload = copy.deepcopy(dict(manifest))
    payload.get("dataset", {}).pop("id", None)
    for key in ("train", "val", "test", "datasets", "genome_sources"):
        payload.pop(key, None)
    payload.get("vocabulary", {}).pop("itos_path", None)
    for group in ("artifacts", "sources"):
        for entry in payload.get(group, {}).values():
            entry.pop("path", None)
    blob = json.dumps(payload, sort_keys=True, separators=(",", ":"), allow_nan=False).encode("utf-8")
    return hashlib.sha256(blob).hexdigest()


def _req(mapping: Mapping, key: str, context: str):
    if key not in mapping:
        raise DatasetManifestError(f"missing {context}.{key}")
    return mapping[key]


def manifest_artifact_path(manifest: Mapping, manifest_path: Path, name: str) -> Path:
    entry = _req(_req(manifest, "artifacts", "manifest"), name, "artifacts")
    path = Path(_req(entry, "path", "artifact"))
    return path if path.is_absolute() else Path(manifest_path).parent / path


def read_itos_strict(path: Path) -> tuple:
    """training/vocabulary.py load_itos: non-empty, no blank or duplicate tokens."""
    if not path.exists():
        raise DatasetManifestError(f"vocabulary not found: {path}")
    tokens = tuple(line.strip() for line in path.read_text().splitlines())
    if not tokens or any(not t for t in tokens) or len(set(tokens)) != len(tokens):
        raise DatasetManifestError(f"vocabulary has empty or duplicate tokens: {path}")
    return tokens


def token_bounds(path: Path) -> tuple:
    """(min, max) token id of a split (training/vocabulary.py:125-142): the X/Y .npy sidecars when
    present (memory-mapped), else the X/Y arrays of the npz shard.  Loaded without pickle."""
    x_side = path.with_name(f"{path.stem}_X.npy")
    y_side = path.with_name(f"{path.stem}_Y.npy")
    arrays = []
    if x_side.exists():
        arrays.append(np.load(x_side, mmap_mode="r", allow_pickle=False))
        if y_side.exists():
            arrays.append(np.load(y_side, mmap_mode="r", allow_pickle=False))
    else:
        if not path.exists():
            raise DatasetManifestError(f"dataset shard not found: {path}")
        with np.load(path, allow_pickle=False) as data:
            if "X" not in data:
                raise DatasetManifestError(f"dataset shard has no X array: {path}")
            arrays = [np.asarray(data[n]) for n in ("X", "Y") if n in data]
    lo = min((int(a.min()) for a in arrays if a.size), default=None)
    hi = max((int(a.max()) for a in arrays if a.size), default=None)
    return lo, hi


def validate_dataset_manifest(manifest: Mapping, manifest_path: Path, *, verify_artifacts: bool = True):
    """dataset_manifest.py:87-189."""
    schema = _req(manifest, "schema", "manifest")
    if schema.get("name") != SCHEMA_NAME or schema.get("version") != SCHEMA_VERSION:
        raise DatasetManifestError(f"unsupported dataset manifest schema: {schema!r}")
    dataset = _req(manifest, "dataset", "manifest")
    declared = _req(dataset, "id", "dataset")
    computed = dataset_identity(manifest)
    if declared != computed:
        raise DatasetManifestError(f"dataset identity mismatch: declared={declared}, computed={computed}")
    policy = _req(manifest, "split_policy", "manifest")
    counts = _req(policy, "record_counts", "split_policy")
    if set(counts) != set(SPLITS) or any(int(counts[s]) < 0 for s in SPLITS):
        raise DatasetManifestError("split record_counts must contain non-negative train/val/test")
    if sum(int(counts[s]) for s in SPLITS) != int(dataset["source_record_count"]):
        raise DatasetManifestError("split record counts do not sum to dataset source_record_count")
    if any(not 0.0 <= float(v) < 1.0 for v in _req(policy, "requested_fractions", "split_policy").values()):
        raise DatasetManifestError("requested split fractions must be in [0, 1)")
    groups = policy.get("groups_by_split")
    if groups:
        sets = [set(groups[s]) for s in SPLITS]
        if any(sets[i] & sets[j] for i in range(3) for j in range(i + 1, 3)):
            raise DatasetManifestError("split groups overlap")
    scientific = bool(dataset.get("scientific_valid"))
    if scientific != bool(policy.get("scientific_valid")):
        raise DatasetManifestError("dataset and split_policy scientific_valid flags disagree")
    leakage = _req(manifest, "leakage_audit", "manifest")
    if scientific and (policy.get("effective_group_by") == "sequence" or policy.get("allow_sequence_split")
                       or leakage.get("status") != "passed" or leakage.get("homology_audit_skipped")
                       or leakage.get("exact_duplicate_override")):
        raise DatasetManifestError("unsafe preparation cannot be marked scientific_valid")
    vocabulary = _req(manifest, "vocabulary", "manifest")
    sources = _req(manifest, "sources", "manifest")
    _req(_req(manifest, "tokenization", "manifest"), "ambiguous_codon_policy", "tokenization")
    packing = _req(manifest, "packing", "manifest")
    reproducibility = _req(manifest, "reproducibility", "manifest")
    if packing.get("mode") not in {"fixed", "dynamic", "multi"}:
        raise DatasetManifestError("packing.mode must be fixed, dynamic, or multi")
    if packing.get("transition_policy") != "exactly_once":
        raise DatasetManifestError("packing transition_policy must be exactly_once")
    for name in ("split_seed", "packing_seed"):
        _req(reproducibility, name, "reproducibility")
    for tok in ("<PAD>", "<BOS_CDS>", "<EOS_CDS>", "<SEP>"):
        _req(vocabulary.get("special_tokens", {}), tok, "vocabulary.special_tokens")
    artifacts = _req(manifest, "artifacts", "manifest")
    for name in REQUIRED_ARTIFACTS:
        _req(artifacts, name, "artifacts")
    if not verify_artifacts:
        return manifest
    for name, src in sources.items():
        p = Path(src["path"])
        if not p.exists():
            raise DatasetManifestError(f"source {name} not found: {p}")
        if p.stat().st_size != int(src["bytes"]) or file_sha256(p) != src["sha256"]:
            raise DatasetManifestError(f"source {name} size / hash mismatch")
    for name in artifacts:
        p = manifest_artifact_path(manifest, manifest_path, name)
        if not p.exists():
            raise DatasetManifestError(f"artifact {name} not found: {p}")
        if p.stat().st_size != int(artifacts[name]["bytes"]) or file_sha256(p) != artifacts[name]["sha256"]:
            raise DatasetManifestError(f"artifact {name} size / hash mismatch: {p}")
    vocab_path = manifest_artifact_path(manifest, manifest_path, "vocabulary")
    tokens = read_itos_strict(vocab_path)
    if len(tokens) != int(vocabulary["size"]) or file_sha256(vocab_path) != vocabulary["sha256"]:
        raise DatasetManifestError("vocabulary size / hash does not match the artifact")
    for tok, tid in vocabulary["special_tokens"].items():
        if not 0 <= int(tid) < len(tokens) or tokens[int(tid)] != tok:
            raise DatasetManifestError(f"special token mapping is invalid for {tok}")
    for split in SPLITS:
        data_path = manifest_artifact_path(manifest, manifest_path, f"{split}_tokens")
        for suffix, role in (("_X.npy", "x_npy"), ("_Y.npy", "y_npy"), ("_lengths.npy", "lengths_npy")):
            if data_path.with_name(data_path.stem + suffix).exists() and f"{split}_{role}" not in artifacts:
                raise DatasetManifestError(f"untracked memory-map sidecar for {split}")
        lo, hi = token_bounds(data_path)
        if lo is not None and lo < 0:
            raise DatasetManifestError(f"{split} contains negative token IDs")
        if hi is not None and hi >= len(tokens):
            raise DatasetManifestError(f"{split} token IDs exceed vocabulary")
    return manifest


def load_dataset_manifest(path, *, verify_artifacts: bool = True) -> dict:
    manifest_path = Path(path).expanduser().resolve()
    try:
        manifest = json.loads(manifest_path.read_text())
    except (OSError, json.JSONDecodeError) as exc:
        raise DatasetManifestError(f"cannot load dataset manifest {manifest_path}: {exc}") from exc
    validate_dataset_manifest(manifest, manifest_path, verify_artifacts=verify_artifacts)
    return manifest


def artifact_provenance(path) -> dict:
    p = Path(path).expanduser().resolve()
    if not p.is_file():
        raise EvaluationProvenanceError(f"evaluation artifact not found: {p}")
    return {"path": str(p), "bytes": p.stat().st_size, "sha256": file_sha256(p)}


def bind_dataset_manifest(manifest_path, *, expected_artifacts: Mapping | None = None,
                          require_scientific: bool = True) -> tuple:
    """evaluation_provenance.py:27-61."""
    resolved = Path(manifest_path).expanduser().resolve()
    manifest = load_dataset_manifest(resolved)
    if require_scientific and not manifest["dataset"].get("scientific_valid"):
        raise EvaluationProvenanceError(f"dataset manifest is not marked scientific_valid: {resolved}")
    bound = {}
    for name, selected in (expected_artifacts or {}).items():
        sel = Path(selected).expanduser().resolve()
        declared = manifest_artifact_path(manifest, resolved, name).resolve()
        if sel != declared:
            raise EvaluationProvenanceError(f"{name} input {sel} does not match manifest artifact {declared}")
        bound[name] = artifact_provenance(declared)
    vocab = manifest_artifact_path(manifest, resolved, "vocabulary").resolve()
    return manifest, {"status": "frozen_manifest_verified", **artifact_provenance(resolved),
                      "dataset_id": manifest["dataset"]["id"],
                      "scientific_valid": bool(manifest["dataset"]["scientific_valid"]),
                      "schema": manifest["schema"], "vocabulary": artifact_provenance(vocab),
                      "bound_artifacts": bound}


def bind_checkpoint_dataset(checkpoint_cfg: Mapping, manifest_provenance: Mapping | None) -> dict:
    """evaluation_provenance.py:64-111."""
    ck_manifest = checkpoint_cfg.get("dataset_manifest")
    ck_id = ck_manifest.get("dataset_id") if isinstance(ck_manifest, Mapping) else None
    if ck_id is None:
        return {"status": "legacy_checkpoint_unverified", "dataset_id": None}
    if manifest_provenance is None:
        raise EvaluationProvenanceError("corrected checkpoint requires an explicit frozen dataset manifest")
    if ck_id != manifest_provenance.get("dataset_id"):
        raise EvaluationProvenanceError(
            f"checkpoint dataset identity mismatch: checkpoint={ck_id!r}, "
            f"manifest={manifest_provenance.get('dataset_id')!r}")
    ck_vocab = checkpoint_cfg.get("vocabulary")
    ck_sha = ck_vocab.get("sha256") if isinstance(ck_vocab, Mapping) else None
    man_sha = manifest_provenance.get("vocabulary", {}).get("sha256")
    if ck_sha is not None and ck_sha != man_sha:
        raise EvaluationProvenanceError(f"checkpoint vocabulary mismatch: checkpoint={ck_sha!r}, manifest={man_sha!r}")
    return {"status": "checkpoint_manifest_verified", "dataset_id": ck_id, "vocabulary_sha256": ck_sha}


__all__ = ["DatasetManifestError", "EvaluationProvenanceError", "bind_checkpoint_dataset", "bind_dataset_manifest",
           "dataset_identity", "load_dataset_manifest", "validate_dataset_manifest"]
