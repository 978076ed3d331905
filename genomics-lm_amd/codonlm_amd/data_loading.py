"""HBM-resident codon datasets and batch loaders (mirrors src/codonlm/data_loading.py).

The reference keeps token arrays in host memory and feeds each microbatch through a
``DataLoader`` (collate on the CPU, then ``xb.to(device)`` at loop.py:1066).  Here the
whole token store is copied to HBM once (288 GB per GPU holds any codon corpus the
reference handles), and a batch is a single gather launch (cg_gather_windows /
cg_gather_sequences) indexed by a device-resident permutation, so the training loop does
no per-step host->device token copy.

Batch ORDER is the reference's, bit for bit:
  * shuffled train loader: what ``DataLoader(shuffle=True, generator=g)`` draws
    (data_loading.py:466-478) -- one int64 base-seed draw from ``g``, then
    ``torch.randperm(n, generator=g)`` -- in consecutive ``batch_size`` chunks, last partial;
  * ``bucket_batching`` on dynamic data: BucketBatchSampler (:332-377) restated;
  * val loader: sequential, unshuffled.
Storage formats: fixed windows (NPZ ``X``/``Y`` [N, T]) or dynamic sequences (NPZ flat
``X`` + ``lengths``), loaded with ``allow_pickle=False`` like the reference.  With ``use_mmap``
(the reference's MmapPackedDataset, data_loading.py:132-200) uncompressed ``<stem>_X.npy`` /
``_Y.npy`` / ``_lengths.npy`` sidecars are memory-mapped and streamed to HBM in chunks, so the
corpus is never materialised in host RAM; without sidecars the NPZ is read, as the reference's
fallback does.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from . import _lib as L

PAD_ID = 0
_ELEM = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}


_CHUNK = 1 << 24  # elements per host->device piece of a memory-mapped array


def _width_for(lo: int, hi: int, dtype: np.dtype) -> int:
    if dtype.itemsize == 1 and dtype.kind == "u":
        return 1
    if lo >= -(1 << 15) and hi < (1 << 15) and dtype.itemsize <= 2:
        return 2
    if lo >= -(1 << 31) and hi < (1 << 31) and dtype.itemsize <= 4:
        return 4
    return 8


def _device_int_stream(a: np.ndarray, device) -> tuple[torch.Tensor, int]:
    """_device_int for a memory-mapped array: min / max and the upload in _CHUNK pieces (one
    pinned staging buffer), never the whole array in host memory."""
    if a.dtype.kind not in "iu":
        raise TypeError(f"token arrays must be integer, got {a.dtype}")
    flat = a.reshape(-1)
    if flat.size == 0:
        return torch.zeros(a.shape, dtype=torch.int32, device=device), 4
    lo, hi = None, None
    for i in range(0, flat.size, _CHUNK):
        c = flat[i:i + _CHUNK]
        clo, chi = int(c.min()), int(c.max())
        lo = clo if lo is None else min(lo, clo)
        hi = chi if hi is None else max(hi, chi)
    eb = _width_for(lo, hi, a.dtype)
    nd = _ELEM[eb]
    out = torch.empty(flat.size, dtype=torch.from_numpy(np.zeros(0, nd)).dtype, device=device)
    stage = torch.empty(min(_CHUNK, flat.size), dtype=out.dtype, pin_memory=torch.cuda.is_available())
    for i in range(0, flat.size, _CHUNK):
        c = np.asarray(flat[i:i + _CHUNK]).astype(nd, copy=False)
        st = stage[:len(c)]
        st.numpy()[:] = c
        out[i:i + len(c)].copy_(st, non_blocking=False)
    return out.view(a.shape), eb


def _npy_sidecars(paths):
    """The reference's MmapPackedDataset probe (data_loading.py:142-158): per path the
    ``<stem>_X.npy`` and ``_Y.npy`` or ``_lengths.npy`` sidecars, or None if any path lacks them."""
    from pathlib import Path
    out = []
    for path in paths:
        p = Path(path)
        x, y, ln = (p.with_name(p.stem + suf) for suf in ("_X.npy", "_Y.npy", "_lengths.npy"))
        if not (x.exists() and (ln.exists() or y.exists())):
            return None
        out.append({"X": x, "Y": y if y.exists() else None, "lengths": ln if ln.exists() else None,
                    "is_dynamic": ln.exists()})
    if len({c["is_dynamic"] for c in out}) > 1:
        raise ValueError("all memory-mapped dataset shards must use the same format")
    return out


def _device_int(a: np.ndarray, device) -> tuple[torch.Tensor, int]:
    """Upload an integer token array keeping a compact storage width (1/2/4/8 bytes)."""
    a = np.ascontiguousarray(a)
    if a.dtype.kind not in "iu":
        raise TypeError(f"token arrays must be integer, got {a.dtype}")
    if a.size == 0:
        return torch.zeros(0, dtype=torch.int32, device=device), 4
    eb = _width_for(int(a.min()), int(a.max()), a.dtype)
    if eb != a.dtype.itemsize or (eb > 1 and a.dtype.kind == "u"):
        a = a.astype(_ELEM[eb])
    return torch.from_numpy(a).to(device), eb


class DeviceCodonDataset:
    """PackedDataset (data_loading.py:43-129) / MmapPackedDataset (:132-329, ``use_mmap``) with
    its token store in HBM."""

    def __init__(self, paths, device=None, use_mmap: bool = False):
        if isinstance(paths, (str, os.PathLike)):
            paths = [paths]
        paths = [str(p) for p in paths]
        self.device = torch.device(device if device is not None else ("cuda", torch.cuda.current_device()))
        self.is_dynamic = False
        self.storage_mode = "npz_memory"
        side = _npy_sidecars(paths) if (use_mmap and paths) else None
        if side is not None:
            self._init_mmap(side)
            return
        if paths:
            with np.load(paths[0], allow_pickle=False) as data:
                self.is_dynamic = "lengths" in data
        if self.is_dynamic:
            flats, lens = [], []
            for p in paths:
                with np.load(p, allow_pickle=False) as data:
                    flats.append(np.asarray(data["X"]).reshape(-1))
                    lens.append(np.asarray(data["lengths"]).astype(np.int64))
            # per-file offsets restart at 0 in the reference; one global store here
            flat = np.concatenate(flats) if flats else np.zeros(0, np.int32)
            self._lengths = np.concatenate(lens) if lens else np.zeros(0, np.int64)
            starts = np.zeros(len(self._lengths), dtype=np.int64)
            base = 0
            k = 0
            for f, ln in zip(flats, lens):
                if len(ln):
                    starts[k:k + len(ln)] = base + np.concatenate([[0], np.cumsum(ln[:-1])])
                k += len(ln)
                base += len(f)
            self.flat, self._eb = _device_int(flat, self.device)
            self.starts = torch.from_numpy(starts).to(self.device)
            self.lens = torch.from_numpy(self._lengths).to(self.device)
            self.n = len(self._lengths)
        else:
            Xs, Ys = [], []
            for p in paths:
                with np.load(p, allow_pickle=False) as data:
                    Xs.append(np.asarray(data["X"]))
                    Ys.append(np.asarray(data["Y"]))
            X = np.concatenate(Xs) if Xs else np.zeros((0, 0), np.int32)
            Y = np.concatenate(Ys) if Ys else np.zeros((0, 0), np.int32)
            if X.shape != Y.shape:
                raise ValueError(f"X {X.shape} and Y {Y.shape} must have the same shape")
            self.T = int(X.shape[1]) if X.ndim == 2 else 0
            self.X, self._eb = _device_int(X, self.device)
            self.Y, self._ebY = _device_int(Y, self.device)
            self.n = int(X.shape[0])

    def _init_mmap(self, side):
        """Uncompressed NPY sidecars, memory-mapped (np.load(mmap_mode="r")) and streamed to HBM."""
        self.storage_mode = "npy_mmap"
        self.is_dynamic = side[0]["is_dynamic"]
        if self.is_dynamic:
            xs = [np.load(c["X"], mmap_mode="r", allow_pickle=False) for c in side]
            lens = [np.asarray(np.load(c["lengths"], mmap_mode="r", allow_pickle=False)).astype(np.int64)
                    for c in side]
            self._lengths = np.concatenate(lens) if lens else np.zeros(0, np.int64)
            starts = np.zeros(len(self._lengths), dtype=np.int64)
            base, k = 0, 0
            for f, ln in zip(xs, lens):
                if len(ln):
                    starts[k:k + len(ln)] = base + np.concatenate([[0], np.cumsum(ln[:-1])])
                k += len(ln)
                base += f.size
            parts = [_device_int_stream(f.reshape(-1), self.device) for f in xs]
            self._eb = max(eb for _, eb in parts) if parts else 4
            nd = torch.from_numpy(np.zeros(0, _ELEM[self._eb])).dtype
            self.flat = torch.cat([t.to(nd) for t, _ in parts]) if parts else torch.zeros(0, dtype=nd,
                                                                                          device=self.device)
            self.starts = torch.from_numpy(starts).to(self.device)
            self.lens = torch.from_numpy(self._lengths).to(self.device)
            self.n = len(self._lengths)
            return
        Xs = [np.load(c["X"], mmap_mode="r", allow_pickle=False) for c in side]
        Ys = [np.load(c["Y"], mmap_mode="r", allow_pickle=False) for c in side]
        for x, y in zip(Xs, Ys):
            if x.shape != y.shape:
                raise ValueError(f"X {x.shape} and Y {y.shape} must have the same shape")
        self.T = int(Xs[0].shape[1]) if Xs and Xs[0].ndim == 2 else 0

        def cat(arrs):
            parts = [_device_int_stream(a, self.device) for a in arrs]
            eb = max(e for _, e in parts)
            nd = torch.from_numpy(np.zeros(0, _ELEM[eb])).dtype
            return torch.cat([t.to(nd) for t, _ in parts]), eb
        self.X, self._eb = cat(Xs)
        self.Y, self._ebY = cat(Ys)
        self.n = int(self.X.shape[0])

    def __len__(self):
        return self.n

    @property
    def seq_lengths(self) -> np.ndarray:
        if self.is_dynamic:
            return self._lengths.astype(np.int32, copy=False)
        return np.full(self.n, self.T, dtype=np.int32)

    def gather(self, rows_dev: torch.Tensor, rows_host: np.ndarray):
        """(x, y) int64 [B, T] on the device for sample indices ``rows`` (one launch)."""
        B = int(len(rows_host))
        st = L.stream_ptr(self.device)
        if self.is_dynamic:
            Tout = max(0, int(self._lengths[rows_host].max()) - 1) if B else 0
            x = torch.empty(B, Tout, dtype=torch.int64, device=self.device)
            y = torch.empty_like(x)
            L.check(L.lib.cg_gather_sequences(self._eb, self.flat.data_ptr(), self.starts.data_ptr(),
                                              self.lens.data_ptr(), self.n, rows_dev.data_ptr(), B, Tout,
                                              x.data_ptr(), y.data_ptr(), st), "cg_gather_sequences")
            return x, y
        x = torch.empty(B, self.T, dtype=torch.int64, device=self.device)
        y = torch.empty_like(x)
        L.check(L.lib.cg_gather_windows(self._eb, self.X.data_ptr(), self.T, self.n, rows_dev.data_ptr(), B, self.T,
                                        x.data_ptr(), st), "cg_gather_windows")
        L.check(L.lib.cg_gather_windows(self._ebY, self.Y.data_ptr(), self.T, self.n, rows_dev.data_ptr(), B, self.T,
                                        y.data_ptr(), st), "cg_gather_windows")
        return x, y


def bucket_batches(lengths: np.ndarray, batch_size: int, n_buckets: int = 8, shuffle: bool = True,
                   drop_last: bool = False, seed: int | None = None) -> list[list[int]]:
    """BucketBatchSampler (data_loading.py:332-377) restated: same buckets, same rng draws."""
    edges = np.linspace(lengths.min(), lengths.max() + 1, n_buckets + 1)
    bucket_ids = np.digitize(lengths, edges[1:])
    buckets: list[list[int]] = [[] for _ in range(n_buckets)]
    for i, bid in enumerate(bucket_ids):
        buckets[bid].append(i)
    rng = np.random.default_rng(seed)
    out: list[list[int]] = []
    for bucket in buckets:
        if not bucket:
            continue
        idx = list(bucket)
        if shuffle:
            rng.shuffle(idx)
        for s in range(0, len(idx), batch_size):
            b = idx[s:s + batch_size]
            if drop_last and len(b) < batch_size:
                continue
            out.append(b)
    if shuffle:
        rng.shuffle(out)
    return out


def epoch_batches(n: int, batch_size: int, *, shuffle: bool = False, seed: int | None = None,
                  lengths: np.ndarray | None = None, n_buckets: int = 8):
    """(order, bounds): sample order of one epoch and the batch boundaries into it, as the
    reference DataLoader draws them (RandomSampler with a seeded generator, or the
    BucketBatchSampler when ``lengths`` is given)."""
    if lengths is not None and n:
        batches = bucket_batches(np.asarray(lengths), batch_size, n_buckets, shuffle=True, seed=seed)
        order = np.array([i for b in batches for i in b], dtype=np.int64)
        return order, np.cumsum([0] + [len(b) for b in batches])
    if shuffle:
        g = torch.Generator()
        g.manual_seed(int(seed) if seed is not None else int(torch.empty((), dtype=torch.int64).random_().item()))
        # the DataLoader iterator draws its worker base seed from the generator first
        # (_BaseDataLoaderIter.__init__), then RandomSampler draws the permutation
        torch.empty((), dtype=torch.int64).random_(generator=g)
        order = torch.randperm(n, generator=g).numpy().astype(np.int64)
    else:
        order = np.arange(n, dtype=np.int64)
    nb = math.ceil(n / batch_size) if n else 0
    return order, np.minimum(np.arange(nb + 1) * batch_size, n)


class DeviceBatchLoader:
    """Iterates (x, y) device batches in the reference DataLoader's order.

    ``rank``/``world`` shard the batch sequence round-robin for data parallelism (rank r
    takes batches r, r+world, ...), each rank keeping the same global order.  Training
    (``drop_remainder=True``): every rank runs floor(n_batches / world) batches so the
    per-group collectives stay matched.  Evaluation (``drop_remainder=False``): the first
    n_batches % world ranks run one batch more, so every batch is evaluated exactly once and
    the sums reduced over ranks do not depend on the GPU count."""

    def __init__(self, ds: DeviceCodonDataset, batch_size: int, *, shuffle: bool = False, seed: int | None = None,
                 bucket_batching: bool = False, n_buckets: int = 8, rank: int = 0, world: int = 1,
                 drop_remainder: bool = True):
        self.ds, self.bs = ds, int(batch_size)
        self.rank, self.world = int(rank), max(1, int(world))
        self.drop_remainder = bool(drop_remainder)
        n = len(ds)
        self.order, self._bounds = epoch_batches(n, self.bs, shuffle=shuffle, seed=seed,
                                                 lengths=ds.seq_lengths if (bucket_batching and ds.is_dynamic) else None,
                                                 n_buckets=n_buckets)
        self._order_dev = torch.from_numpy(self.order).to(ds.device) if n else None

    def __len__(self):
        return len(self.shard())

    def global_batches(self) -> int:
        return len(self._bounds) - 1

    def shard(self) -> list:
        """Global batch indices this rank runs, in order."""
        nb = len(self._bounds) - 1
        if self.world == 1:
            return list(range(nb))
        n = nb // self.world if self.drop_remainder else (nb - self.rank + self.world - 1) // self.world
        return [self.rank + j * self.world for j in range(max(0, n))]

    def __iter__(self):
        for k in self.shard():
            a, b = int(self._bounds[k]), int(self._bounds[k + 1])
            yield self.ds.gather(self._order_dev[a:b], self.order[a:b])


__all__ = ["DeviceCodonDataset", "DeviceBatchLoader", "bucket_batches", "PAD_ID"]
