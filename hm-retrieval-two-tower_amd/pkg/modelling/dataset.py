"""Encoded batch datasets: this framework's replacement for the TFRecord
input pipeline (/root/reference/pkg/modelling/tfrecord_dataset.py:10-98,
SURVEY §8f row 1, outside the hot path).

Rows are stored already encoded: int32 embedding rows for categorical
features (the reference's StringLookup applied once, offline), float32 for
numeric features, plus optional extra columns (e.g. "__logq__", raw id
codes).  Shards are .npz files (numpy.load with allow_pickle=False).
Batches keep the reference's semantics: fixed batch size, the last batch
partial (no drop_remainder, tfrecord_dataset.py:97), optional shuffling.
"""
from __future__ import annotations

import glob
import os
from typing import Callable, Dict, Iterator, List, Optional, Sequence

import numpy as np
import pandas as pd
import torch

from pkg import dtypes
from pkg.schema.features import Feature
from pkg.modelling.device import default_device
from pkg.modelling import hip_ops

__all__ = ["EncodedDataset", "DeviceDataset", "encode_dataframe", "epoch_order"]


def epoch_order(num_rows: int, shuffle_size: Optional[int], seed: int, epoch: int) -> np.ndarray:
    """Example order of one epoch: identity, or a permutation inside consecutive
    windows of shuffle_size (a shuffle buffer of that size never moves an
    element further; tfrecord_dataset.py:95 shuffles with such a buffer)."""
    if not shuffle_size:
        return np.arange(num_rows)
    rng = np.random.default_rng(seed + epoch)
    order = np.arange(num_rows)
    w = int(shuffle_size)
    for s in range(0, num_rows, w):
        rng.shuffle(order[s:s + w])
    return order


def encode_dataframe(df: pd.DataFrame, features: Sequence[Feature],
                     extra: Optional[Dict[str, np.ndarray]] = None, logq=None,
                     candidate_col: Optional[str] = None) -> Dict[str, np.ndarray]:
    """Encode a DataFrame with the schema's features (StringLookup on the host,
    libtt's multi-threaded hash table).  logq: a LogQCorrection (or its
    {id: p} dict) — adds the exact per-example "__logq__" column from the raw
    candidate ids (logq_correction.py:66-71), needed when the probability
    lookup covers ids outside the candidate vocab."""
    cols: Dict[str, np.ndarray] = {}
    if logq is not None:
        from pkg.modelling.layers.logq_correction import LogQCorrection

        corr = logq if isinstance(logq, LogQCorrection) else LogQCorrection(logq)
        if candidate_col is None:
            raise ValueError("encode_dataframe: logq needs candidate_col")
        cols["__logq__"] = corr.log_probs(df[candidate_col].values)
    for f in features:
        if f.name in cols:
            continue
        if f.dtype == dtypes.string:
            cols[f.name] = f.encode(df[f.name].values)
        else:
            cols[f.name] = df[f.name].values.astype(np.float32)
    for k, v in (extra or {}).items():
        cols[k] = np.asarray(v)
    return cols


class EncodedDataset:
    """Batches of device tensors from in-memory encoded columns."""

    def __init__(self, columns: Dict[str, np.ndarray], batch_size: Optional[int] = None,
                 shuffle_size: Optional[int] = None, seed: int = 0, device: Optional[torch.device] = None,
                 fn: Optional[Callable] = None):
        lens = {len(v) for v in columns.values()}
        if len(lens) > 1:
            raise ValueError(f"columns have different lengths: {lens}")
        self.columns = {k: np.ascontiguousarray(v) for k, v in columns.items()}
        self.num_rows = lens.pop() if lens else 0
        self.batch_size = batch_size
        self.shuffle_size = shuffle_size
        self.seed = seed
        self.device = device if device is not None else default_device()
        self.fn = fn
        self._epoch = 0

    def __len__(self) -> int:
        bs = self.batch_size or 1
        return (self.num_rows + bs - 1) // bs

    def map(self, fn: Callable) -> "EncodedDataset":
        prev = self.fn
        new = EncodedDataset(self.columns, self.batch_size, self.shuffle_size, self.seed, self.device,
                             (lambda b: fn(prev(b))) if prev else fn)
        return new

    def _order(self) -> np.ndarray:
        return epoch_order(self.num_rows, self.shuffle_size, self.seed, self._epoch)

    def __iter__(self) -> Iterator:
        order = self._order()
        self._epoch += 1
        bs = self.batch_size or self.num_rows or 1
        for s in range(0, self.num_rows, bs):
            sel = order[s:s + bs]
            batch = {}
            for k, v in self.columns.items():
                a = v[sel] if self.shuffle_size else v[s:s + bs]
                t = torch.from_numpy(np.ascontiguousarray(a))
                batch[k] = t.to(self.device, non_blocking=True) if self.device.type == "cuda" else t
            yield self.fn(batch) if self.fn else batch

    # ---- shards ---------------------------------------------------------
    def save(self, dirpath: str, max_rows: Optional[int] = None) -> List[str]:
        os.makedirs(dirpath, exist_ok=True)
        step = max_rows or max(self.num_rows, 1)
        paths = []
        for i, s in enumerate(range(0, max(self.num_rows, 1), step)):
            p = os.path.join(dirpath, f"part-{i:05d}.npz")
            np.savez(p, **{k: v[s:s + step] for k, v in self.columns.items()})
            paths.append(p)
        return paths

    @classmethod
    def load(cls, dirpath: str, batch_size: Optional[int] = None, shuffle_size: Optional[int] = None,
             seed: int = 0, device: Optional[torch.device] = None) -> "EncodedDataset":
        files = sorted(glob.glob(os.path.join(dirpath, "*.npz")))
        if not files:
            raise FileNotFoundError(f"no .npz shards in {dirpath}")
        parts: Dict[str, List[np.ndarray]] = {}
        for p in files:
            with np.load(p, allow_pickle=False) as z:
                for k in z.files:
                    parts.setdefault(k, []).append(z[k])
        cols = {k: np.concatenate(v) for k, v in parts.items()}
        return cls(cols, batch_size, shuffle_size, seed, device)


class DeviceDataset:
    """Encoded columns resident in HBM; every batch assembled on the device.

    The columns (int32 rows / float32 values, 1-D, equal length) are stored
    as one [C, N] matrix of 32-bit words, int columns first then float
    columns, each group in sorted key order (GraphedTrainStep's static batch
    layout).  An epoch's order is epoch_order(...) — the same batches, in the
    same order, as EncodedDataset with the same seed — uploaded once per
    epoch; a batch is one tt_batch_take launch reading the position from a
    device cursor, so TwoTowerModel.fit can replay take + train step as one
    hipGraph with no host work per step.  Batches are fixed-size with a
    partial last batch (tfrecord_dataset.py:97, no drop_remainder)."""

    def __init__(self, columns: Dict[str, np.ndarray], batch_size: Optional[int] = None,
                 shuffle_size: Optional[int] = None, seed: int = 0, device: Optional[torch.device] = None,
                 fn: Optional[Callable] = None, _shared=None):
        self.batch_size = batch_size
        self.shuffle_size = shuffle_size
        self.seed = seed
        self.fn = fn
        if _shared is not None:
            self.__dict__.update(_shared)
            self._epoch = 0
            return
        self.device = device if device is not None else default_device()
        if self.device.type != "cuda":
            raise ValueError("DeviceDataset keeps its columns in GPU memory (got device %s)" % self.device)
        lens = {len(v) for v in columns.values()}
        if len(lens) != 1:
            raise ValueError(f"columns must be non-empty and of one length, got {lens}")
        self.num_rows = lens.pop()
        words, ikeys, fkeys = [], [], []
        for k in sorted(columns):
            v = np.asarray(columns[k]).reshape(-1)
            if v.dtype.kind in "iu":
                if v.size and (v.min() < -(1 << 31) or v.max() >= (1 << 31)):
                    raise ValueError(f"column {k} does not fit int32")
                ikeys.append(k)
            elif v.dtype.kind == "f":
                fkeys.append(k)
            else:
                raise TypeError(f"column {k} has dtype {v.dtype}; DeviceDataset holds int32 / float32 columns")
        self.int_keys, self.float_keys = ikeys, fkeys
        for k in ikeys:
            words.append(np.ascontiguousarray(np.asarray(columns[k]).reshape(-1), dtype=np.int32))
        for k in fkeys:
            words.append(np.ascontiguousarray(np.asarray(columns[k]).reshape(-1), dtype=np.float32).view(np.int32))
        host = torch.from_numpy(np.stack(words))
        self.words = host.pin_memory().to(self.device, non_blocking=True) if host.numel() else host.to(self.device)
        self._perm = torch.empty(self.num_rows, dtype=torch.int64, device=self.device)
        self._perm_tag = [("unset",)]  # shared with mapped views: which order _perm holds
        self._order_pool = [None]
        self._order_futures: Dict[tuple, object] = {}
        self.cursor = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.status = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._epoch = 0

    @classmethod
    def from_encoded(cls, ds: EncodedDataset, device: Optional[torch.device] = None) -> "DeviceDataset":
        return cls(ds.columns, ds.batch_size, ds.shuffle_size, ds.seed, device or ds.device, ds.fn)

    @classmethod
    def load(cls, dirpath: str, batch_size: Optional[int] = None, shuffle_size: Optional[int] = None,
             seed: int = 0, device: Optional[torch.device] = None) -> "DeviceDataset":
        return cls.from_encoded(EncodedDataset.load(dirpath, batch_size, shuffle_size, seed, device))

    @property
    def keys(self) -> List[str]:
        return self.int_keys + self.float_keys

    def _shared(self) -> dict:
        names = ("device", "num_rows", "int_keys", "float_keys", "words", "_perm", "_perm_tag", "_order_pool",
                 "_order_futures", "cursor", "status")
        return {k: self.__dict__[k] for k in names}

    def map(self, fn: Callable) -> "DeviceDataset":
        prev = self.fn
        return DeviceDataset({}, self.batch_size, self.shuffle_size, self.seed,
                             fn=(lambda b: fn(prev(b))) if prev else fn, _shared=self._shared())

    def __len__(self) -> int:
        bs = self.batch_size or 1
        return (self.num_rows + bs - 1) // bs

    @property
    def full_batches(self) -> int:
        return self.num_rows // (self.batch_size or self.num_rows)

    # ---- epochs and batches ----------------------------------------------
    def begin_epoch(self) -> int:
        """Upload this epoch's order, reset the cursor; returns the epoch index."""
        epoch = self._epoch
        self._epoch += 1
        tag = (self.shuffle_size, self.seed, epoch) if self.shuffle_size else ("identity",)
        if self._perm_tag[0] != tag:
            # pinned here, on the calling thread (not on the order thread: a
            # pinned allocation on another thread while this one captures or
            # replays a hipGraph crashed the replay)
            order = self._host_order(epoch)
            if self._perm.is_cuda:
                order = order.pin_memory()
            self._perm.copy_(order, non_blocking=True)
            self._perm_tag[0] = tag
        if self.shuffle_size:
            # the next epoch's order is built on a host thread while this epoch's
            # graph replays run (an epoch of 10M rows shuffles in ~0.15 s)
            self._prefetch_order(epoch + 1)
        self.cursor.zero_()
        self.status.zero_()
        return epoch

    def _make_order(self, epoch: int) -> torch.Tensor:
        order = epoch_order(self.num_rows, self.shuffle_size, self.seed, epoch).astype(np.int64)
        return torch.from_numpy(order)  # host only: no HIP call on the order thread

    def _prefetch_order(self, epoch: int) -> None:
        from concurrent.futures import ThreadPoolExecutor

        pool = self._order_pool[0]
        if pool is None:
            pool = self._order_pool[0] = ThreadPoolExecutor(1, thread_name_prefix="epoch-order")
        key = (self.shuffle_size, self.seed, epoch)
        if key not in self._order_futures:
            self._order_futures.clear()
            self._order_futures[key] = pool.submit(self._make_order, epoch)

    def _host_order(self, epoch: int) -> torch.Tensor:
        fut = self._order_futures.pop((self.shuffle_size, self.seed, epoch), None)
        return fut.result() if fut is not None else self._make_order(epoch)

    def view(self, words: torch.Tensor) -> Dict[str, torch.Tensor]:
        """Batch dict of [B] views over a [C, B] word buffer."""
        out = {k: words[i] for i, k in enumerate(self.int_keys)}
        out.update({k: words[len(self.int_keys) + j].view(torch.float32) for j, k in enumerate(self.float_keys)})
        return out

    def take(self, rows: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The next `rows` examples as a [C, rows] word buffer (advances the cursor)."""
        if out is None:
            out = torch.empty(len(self.keys), rows, dtype=torch.int32, device=self.device)
        return hip_ops.batch_take(self.words, self._perm, self.cursor, out, True, self.status)

    def check_status(self) -> None:
        """Raise if a take ran past the epoch (synchronises)."""
        if int(self.status.item()) != 0:
            raise RuntimeError("DeviceDataset: a batch was taken past the end of the epoch")

    def __iter__(self) -> Iterator:
        self.begin_epoch()
        bs = self.batch_size or self.num_rows or 1
        for s in range(0, self.num_rows, bs):
            batch = self.view(self.take(min(bs, self.num_rows - s)))
            yield self.fn(batch) if self.fn else batch
