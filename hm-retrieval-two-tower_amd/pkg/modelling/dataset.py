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

__all__ = ["EncodedDataset", "encode_dataframe"]


def encode_dataframe(df: pd.DataFrame, features: Sequence[Feature],
                     extra: Optional[Dict[str, np.ndarray]] = None) -> Dict[str, np.ndarray]:
    """Encode a DataFrame with the schema's features (StringLookup on the host)."""
    cols: Dict[str, np.ndarray] = {}
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
        if not self.shuffle_size:
            return np.arange(self.num_rows)
        rng = np.random.default_rng(self.seed + self._epoch)
        # windowed shuffle: permutation inside consecutive windows of shuffle_size
        # (a buffer of shuffle_size never moves an element further than that)
        order = np.arange(self.num_rows)
        w = int(self.shuffle_size)
        for s in range(0, self.num_rows, w):
            rng.shuffle(order[s:s + w])
        return order

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
