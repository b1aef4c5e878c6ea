"""InputLayer: categorical features -> embedding rows, concatenated.

Mirror of /root/reference/pkg/modelling/layers/input_layer.py:6-69.  The
StringLookup (input_layer.py:33-36) runs once on the host when a batch is
encoded (Feature.encode); on the device a batch is a dict of int32 row ids
(categorical) and float32 values (numeric).  The embedding gather + concat
(input_layer.py:37-41, 66-68) is ONE libtt launch (tt_gather_grouped) that
writes every feature's rows into its column range of the output.

The backward pass of the gather does not build dense table gradients: it
keeps the gradient w.r.t. the concatenated output (the reference's
IndexedSlices values) and the ids, and the optimizer applies the sparse
update from them (tt_sparse_adagrad / tt_sparse_adam).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from pkg import dtypes
from pkg.schema.features import Feature
from pkg.modelling import hip_ops
from pkg.modelling.device import default_device, make_generator

__all__ = ["InputLayer", "EmbeddingTable"]


class EmbeddingTable:
    """fp32 table [len(vocab)+1, D] with Keras Embedding's default init
    RandomUniform(-0.05, 0.05) (row 0 is the OOV row)."""

    def __init__(self, name: str, num_rows: int, dim: int, device: torch.device, generator: torch.Generator):
        self.name = name
        self.num_rows = int(num_rows)
        self.dim = int(dim)
        w = torch.empty(self.num_rows, self.dim, dtype=torch.float32)
        w.uniform_(-0.05, 0.05, generator=generator)
        self.weight = w.to(device)

    def __repr__(self) -> str:
        return f"EmbeddingTable({self.name!r}, rows={self.num_rows}, dim={self.dim})"


class _GatherFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, layer, segments, batch):
        out = torch.empty(batch, layer.row_stride, dtype=torch.float32, device=layer.device)
        hip_ops.gather_grouped(segments, batch, out)
        ctx.layer = layer
        return out[:, : layer.output_dim]

    @staticmethod
    def backward(ctx, grad_out):
        g = grad_out
        if g.stride(1) != 1:
            g = g.contiguous()
        ctx.layer.last_grad = g
        return None, None, None, None


class _MultiGatherFn(torch.autograd.Function):
    """Several InputLayers of one batch gathered by one tt_gather_multi launch."""

    @staticmethod
    def forward(ctx, layers, seglists, batch, extra, pack_jobs, *anchors):
        outs = [torch.empty(batch, l.row_stride, dtype=torch.float32, device=l.device) for l in layers]
        hip_ops.gather_multi(list(zip(seglists, outs)) + list(extra), batch, pack_jobs=pack_jobs)
        ctx.layers = layers
        return tuple(o[:, : l.output_dim] for o, l in zip(outs, layers))

    @staticmethod
    def backward(ctx, *grads):
        for layer, g in zip(ctx.layers, grads):
            if g is not None and g.stride(1) != 1:
                g = g.contiguous()
            layer.last_grad = g
        return (None, None, None, None, None) + (None,) * len(ctx.layers)


class InputLayer:
    """
    Convert a dict of tensors, embed categorical and concat together
    (input_layer.py:6-22).

    Parameters
    ----------
    features: List[Feature]
        Features of one tower.  Categorical = pkg.dtypes.string.
    """

    def __init__(self, features: List[Feature], device: Optional[torch.device] = None,
                 generator: Optional[torch.Generator] = None):
        self.device = device if device is not None else default_device()
        self.numerical_features = [f for f in features if f.dtype != dtypes.string]
        self.categorical_features = [f for f in features if f.dtype == dtypes.string]
        self._generator = generator if generator is not None else make_generator()
        self._init_embedding_layers()
        self.output_dim = len(self.numerical_features) + sum(
            self.embedding_layers[f.name].dim for f in self.categorical_features)
        # 16-byte aligned rows let the gather use dwordx4 stores
        self.row_stride = (self.output_dim + 3) // 4 * 4
        self._anchor = torch.zeros((), requires_grad=True)
        self.last_ids: Dict[str, torch.Tensor] = {}
        self.last_grad: Optional[torch.Tensor] = None

    def _init_embedding_layers(self) -> None:
        """One table per categorical feature NAME (input_layer.py:24-43).  As in
        the reference, a name declared twice keeps the last declaration's
        table (dict overwrite at input_layer.py:31) and is still looked up once
        per declaration (input_layer.py:66-67)."""
        self.embedding_layers: Dict[str, EmbeddingTable] = {}
        for f in self.categorical_features:
            if f.vocab is None:
                raise ValueError(f"categorical feature {f.name} has no vocab (build the schema first)")
            if not f.embedding_size:
                raise ValueError(f"categorical feature {f.name} needs an embedding_size")
            self.embedding_layers[f.name] = EmbeddingTable(f.name, len(f.vocab) + 1, f.embedding_size, self.device,
                                                           self._generator)

    # ------------------------------------------------------------------
    def tables(self) -> List[EmbeddingTable]:
        return list(self.embedding_layers.values())

    def column_offsets(self) -> List[int]:
        """Output column of each categorical lookup, in call order."""
        off = len(self.numerical_features)
        out = []
        for f in self.categorical_features:
            out.append(off)
            off += self.embedding_layers[f.name].dim
        return out

    def encode(self, x: Dict[str, Sequence]) -> Dict[str, torch.Tensor]:
        """Host StringLookup: raw values -> device int32 rows / float32 values."""
        out = {}
        for f in self.numerical_features:
            out[f.name] = torch.as_tensor(np.asarray(x[f.name], np.float32).reshape(-1), device=self.device)
        for f in self.categorical_features:
            out[f.name] = torch.as_tensor(f.encode(x[f.name]), device=self.device)
        return out

    def _ids(self, v, feature: Optional[Feature] = None) -> torch.Tensor:
        if not isinstance(v, torch.Tensor):
            a = np.asarray(v)
            # raw values (the reference's tf.string inputs): StringLookup on the host
            if feature is not None and a.dtype.kind in "OUS":
                return torch.as_tensor(feature.encode(a), device=self.device)
            v = a
        t = v if isinstance(v, torch.Tensor) else torch.as_tensor(v)
        t = t.reshape(-1)
        if t.dtype != torch.int32:
            t = t.to(torch.int32)
        if t.device != self.device:
            t = t.to(self.device)
        return t.contiguous()

    def _segments(self, x: Dict[str, torch.Tensor]):
        segments = []
        batch = None
        for f in self.numerical_features:
            v = x[f.name]
            v = (v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v, np.float32)))
            v = v.reshape(-1).to(device=self.device, dtype=torch.float32).contiguous()
            batch = v.numel() if batch is None else batch
            segments.append((v, None, len(segments)))
        ids_by_call = []
        for f, off in zip(self.categorical_features, self.column_offsets()):
            ids = self._ids(x[f.name], f)
            batch = ids.numel() if batch is None else batch
            if ids.numel() != batch:
                raise ValueError(f"feature {f.name} has {ids.numel()} rows, expected {batch}")
            segments.append((self.embedding_layers[f.name].weight, ids, off))
            ids_by_call.append((f.name, ids, off))
        if batch is None:
            raise ValueError("InputLayer called with no features")
        self._last_calls = ids_by_call
        self.last_grad = None
        return segments, batch

    def __call__(self, x: Dict[str, torch.Tensor]) -> torch.Tensor:
        """Pass a dict of [B] or [B,1] tensors; returns [B, output_dim] fp32."""
        segments, batch = self._segments(x)
        return _GatherFn.apply(self._anchor, self, segments, batch)

    @staticmethod
    def gather_many(layers: Sequence["InputLayer"], xs: Sequence[Dict[str, torch.Tensor]],
                    extra: Sequence = (), pack_jobs: Optional[Sequence] = None) -> List[torch.Tensor]:
        """The outputs of several InputLayers on one batch from ONE gather launch
        (the query and candidate towers of a train step).  `extra`: further
        (segments, out) calls of the same batch riding in that launch without
        gradients (the logQ lookup); `pack_jobs`: the towers' MLP weight
        images packed by the same launch (hip_ops.gather_multi)."""
        prepared = [l._segments(x) for l, x in zip(layers, xs)]
        batches = {b for _, b in prepared}
        if len(batches) != 1:
            raise ValueError(f"gather_many needs one batch size, got {sorted(batches)}")
        nseg = sum(len(segs) for segs, _ in prepared) + sum(len(segs) for segs, _ in extra)
        if nseg > hip_ops._native.MAX_SEGMENTS:
            b = batches.pop()
            for segs, out in extra:
                hip_ops.gather_grouped(segs, b, out)
            if pack_jobs:
                hip_ops.mlp_pack_many(pack_jobs)
            return [_GatherFn.apply(l._anchor, l, segs, bb) for l, (segs, bb) in zip(layers, prepared)]
        return list(_MultiGatherFn.apply(list(layers), [segs for segs, _ in prepared], batches.pop(), list(extra),
                                         pack_jobs or None, *[l._anchor for l in layers]))

    def sparse_sources(self) -> List[dict]:
        """Per table: its lookups of the last call as (ids, grad column) sources."""
        by_name: Dict[str, dict] = {}
        for name, ids, off in self._last_calls:
            d = by_name.setdefault(name, {"table": self.embedding_layers[name], "ids": [], "grad_col_offset": []})
            d["ids"].append(ids)
            d["grad_col_offset"].append(off)
        return list(by_name.values())
