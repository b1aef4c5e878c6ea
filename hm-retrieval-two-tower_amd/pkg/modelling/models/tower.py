"""Tower: InputLayer -> Dense(relu)* -> Dense(E, relu)
(mirror of /root/reference/pkg/modelling/models/tower.py:8-91).

Dense layers follow Keras defaults: kernel [fan_in, units] glorot_uniform,
zero bias, relu on every layer including the last (tower.py:45,48), so the
joint embeddings are non-negative.  All kernels and biases of a tower live in
ONE flat fp32 buffer (views per layer), so its gradient is one contiguous
tensor and the dense optimizer step is a single tt_dense_* launch.  The GEMMs
run through torch (hipBLASLt), fp32.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

from pkg.schema.features import Feature
from pkg.modelling.device import default_device, make_generator
from pkg.modelling.layers.input_layer import InputLayer
from pkg.modelling.models.abstract_keras_model import AbstractKerasModel, TensorSpec

__all__ = ["Tower", "DenseStack"]


def _splitk_mm_tn(a: torch.Tensor, g: torch.Tensor, out: torch.Tensor, splits: int = 16) -> None:
    """out = a^T g for tall a [B, fin], g [B, fout] (the weight gradient).
    hipBLASLt runs this skinny, K=B-long product on a handful of tiles; a
    batched split over B (bmm of `splits` slices, then a sum) fills the GPU
    (≈3x faster at B=16384)."""
    B = a.shape[0]
    if B >= 4096 and B % splits == 0:
        part = torch.bmm(a.view(splits, B // splits, a.shape[1]).transpose(1, 2),
                         g.view(splits, B // splits, g.shape[1]))
        torch.sum(part, 0, out=out)
    else:
        torch.mm(a.t(), g, out=out)


class _DenseStackFn(torch.autograd.Function):
    """Forward relu(addmm) per layer; backward writes every weight / bias
    gradient straight into ONE flat gradient buffer (no per-view autograd
    copies), so the optimizer step stays a single launch per tower."""

    @staticmethod
    def forward(ctx, x, flat, stack):
        h = x
        acts = [x]
        for w, b in stack.params(flat):
            h = torch.addmm(b, h, w)
            h.relu_()
            acts.append(h)
        ctx.stack = stack
        ctx.save_for_backward(flat, *acts)
        return h

    @staticmethod
    def backward(ctx, gout):
        flat, *acts = ctx.saved_tensors
        stack = ctx.stack
        gflat = torch.empty_like(flat)
        params = stack.params(flat)
        gparams = stack.params(gflat)
        g = gout
        for li in range(len(params) - 1, -1, -1):
            g = torch.ops.aten.threshold_backward(g, acts[li + 1], 0.0)
            dw, db = gparams[li]
            _splitk_mm_tn(acts[li], g, dw)
            torch.sum(g, 0, out=db)
            if li > 0 or ctx.needs_input_grad[0]:
                g = torch.mm(g, params[li][0].t())
        return (g if ctx.needs_input_grad[0] else None), gflat, None


class DenseStack:
    """relu(x W_l + b_l) for each layer; parameters are views of `flat`."""

    def __init__(self, in_dim: int, units: List[int], device: torch.device, generator: torch.Generator):
        self.layout: List[Tuple[int, int, int, int]] = []  # (w_off, fan_in, fan_out, b_off)
        off = 0
        fan_in = in_dim
        for u in units:
            self.layout.append((off, fan_in, u, off + fan_in * u))
            off += fan_in * u + u
            fan_in = u
        flat = torch.zeros(off, dtype=torch.float32)
        for w_off, fi, fo, _ in self.layout:
            lim = (6.0 / (fi + fo)) ** 0.5
            w = torch.empty(fi, fo, dtype=torch.float32).uniform_(-lim, lim, generator=generator)
            flat[w_off:w_off + fi * fo] = w.reshape(-1)
        self.flat = flat.to(device).requires_grad_(True)
        self.out_dim = fan_in

    def params(self, flat: Optional[torch.Tensor] = None):
        f = self.flat if flat is None else flat
        return [(f[w:w + fi * fo].view(fi, fo), f[b:b + fo]) for w, fi, fo, b in self.layout]

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        if torch.is_grad_enabled() and (x.requires_grad or self.flat.requires_grad):
            return _DenseStackFn.apply(x, self.flat, self)
        h = x
        for w, b in self.params(self.flat.detach()):
            h = torch.relu(torch.addmm(b, h, w))
        return h


class Tower(AbstractKerasModel):
    """
    Tower as a simple feed forward network for a two tower model.

    Parameters
    ----------
    features: List[Feature]
        Feature objects of this tower.
    joint_embedding_size: int
        Size used for taking the dot product with the other tower.
    hidden_units: Optional[List[int]]
        Optional hidden units.
    """

    def __init__(self, features: List[Feature], joint_embedding_size: int,
                 hidden_units: Optional[List[int]] = None, device: Optional[torch.device] = None,
                 generator: Optional[torch.Generator] = None):
        self.features = features
        self.joint_embedding_size = joint_embedding_size
        self.hidden_units = hidden_units
        self.device = device if device is not None else default_device()
        self._generator = generator if generator is not None else make_generator()
        self._init_layers()
        self.initialise_model()

    def _init_layers(self) -> None:
        self.input_layer = InputLayer(self.features, self.device, self._generator)
        units = list(self.hidden_units or []) + [self.joint_embedding_size]
        self.dense = DenseStack(self.input_layer.output_dim, units, self.device, self._generator)
        self.model_layers = [self.input_layer, self.dense]

    def call(self, x: Dict[str, torch.Tensor], training: bool = True) -> torch.Tensor:
        """[B, E] embeddings of the batch dict (tower.py:51-75)."""
        return self.dense(self.input_layer(x))

    def __call__(self, x, training: bool = False) -> torch.Tensor:
        if training:
            return self.call(x, training)
        with torch.no_grad():
            return self.call(x, training)

    def get_input_signature(self) -> Dict[str, TensorSpec]:
        return {f.name: TensorSpec((None, 1), f.dtype, f.name) for f in self.features}

    # -- parameters --------------------------------------------------------
    def dense_parameters(self) -> List[torch.Tensor]:
        return [self.dense.flat]

    def state_dict(self) -> Dict[str, torch.Tensor]:
        sd = {f"tables.{t.name}": t.weight.detach().cpu() for t in self.input_layer.tables()}
        sd["dense.flat"] = self.dense.flat.detach().cpu()
        return sd

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        for t in self.input_layer.tables():
            t.weight.copy_(sd[f"tables.{t.name}"].to(t.weight.device))
        with torch.no_grad():
            self.dense.flat.copy_(sd["dense.flat"].to(self.dense.flat.device))
