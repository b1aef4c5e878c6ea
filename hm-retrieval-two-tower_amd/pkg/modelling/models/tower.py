"""Tower: InputLayer -> Dense(relu)* -> Dense(E, relu)
(mirror of /root/reference/pkg/modelling/models/tower.py:8-91).

Dense layers follow Keras defaults: kernel [fan_in, units] glorot_uniform,
zero bias, relu on every layer including the last (tower.py:45,48), so the
joint embeddings are non-negative.  All kernels and biases of a tower live in
ONE flat fp32 buffer (views per layer; each layer's bias right after its
kernel), so its gradient is one contiguous tensor and the dense optimizer
step is a single tt_dense_* launch.  Every GEMM is libtt's, on bf16x3 MFMA
(hi/lo split operands, fp32-faithful), with no vendor GEMM in the step:
  * forward: tt_mlp_rows per layer with the bias + relu epilogue; one
    tt_mlp_pack_many launch per tower per step packs its weight images;
  * backward, per layer from the top: [dW_l; db_l] by ONE tt_mlp_wgrad
    straight into the flat gradient (the top layer's ReluGrad and loss scale
    applied inside its loads), then ONE tt_mlp_rows for the layer below with
    the ReluGrad mask fused (G_{l-1} = (G_l W_l^T) * relu'(h_{l-1})), or the
    input gradient of the first layer.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

from pkg.schema.features import Feature
from pkg.modelling import hip_ops
from pkg.modelling.device import default_device, make_generator
from pkg.modelling.layers.input_layer import InputLayer
from pkg.modelling.models.abstract_keras_model import AbstractKerasModel, TensorSpec

__all__ = ["Tower", "DenseStack"]


class _DenseStackFn(torch.autograd.Function):
    """Forward relu(addmm) per layer; backward writes every weight / bias
    gradient straight into ONE flat gradient buffer (no per-view autograd
    copies), so the optimizer step stays a single launch per tower."""

    @staticmethod
    def forward(ctx, x, flat, stack):
        acts = stack.forward_acts(x, flat)
        ctx.stack = stack
        ctx.save_for_backward(flat, *acts)
        return acts[-1]

    @staticmethod
    def backward(ctx, gout):
        flat, *acts = ctx.saved_tensors
        gx, gflat = ctx.stack.backward_acts(acts, flat, gout.contiguous(), None, ctx.needs_input_grad[0])
        return gx, gflat, None


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

    def _pack_images(self, flat: torch.Tensor) -> Dict[Tuple[str, int], torch.Tensor]:
        """Every layer's packed bf16 hi/lo weight images, forward ("f": B = W)
        and transposed ("t": B = W^T, the input-gradient GEMMs), in ONE
        tt_mlp_pack_many launch into buffers owned by the stack (fixed
        addresses: graph-capturable).  Packed at the start of each forward,
        so they always match `flat`."""
        imgs = self.__dict__.setdefault("_images", {})
        jobs = []
        for li, (w, _) in enumerate(self.params(flat)):
            for kind, trans in (("f", False), ("t", True)):
                K, N = (w.shape[1], w.shape[0]) if trans else (w.shape[0], w.shape[1])
                nbytes = hip_ops.lib().tt_mlp_pack_bytes(K, N)
                buf = imgs.get((kind, li))
                if buf is None or buf.numel() < nbytes or buf.device != w.device:
                    buf = imgs[(kind, li)] = torch.empty(nbytes, dtype=torch.uint8, device=w.device)
                jobs.append((w, trans, buf))
        for i in range(0, len(jobs), 8):
            hip_ops.mlp_pack_many(jobs[i:i + 8])
        return imgs

    def forward_acts(self, x: torch.Tensor, flat: torch.Tensor) -> List[torch.Tensor]:
        """[x, h_1, ..., h_L] with h_l = relu(h_{l-1} W_l + b_l) (tt_mlp_rows)."""
        imgs = self._pack_images(flat)
        acts = [x]
        h = x
        for li, (w, b) in enumerate(self.params(flat)):
            out = torch.empty(h.shape[0], w.shape[1], dtype=torch.float32, device=h.device)
            h = hip_ops.mlp_rows(h, imgs[("f", li)], w.shape[0], w.shape[1], out, bias=b, relu=True)
            acts.append(h)
        return acts

    def _wgrad_fits(self, li: int, g: torch.Tensor, acts: List[torch.Tensor]) -> bool:
        """tt_mlp_wgrad's contract for layer li: N % 4 == 0, N and K <= 4096,
        16-B aligned rows of its activations, gradient and mask operands."""
        _, fi, fo, _ = self.layout[li]
        for t in (g, acts[li], acts[-1]):
            if t.stride(1) != 1 or t.stride(0) % 4 or t.data_ptr() % 16:
                return False
        return fo % 4 == 0 and fo <= 4096 and fi <= 4096

    def backward_acts(self, acts: List[torch.Tensor], flat: torch.Tensor, gout: torch.Tensor,
                      gscale: Optional[torch.Tensor], need_input_grad: bool):
        """(d x, d flat) from the saved activations.  Per layer l from the top:
        [dW_l; db_l] = [h_{l-1} | 1]^T G_l by ONE tt_mlp_wgrad straight into the
        flat gradient (the top layer's G_L = relu'(h_L) * s * gout formed inside
        its loads), then ONE tt_mlp_rows for the layer below:
        G_{l-1} = (G_l W_l^T) * relu'(h_{l-1}) (the top layer's relu mask and
        scale applied to its A loads), or the input gradient dx = G_1 W_1^T.
        gout is not modified.  A layer outside tt_mlp_wgrad's contract (output
        width not a multiple of 4, or wider than 4096) takes its weight
        gradient from torch (the only vendor GEMM left, never at the
        reference's configurations)."""
        gflat = torch.empty_like(flat)
        imgs = self.__dict__["_images"]  # packed by this step's forward (same flat)
        L = len(self.layout)
        g = gout
        for li in range(L - 1, -1, -1):
            w_off, fi, fo, _ = self.layout[li]
            dwb = gflat[w_off:w_off + (fi + 1) * fo].view(fi + 1, fo)
            top = li == L - 1
            if self._wgrad_fits(li, g, acts):
                if top:
                    hip_ops.mlp_wgrad(acts[li], gout, dwb, gmask=acts[L], scale=gscale)
                else:
                    hip_ops.mlp_wgrad(acts[li], g, dwb)
            else:
                gm = g * (acts[L] > 0) * (gscale if gscale is not None else 1.0) if top else g
                torch.mm(acts[li].t(), gm, out=dwb[:fi])
                torch.sum(gm, 0, out=dwb[fi])
            if li == 0 and not need_input_grad:
                return None, gflat
            ld = (fi + 3) // 4 * 4  # 16-B rows for the kernel's vector stores
            out = torch.empty(g.shape[0], ld, dtype=torch.float32, device=g.device)[:, :fi]
            g = hip_ops.mlp_rows(g, imgs[("t", li)], fo, fi, out,
                                 amask=acts[L] if top else None, scale=gscale if top else None,
                                 cmask=acts[li] if li > 0 else None)
        return g, gflat

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        if torch.is_grad_enabled() and (x.requires_grad or self.flat.requires_grad):
            return _DenseStackFn.apply(x, self.flat, self)
        return self.forward_acts(x, self.flat.detach())[-1]


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

    def save(self, model_path: str) -> None:
        """Weights (.pt), architecture (.json), vocabularies (.npz)."""
        from pkg.modelling import export

        export.save_tower(self, model_path[:-3] if model_path.endswith(".pt") else model_path)

    @classmethod
    def load(cls, model_path: str, device: Optional[torch.device] = None) -> "Tower":
        from pkg.modelling import export

        return export.load_tower(model_path[:-3] if model_path.endswith(".pt") else model_path, device)

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        for t in self.input_layer.tables():
            t.weight.copy_(sd[f"tables.{t.name}"].to(t.weight.device))
        with torch.no_grad():
            self.dense.flat.copy_(sd["dense.flat"].to(self.dense.flat.device))
