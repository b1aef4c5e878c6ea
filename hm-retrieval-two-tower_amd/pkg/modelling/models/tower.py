"""Tower: InputLayer -> Dense(relu)* -> Dense(E, relu)
(mirror of /root/reference/pkg/modelling/models/tower.py:8-91).

Dense layers follow Keras defaults: kernel [fan_in, units] glorot_uniform,
zero bias, relu on every layer including the last (tower.py:45,48), so the
joint embeddings are non-negative.  All kernels and biases of a tower live in
ONE flat fp32 buffer (views per layer; each layer's bias right after its
kernel), so its gradient is one contiguous tensor and the dense optimizer
step is a single tt_dense_* launch.  Three GEMM backends (DenseStack.backend,
default from $TT_TOWER_BACKEND, else "mlp"):
  * "mlp" (default): libtt's tt_mlp_rows (bf16x3 MFMA, fp32-faithful) for the
    forward GEMMs (bias + relu epilogue) and the input-gradient GEMMs (the
    layer below's ReluGrad mask and BiasAddGrad column sums fused into the
    epilogue); one tt_mlp_pack_many launch per tower per step packs its
    weight images; the weight gradients stay hipBLASLt split-K +
    tt_sum_slices, the top layer's ReluGrad/BiasAddGrad tt_relu_bias_grad;
  * "hipblaslt": torch fp32 GEMMs (bias + relu in the forward GEMM's
    epilogue); libtt's tt_relu_bias_grad for the ReluGrad/BiasAddGrad
    pair and tt_sum_slices for the split-K weight gradient;
  * "tt": libtt's tt_gemm on bf16 MFMA (GEMM_BF16X3 hi/lo split =
    fp32-faithful, or GEMM_BF16): bias + relu fused into the forward
    epilogue, the relu mask applied while loading the gradient operand, the
    bias gradient as the ones-row of the weight-gradient GEMM.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import torch

from pkg.schema.features import Feature
from pkg.modelling import hip_ops
from pkg.modelling.device import default_device, make_generator
from pkg.modelling.layers.input_layer import InputLayer
from pkg.modelling.models.abstract_keras_model import AbstractKerasModel, TensorSpec

__all__ = ["Tower", "DenseStack"]


# weight-gradient side streams of the "mlp" backend (losses.WGRAD_STREAM)
_WGRAD_STREAMS = {}
# the "mlp" backend's weight gradients: "blas" (default: hipBLASLt split-K +
# tt_sum_slices, with the separate ReluGrad / bias-gradient launches) or "tt"
# (tt_mlp_wgrad: no vendor GEMM and no glue launch in the step, but the C3
# step measured 0.609 vs 0.595 ms — its split partials and the activation
# re-reads of its column groups keep it HBM-bound at 28-30 us per layer)
WGRAD_KERNEL = os.environ.get("TT_WGRAD", "blas")


def _wgrad_stream(cur: torch.cuda.Stream) -> torch.cuda.Stream:
    """The weight-gradient stream of the tower whose backward runs now, one per
    device and workspace scope (query / candidate tower): created by the first
    (eager) step, never inside a graph capture, whose stream is a fresh one."""
    key = (cur.device.index, hip_ops.Workspace._scope)
    if key not in _WGRAD_STREAMS:
        _WGRAD_STREAMS[key] = torch.cuda.Stream(device=cur.device)
    return _WGRAD_STREAMS[key]


def _splitk_mm_tn(a: torch.Tensor, g: torch.Tensor, out: torch.Tensor, splits: int = 16) -> None:
    """out = a^T g for tall a [B, fin], g [B, fout] (the weight gradient).
    hipBLASLt runs this skinny, K=B-long product on a handful of tiles; a
    batched split over B (bmm of `splits` slices, then tt_sum_slices in slice
    order) fills the GPU (~3x faster at B=16384)."""
    B = a.shape[0]
    if B >= 4096 and B % splits == 0:
        part = torch.bmm(a.view(splits, B // splits, a.shape[1]).transpose(1, 2),
                         g.view(splits, B // splits, g.shape[1]))
        hip_ops.sum_slices(part, out)
    else:
        torch.mm(a.t(), g, out=out)


def _mm_fast_fp32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b through hipBLASLt's fast-fp32 path (torch's allow_tf32 switch; on
    gfx950 an emulated mode measured at ~4e-6 relative error vs fp64 for the
    C3 tower shapes, i.e. fp32-faithful).  For the input-gradient GEMM it
    selects a far better kernel when N is not a tile multiple (query tower,
    N = 258: 44.7 -> 19.4 us; candidate N = 200: 24.1 -> 20.0 us; at N = 256
    it is 7 % slower, and the forward and weight-gradient GEMMs gain nothing:
    tools/tf32_probe.py), so only ragged input-gradient GEMMs take it."""
    prev = torch.backends.cuda.matmul.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = True
    try:
        return torch.mm(a, b)
    finally:
        torch.backends.cuda.matmul.allow_tf32 = prev


def _weight_grad_splits(rows: int, fan_in: int, fan_out: int) -> int:
    """Split-K factor of the weight-gradient GEMM ([fan_in+1, fan_out] over
    `rows`): enough workgroups to fill 256 CUs twice, >= 256 rows per split."""
    bm = 64 if fan_out > 128 else 128
    tiles = -(-(fan_in + 1) // bm) * -(-fan_out // (16384 // bm))
    s = 1
    while tiles * s < 512 and rows // (2 * s) >= 256:
        s *= 2
    return s


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
        gx, gflat = ctx.stack.backward_acts(acts, flat, gout.contiguous(), None, ctx.needs_input_grad[0],
                                            inplace=False)
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
        # GEMM backend: "hipblaslt" (torch fp32 GEMMs + libtt relu/bias-grad and
        # split-K reduction), "mlp" (libtt tt_mlp_rows, bf16x3 MFMA, for the
        # forward and input-gradient GEMMs; weight gradients as "hipblaslt"),
        # or "tt" (libtt tt_gemm, bf16 MFMA; `precision` GEMM_BF16X3 =
        # fp32-faithful hi/lo split, GEMM_BF16 = plain bf16)
        self.backend = os.environ.get("TT_TOWER_BACKEND", "mlp")
        self.precision = hip_ops.GEMM_BF16X3

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
        """[x, h_1, ..., h_L] with h_l = relu(h_{l-1} W_l + b_l)."""
        if self.backend == "tt":
            return self._forward_tt(x, flat)
        if self.backend == "mlp":
            imgs = self._pack_images(flat)
            acts = [x]
            h = x
            for li, (w, b) in enumerate(self.params(flat)):
                out = torch.empty(h.shape[0], w.shape[1], dtype=torch.float32, device=h.device)
                h = hip_ops.mlp_rows(h, imgs[("f", li)], w.shape[0], w.shape[1], out, bias=b, relu=True)
                acts.append(h)
            return acts
        acts = [x]
        h = x
        for w, b in self.params(flat):
            h = torch._addmm_activation(b, h, w)  # hipBLASLt, bias + relu epilogue
            acts.append(h)
        return acts

    def backward_acts(self, acts: List[torch.Tensor], flat: torch.Tensor, gout: torch.Tensor,
                      gscale: Optional[torch.Tensor], need_input_grad: bool, inplace: bool = True,
                      joins: Optional[List[torch.cuda.Stream]] = None):
        """(d x, d flat) from the saved activations.  hipBLASLt backend, per
        layer: one tt_relu_bias_grad (relu mask x the incoming gradient, times
        gscale on the top layer, and the bias gradient), the weight gradient
        (split-K GEMM + tt_sum_slices) and the input gradient (GEMM).
        inplace: gout may be overwritten.  joins ("mlp" backend, GPU): the weight
        gradients run on a side stream appended to this list, which the caller
        must make its stream wait on before using d flat."""
        if self.backend == "tt":
            return self._backward_tt(acts, flat, gout, gscale, need_input_grad)
        if self.backend == "mlp":
            return self._backward_mlp(acts, flat, gout, gscale, need_input_grad, inplace, joins)
        gflat = torch.empty_like(flat)
        params = self.params(flat)
        gparams = self.params(gflat)
        g = gout
        for li in range(len(params) - 1, -1, -1):
            dw, db = gparams[li]
            top = li == len(params) - 1
            g, _ = hip_ops.relu_bias_grad(g, acts[li + 1], gscale if top else None,
                                          out=None if (top and not inplace) else g, db=db)
            _splitk_mm_tn(acts[li], g, dw)
            if li > 0 or need_input_grad:
                w = params[li][0]
                # fast path only where it picks the better kernel (ragged output widths)
                g = _mm_fast_fp32(g, w.t()) if w.shape[0] % 64 else torch.mm(g, w.t())
        return (g if need_input_grad else None), gflat

    def _backward_mlp(self, acts: List[torch.Tensor], flat: torch.Tensor, gout: torch.Tensor,
                      gscale: Optional[torch.Tensor], need_input_grad: bool, inplace: bool,
                      joins: Optional[List[torch.cuda.Stream]] = None):
        """"mlp" backend.  Top layer: G_L = relu'(h_L) * s * gout and db_L by
        one tt_relu_bias_grad.  Per layer l from the top: [dW_l] = h_{l-1}^T G_l
        (hipBLASLt split-K + tt_sum_slices), then ONE tt_mlp_rows for the layer
        below: G_{l-1} = (G_l W_l^T) * relu'(h_{l-1}) with db_{l-1} = colsum
        G_{l-1} in its epilogue (the ReluGrad / BiasAddGrad pair fused), or the
        input gradient dx = G_1 W_1^T (16-B padded rows, returned as a view)."""
        if WGRAD_KERNEL == "tt" and gout.is_cuda and self._wgrad_fits(gout, acts):
            return self._backward_mlp_tt(acts, flat, gout, gscale, need_input_grad)
        gflat = torch.empty_like(flat)
        params = self.params(flat)
        gparams = self.params(gflat)
        imgs = self.__dict__["_images"]  # packed by this step's forward (same flat)
        L = len(params)
        g, _ = hip_ops.relu_bias_grad(gout, acts[L], gscale, out=gout if inplace else None, db=gparams[L - 1][1])
        # joins given: the weight gradients (hipBLASLt) leave the input-gradient
        # chain (which gates the embedding update) for a stream of their own,
        # each started as soon as its G_l exists.  That stream never feeds back
        # into this one: the CALLER joins it from the capture's origin stream (a
        # captured branch that waits on a sub-branch it forked crashes
        # hipGraph instantiation on this ROCm).
        cur = torch.cuda.current_stream(g.device) if (joins is not None and g.is_cuda) else None
        ws = _wgrad_stream(cur) if cur is not None else None
        dx = None
        for li in range(L - 1, -1, -1):
            w = params[li][0]
            if ws is not None:
                ws.wait_stream(cur)
                with torch.cuda.stream(ws):
                    _splitk_mm_tn(acts[li], g, gparams[li][0])
                    g.record_stream(ws)
            else:
                _splitk_mm_tn(acts[li], g, gparams[li][0])
            if li == 0 and not need_input_grad:
                break
            fi, fo = w.shape
            ld = (fi + 3) // 4 * 4  # 16-B rows for the kernel's vector stores
            out = torch.empty(g.shape[0], ld, dtype=torch.float32, device=g.device)[:, :fi]
            if li > 0:
                g = hip_ops.mlp_rows(g, imgs[("t", li)], fo, fi, out, cmask=acts[li], colsum=gparams[li - 1][1])
            else:
                dx = g = hip_ops.mlp_rows(g, imgs[("t", li)], fo, fi, out)
        if ws is not None:
            joins.append(ws)
        return dx, gflat

    def _wgrad_fits(self, gout: torch.Tensor, acts: List[torch.Tensor]) -> bool:
        """tt_mlp_wgrad's contract: N % 4 == 0, 16-B aligned rows of the
        activations and gradients (16-B vector loads)."""
        for t in [gout] + list(acts):
            if t.stride(1) != 1 or t.stride(0) % 4 or t.data_ptr() % 16:
                return False
        return all(fo % 4 == 0 and fo <= 4096 and fi <= 4096 for _, fi, fo, _ in self.layout)

    def _backward_mlp_tt(self, acts: List[torch.Tensor], flat: torch.Tensor, gout: torch.Tensor,
                         gscale: Optional[torch.Tensor], need_input_grad: bool):
        """"mlp" backend, every GEMM hand-written.  Per layer l from the top:
        [dW_l; db_l] = [h_{l-1} | 1]^T G_l by ONE tt_mlp_wgrad straight into
        the flat gradient (the top layer's G_L = relu'(h_L) * s * gout is formed
        inside its loads), then ONE tt_mlp_rows for the layer below:
        G_{l-1} = (G_l W_l^T) * relu'(h_{l-1}) (the top layer's relu mask and
        scale applied to its A loads), or the input gradient dx = G_1 W_1^T.
        No ReluGrad / BiasAddGrad / split-K glue launches remain.  gout is not
        modified."""
        gflat = torch.empty_like(flat)
        imgs = self.__dict__["_images"]  # packed by this step's forward (same flat)
        L = len(self.layout)
        g = gout
        for li in range(L - 1, -1, -1):
            w_off, fi, fo, _ = self.layout[li]
            dwb = gflat[w_off:w_off + (fi + 1) * fo].view(fi + 1, fo)
            top = li == L - 1
            if top:
                hip_ops.mlp_wgrad(acts[li], gout, dwb, gmask=acts[L], scale=gscale)
            else:
                hip_ops.mlp_wgrad(acts[li], g, dwb)
            if li == 0 and not need_input_grad:
                return None, gflat
            ld = (fi + 3) // 4 * 4  # 16-B rows for the kernel's vector stores
            out = torch.empty(g.shape[0], ld, dtype=torch.float32, device=g.device)[:, :fi]
            g = hip_ops.mlp_rows(g, imgs[("t", li)], fo, fi, out,
                                 amask=acts[L] if top else None, scale=gscale if top else None,
                                 cmask=acts[li] if li > 0 else None)
        return g, gflat

    def _forward_tt(self, x: torch.Tensor, flat: torch.Tensor) -> List[torch.Tensor]:
        """libtt backend: one tt_gemm per layer (bias + relu in the epilogue)."""
        acts = [x]
        h = x
        for w, b in self.params(flat):
            out = torch.empty(h.shape[0], w.shape[1], dtype=torch.float32, device=h.device)
            h = hip_ops.gemm(h, w, out, bias=b, relu=True, precision=self.precision)
            acts.append(h)
        return acts

    def _backward_tt(self, acts: List[torch.Tensor], flat: torch.Tensor, gout: torch.Tensor,
                     gscale: Optional[torch.Tensor], need_input_grad: bool):
        """libtt backend.  Per layer l (G = relu'(h_l) * s * g, s = gscale on the
        top layer, applied inside the GEMM loads): [dW_l; db_l] = [h_{l-1}; 1]^T G
        as one split-K tt_gemm + tt_sum_slices written straight into the flat
        gradient, and g_{l-1} = G W_l^T.  gout is not modified."""
        gflat = torch.empty_like(flat)
        params = self.params(flat)
        g = gout
        for li in range(len(params) - 1, -1, -1):
            w_off, fi, fo, _ = self.layout[li]
            w = params[li][0]
            x, act = acts[li], acts[li + 1]
            s = gscale if li == len(params) - 1 else None
            rows = x.shape[0]
            dwb = gflat[w_off:w_off + (fi + 1) * fo].view(fi + 1, fo)
            splits = _weight_grad_splits(rows, fi, fo)
            if splits > 1:
                part = hip_ops.Workspace.get(splits * (fi + 1) * fo * 4, x.device, "dense_wgrad")
                part = part[:splits * (fi + 1) * fo * 4].view(torch.float32).view(splits, fi + 1, fo)
                hip_ops.gemm(x, g, part, a_t=True, mask=act, mask_on="b", scale=s, ones_row=True, splits=splits,
                             precision=self.precision)
                hip_ops.sum_slices(part, dwb)
            else:
                hip_ops.gemm(x, g, dwb, a_t=True, mask=act, mask_on="b", scale=s, ones_row=True,
                             precision=self.precision)
            if li > 0 or need_input_grad:
                gx = torch.empty(rows, fi, dtype=torch.float32, device=x.device)
                g = hip_ops.gemm(g, w, gx, b_t=True, mask=act, mask_on="a", scale=s, precision=self.precision)
        return (g if need_input_grad else None), gflat

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
