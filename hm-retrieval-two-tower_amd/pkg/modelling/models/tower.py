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
    input gradient of the first layer;
  * forward_acts_pair / backward_acts_pair: the same per-layer work of the
    query and the candidate tower as ONE launch per layer and kind
    (tt_mlp_rows_pair, tt_mlp_wgrad_pair) on one stream, bit-identical to the
    single calls.
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

__all__ = ["Tower", "DenseStack", "pair_compatible", "forward_acts_pair", "backward_acts_pair"]

# DenseStack.backward_acts: every input gradient before any weight gradient
# (C3 step, 3 interleaved runs each: unfused 0.535-0.541 vs 0.533-0.536 ms;
# fused apply 0.570-0.573 vs 0.564-0.565 ms — off)
IGRAD_FIRST = os.environ.get("TT_IGRAD_FIRST", "0") == "1"


def _rows(p: dict) -> torch.Tensor:
    """hip_ops.mlp_rows on a problem dict (as mlp_rows_pair takes them)."""
    q = dict(p)
    return hip_ops.mlp_rows(q.pop("a"), q.pop("img"), q.pop("k"), q.pop("n"), q.pop("out"), **q)


def _aligned(t: torch.Tensor, width: Optional[int] = None) -> torch.Tensor:
    """t itself when its rows are 16-B aligned and it has `width` columns
    (default: its own), else a copy with 16-B rows, zero-padded to `width`."""
    width = t.shape[1] if width is None else width
    if t.stride(1) == 1 and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0 and t.shape[1] == width:
        return t
    out = torch.zeros(t.shape[0], (width + 3) // 4 * 4, dtype=t.dtype, device=t.device)
    out[:, :t.shape[1]] = t
    return out[:, :width]


def _wgrad(p: dict) -> torch.Tensor:
    q = dict(p)
    return hip_ops.mlp_wgrad(q.pop("a"), q.pop("g"), q.pop("dwb"), **q)


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
            if not 1 <= u <= 384 or fan_in > 384:
                # tt_mlp_rows' output width (the forward's units, the input
                # gradient's fan-in) is at most 384: no fallback GEMM
                raise ValueError(f"Dense layer {fan_in} -> {u}: widths must be in 1..384 (tt_mlp_rows)")
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
        # (accumulator of flat, lr, eps) while a train step applies this
        # stack's Adagrad inside its weight-gradient launches (TwoTowerModel:
        # FUSED_DENSE_WGRAD); the layers it was applied to in this backward
        self.fused_adagrad = None
        self.fused_applied: set = set()

    def params(self, flat: Optional[torch.Tensor] = None):
        f = self.flat if flat is None else flat
        return [(f[w:w + fi * fo].view(fi, fo), f[b:b + fo]) for w, fi, fo, b in self.layout]

    def _pack_jobs(self, flat: torch.Tensor) -> Tuple[Dict[Tuple[str, int], torch.Tensor], list]:
        """Image buffers (owned by the stack: fixed addresses, graph-capturable)
        and the tt_mlp_pack_many jobs that fill them from `flat`."""
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
        return imgs, jobs

    def prepack_jobs(self, flat: torch.Tensor) -> list:
        """The pack jobs of this stack's images for a forward on `flat`, to be
        run by another launch (the train step's gather: hip_ops.gather_multi
        with pack_jobs); the next forward_acts on the same flat then uses the
        images as they are (once)."""
        imgs, jobs = self._pack_jobs(flat)
        self.__dict__["_prepacked"] = flat.data_ptr()
        return jobs

    def _images_for(self, flat: torch.Tensor) -> Dict[Tuple[str, int], torch.Tensor]:
        """This forward's images: prepacked by the gather launch, or packed now."""
        if self.__dict__.get("_prepacked") == flat.data_ptr():
            self.__dict__["_prepacked"] = None
            return self.__dict__["_images"]
        return self._pack_images(flat)

    def _pack_images(self, flat: torch.Tensor) -> Dict[Tuple[str, int], torch.Tensor]:
        """Every layer's packed bf16 hi/lo weight images, forward ("f": B = W)
        and transposed ("t": B = W^T, the input-gradient GEMMs), in ONE
        tt_mlp_pack_many launch.  Packed at the start of each forward, so they
        always match `flat`."""
        imgs, jobs = self._pack_jobs(flat)
        for i in range(0, len(jobs), 8):
            hip_ops.mlp_pack_many(jobs[i:i + 8])
        return imgs

    def _fwd_problem(self, li: int, h: torch.Tensor, flat: torch.Tensor, imgs) -> dict:
        w, b = self.params(flat)[li]
        n = w.shape[1]
        # hidden layers: 16-B output rows (the next layer's A operand); the top
        # layer's output (the joint embedding) stays contiguous
        ld = n if li == len(self.layout) - 1 else (n + 3) // 4 * 4
        out = torch.empty(h.shape[0], ld, dtype=torch.float32, device=h.device)[:, :n]
        return dict(a=h, img=imgs[("f", li)], k=w.shape[0], n=n, out=out, bias=b, relu=True)

    def forward_acts(self, x: torch.Tensor, flat: torch.Tensor) -> List[torch.Tensor]:
        """[x, h_1, ..., h_L] with h_l = relu(h_{l-1} W_l + b_l) (tt_mlp_rows)."""
        imgs = self._images_for(flat)
        acts = [x]
        for li in range(len(self.layout)):
            p = self._fwd_problem(li, acts[-1], flat, imgs)
            acts.append(_rows(p))
        return acts

    def _wgrad_fits(self, li: int, g: torch.Tensor, acts: List[torch.Tensor]) -> bool:
        """tt_mlp_wgrad's alignment contract for layer li: N % 4 == 0 and
        16-B aligned rows of its activations, gradient and mask operands
        (widths over 384 are refused when the stack is built)."""
        _, fi, fo, _ = self.layout[li]
        for t in (g, acts[li], acts[-1]):
            if t.stride(1) != 1 or t.stride(0) % 4 or t.data_ptr() % 16:
                return False
        return fo % 4 == 0 and fo <= 4096 and fi <= 4096

    def _wgrad_problem(self, li: int, acts, gflat, gout, g, gscale) -> dict:
        """Layer li's [dW; db] as an mlp_wgrad problem (the top layer's
        ReluGrad and scale applied to gout inside its loads)."""
        w_off, fi, fo, _ = self.layout[li]
        dwb = gflat[w_off:w_off + (fi + 1) * fo].view(fi + 1, fo)
        if li == len(self.layout) - 1:
            return dict(a=acts[li], g=gout, dwb=dwb, gmask=acts[-1], scale=gscale)
        return dict(a=acts[li], g=g, dwb=dwb)

    def _wgrad_padded(self, li: int, acts, gflat, g, gscale) -> None:
        """The weight gradient outside tt_mlp_wgrad's alignment contract (an
        output width that is not a multiple of 4, or unaligned operand rows):
        the same tt_mlp_wgrad on zero-padded copies — operands with 16-B rows
        of width ceil4(N) (the padding columns of G are zero, so their
        gradient columns are zero and dropped) — then the [K + 1, N] block
        copied into the flat gradient.  The same sums in the same order as an
        aligned layer's (no vendor GEMM)."""
        w_off, fi, fo, _ = self.layout[li]
        dwb = gflat[w_off:w_off + (fi + 1) * fo].view(fi + 1, fo)
        top = li == len(self.layout) - 1
        n4 = (fo + 3) // 4 * 4

        a = _aligned(acts[li])
        gp = _aligned(g, n4)
        out = torch.empty(fi + 1, n4, dtype=torch.float32, device=g.device)
        if top:
            hip_ops.mlp_wgrad(a, gp, out, gmask=_aligned(acts[-1], n4), scale=gscale)
        else:
            hip_ops.mlp_wgrad(a, gp, out)
        dwb.copy_(out[:, :fo])

    def _igrad_problem(self, li: int, acts, g, gscale) -> dict:
        """G_{l-1} = (G_l W_l^T) * relu'(h_{l-1}) (the top layer's relu mask and
        scale on its A loads), or dx = G_1 W_1^T, as an mlp_rows problem."""
        _, fi, fo, _ = self.layout[li]
        top = li == len(self.layout) - 1
        ld = (fi + 3) // 4 * 4  # 16-B rows for the kernel's vector stores
        out = torch.empty(g.shape[0], ld, dtype=torch.float32, device=g.device)[:, :fi]
        amask = acts[-1] if top else None
        if top and fo % 4:  # the joint embedding's rows are not 16-B: aligned copies
            g, amask = _aligned(g), _aligned(amask)
        return dict(a=g, img=self.__dict__["_images"][("t", li)], k=fo, n=fi, out=out,
                    amask=amask, scale=gscale if top else None,
                    cmask=acts[li] if li > 0 else None)

    def backward_acts(self, acts: List[torch.Tensor], flat: torch.Tensor, gout: torch.Tensor,
                      gscale: Optional[torch.Tensor], need_input_grad: bool, on_dx=None):
        """(d x, d flat) from the saved activations.  Per layer l from the top:
        [dW_l; db_l] = [h_{l-1} | 1]^T G_l by ONE tt_mlp_wgrad straight into the
        flat gradient (the top layer's G_L = relu'(h_L) * s * gout formed inside
        its loads), then ONE tt_mlp_rows for the layer below:
        G_{l-1} = (G_l W_l^T) * relu'(h_{l-1}) (the top layer's relu mask and
        scale applied to its A loads), or the input gradient dx = G_1 W_1^T.
        gout is not modified.  A layer outside tt_mlp_wgrad's alignment
        contract (output width not a multiple of 4) runs it on zero-padded
        copies (_wgrad_padded).  Images: packed by this step's forward
        (same flat).  With TT_IGRAD_FIRST=1 the input-gradient chain runs
        before the weight gradients, and on_dx(dx), if given, is called
        between them (the fused step's embedding update); the kernels and
        their results are the same in either order (off by default: same step
        time unfused, slower fused — DESIGN §9)."""
        if IGRAD_FIRST:
            # the input-gradient chain first (the embedding update waits for it,
            # the weight gradients do not), on_dx(dx) between the two
            dx, finish = self.backward_split(acts, flat, gout, gscale, need_input_grad)
            if on_dx is not None:
                on_dx(dx)
            return dx, finish()
        gflat = torch.empty_like(flat)
        g = gout
        for li in range(len(self.layout) - 1, -1, -1):
            self._wgrad_layer(li, acts, gflat, gout, g, gscale)
            if li == 0 and not need_input_grad:
                g = None
                break
            p = self._igrad_problem(li, acts, g, gscale)
            g = _rows(p)
        if on_dx is not None:
            on_dx(g)
        return g, gflat

    def backward_split(self, acts: List[torch.Tensor], flat: torch.Tensor, gout: torch.Tensor,
                       gscale: Optional[torch.Tensor], need_input_grad: bool):
        """backward_acts in two phases: the input-gradient chain now (returns
        dx, None without need_input_grad) and the weight gradients when the
        returned finish() is called (returns the flat gradient) — the same
        kernels on the same operands as backward_acts, in IGRAD_FIRST order;
        finish() applies the fused Adagrad step that was set at the split,
        whenever it runs."""
        gs, g, dx = {}, gout, None
        for li in range(len(self.layout) - 1, -1, -1):
            gs[li] = g
            if li == 0 and not need_input_grad:
                break
            g = _rows(self._igrad_problem(li, acts, g, gscale))
            if li == 0:
                dx = g
        fused_adagrad = self.fused_adagrad

        def finish() -> torch.Tensor:
            gflat = torch.empty_like(flat)
            prev, self.fused_adagrad = self.fused_adagrad, fused_adagrad
            try:
                for li in range(len(self.layout) - 1, -1, -1):
                    self._wgrad_layer(li, acts, gflat, gout, gs[li], gscale)
            finally:
                self.fused_adagrad = prev
            return gflat

        return dx, finish

    def _layer_adagrad(self, li: int):
        """(param, accum, lr, eps) of layer li for its weight-gradient launches
        to apply (marked in fused_applied), or None: no fused step, or the
        layer's region of the flat buffer is not 16-B aligned (a layer after
        one whose width is not a multiple of 4: the dense step applies it)."""
        if self.fused_adagrad is None:
            return None
        acc, lr, eps = self.fused_adagrad
        w_off, fi, fo, _ = self.layout[li]
        n = (fi + 1) * fo
        param, accum = self.flat.data[w_off:w_off + n], acc[w_off:w_off + n]
        if param.data_ptr() % 16 or accum.data_ptr() % 16:
            return None
        self.fused_applied.add(li)
        return param, accum, lr, eps

    def _wgrad_layer(self, li, acts, gflat, gout, g, gscale) -> None:
        if self._wgrad_fits(li, g, acts):
            p = self._wgrad_problem(li, acts, gflat, gout, g, gscale)
            ad = self._layer_adagrad(li)
            if ad is not None:  # this layer's Adagrad step in the same launches
                p["adagrad"] = ad
            _wgrad(p)
        else:
            self._wgrad_padded(li, acts, gflat, g, gscale)

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        if torch.is_grad_enabled() and (x.requires_grad or self.flat.requires_grad):
            return _DenseStackFn.apply(x, self.flat, self)
        return self.forward_acts(x, self.flat.detach())[-1]


def pair_compatible(a: "DenseStack", b: "DenseStack") -> bool:
    """Both towers' layers can run as paired launches (same depth)."""
    return len(a.layout) == len(b.layout) and len(a.layout) > 0


def forward_acts_pair(stacks, xs, flats) -> List[List[torch.Tensor]]:
    """DenseStack.forward_acts of the two towers on ONE stream with every
    launch shared: one tt_mlp_pack_many for both towers' images (8 jobs at
    one hidden layer), then one tt_mlp_rows_pair per layer."""
    pre = [st.__dict__.get("_prepacked") == f.data_ptr() for st, f in zip(stacks, flats)]
    packed = [st._pack_jobs(f) for st, f in zip(stacks, flats)]
    jobs = [j for p, (_, js) in zip(pre, packed) if not p for j in js]
    for st, p in zip(stacks, pre):
        if p:
            st.__dict__["_prepacked"] = None
    for i in range(0, len(jobs), 8):
        hip_ops.mlp_pack_many(jobs[i:i + 8])
    acts = [[xs[0]], [xs[1]]]
    for li in range(len(stacks[0].layout)):
        probs = [st._fwd_problem(li, a[-1], f, pk[0]) for st, a, f, pk in zip(stacks, acts, flats, packed)]
        hip_ops.mlp_rows_pair(probs)
        for a, p in zip(acts, probs):
            a.append(p["out"])
    return acts


def backward_acts_pair(stacks, acts, flats, gouts, gscale, need_input_grad):
    """DenseStack.backward_acts of the two towers with each layer's two weight
    gradients in one tt_mlp_wgrad_pair and its two input-gradient GEMMs in one
    tt_mlp_rows_pair (bit-identical to the single calls).  Returns
    [(dx, dflat)] per tower."""
    gflats = [torch.empty_like(f) for f in flats]
    gs = list(gouts)
    L = len(stacks[0].layout)
    for li in range(L - 1, -1, -1):
        fits = [st._wgrad_fits(li, g, a) for st, g, a in zip(stacks, gs, acts)]
        if all(fits):
            hip_ops.mlp_wgrad_pair([st._wgrad_problem(li, a, gf, go, g, gscale)
                                    for st, a, gf, go, g in zip(stacks, acts, gflats, gouts, gs)])
        else:
            for t, st in enumerate(stacks):
                if fits[t]:
                    p = st._wgrad_problem(li, acts[t], gflats[t], gouts[t], gs[t], gscale)
                    _wgrad(p)
                else:
                    st._wgrad_padded(li, acts[t], gflats[t], gs[t], gscale)
        want = [li > 0 or need_input_grad[t] for t in range(2)]
        probs = [st._igrad_problem(li, a, g, gscale) if w else None
                 for st, a, g, w in zip(stacks, acts, gs, want)]
        if all(want):
            hip_ops.mlp_rows_pair(probs)
        else:
            for p in probs:
                if p is not None:
                    _rows(p)
        gs = [p["out"] if p is not None else None for p in probs]
    return [(gs[t], gflats[t]) for t in range(2)]


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
