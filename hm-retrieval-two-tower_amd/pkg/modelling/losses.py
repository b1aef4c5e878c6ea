"""In-batch softmax cross-entropy with eye labels, fused on the GPU.

Replaces, in one autograd node, the reference's chain
  TwoTowerModel.call matmul          (two_tower_model.py:92)
  LogQCorrection                     (two_tower_model.py:113-116)
  labels = eye(B); CategoricalCrossentropy(from_logits=True, reduction=SUM)
                                     (two_tower_model.py:119-122, runner.py:78-83)
The forward runs both libtt passes (rows: lse, row loss, dQ; cols: dC) and
keeps dQ, dC for the backward, which only scales them by the incoming
gradient.  The [B, B] score matrix never exists.
"""
from __future__ import annotations

import os

from typing import Optional

import torch

from pkg.modelling import hip_ops

__all__ = ["InBatchSoftmaxCrossEntropy", "inbatch_softmax_xent", "towers_inbatch_softmax_xent",
           "global_inbatch_grads", "global_towers_inbatch_softmax_xent", "TOWER_C_SCOPE"]


def x3_scores() -> bool:
    """TT_INBATCH_X3=1 (read at each call): the single-device in-batch loss
    with fp32-faithful products (hip_ops.inbatch_fused(x3=True): S and P.V
    as bf16x3 products) — the reference's fp32 logits and gradients to
    ~2^-16, dQ / dC within 1e-3 of fp64 at trained score magnitudes; ~3x the
    passes' time.  The
    default is the bf16-operand contract (include/tt.h K5-K7)."""
    return os.environ.get("TT_INBATCH_X3", "0") == "1"


class _InBatchXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, c, logq, scale):
        lse, row_loss, dq, dc = hip_ops.inbatch_fused(q, c, logq, x3=x3_scores())
        ctx.scale = scale
        ctx.save_for_backward(dq, dc)
        return hip_ops.loss_sum(row_loss, scale)

    @staticmethod
    def backward(ctx, g):
        dq, dc = ctx.saved_tensors
        s = g * ctx.scale
        return dq * s, dc * s, None, None


_SIDE: dict = {}

# Workspace scope of the candidate tower's work on its own stream (the fused
# train step sorts and applies that tower's embedding update in this scope).
TOWER_C_SCOPE = "tower_c"

def _tower_stream(device: torch.device) -> torch.cuda.Stream:
    """The stream the candidate tower's MLP runs on, beside the query tower's."""
    key = device.index if device.index is not None else torch.cuda.current_device()
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=device)
    return _SIDE[key]


# The global-negatives step runs the two towers on two streams from this many
# rows per rank (TT_GLOBAL_TOWER_STREAMS overrides; 0: always one stream).
# World-1 sharded step, interleaved pairs: 16384 rows 0.896-0.903 vs
# 0.942-0.945 ms; 2048 rows (an 8-way split) 0.579-0.605 vs 0.562-0.599.
GLOBAL_TOWER_STREAMS = int(os.environ.get("TT_GLOBAL_TOWER_STREAMS", "4096"))
# The single-GPU step's towers on two streams (TT_TOWER_STREAMS=0: one).
TOWER_STREAMS = int(os.environ.get("TT_TOWER_STREAMS", "1"))
# The single-device step's loss summed by an extra workgroup of the loss
# entry's last launch (tt_inbatch_softmax_xent_loss) instead of a tt_sum
# launch after it (TT_LOSS_IN_COMBINE=0); the same value bit for bit.
LOSS_IN_COMBINE = os.environ.get("TT_LOSS_IN_COMBINE", "1") == "1"
# The global-negatives loss at one rank through the single-device entry
# (TT_WORLD1_FUSED=0: the rows and columns entries, as at G > 1).
WORLD1_FUSED = os.environ.get("TT_WORLD1_FUSED", "1") == "1"
# Each tower's bf16 loss operand prepared on that tower's stream
# (tt_inbatch_prep) instead of one prep of both after the join.
SPLIT_PREP = os.environ.get("TT_SPLIT_PREP", "0") == "1"
# Both towers' layers as paired launches on one stream (tower.forward_acts_pair).
TOWER_PAIR = int(os.environ.get("TT_TOWER_PAIR", "0"))


def _paired(x: torch.Tensor, stack_q, stack_c) -> bool:
    from pkg.modelling.models.tower import pair_compatible
    return bool(TOWER_PAIR) and x.is_cuda and pair_compatible(stack_q, stack_c)


def _pair_forward(qi, ci, flat_q, flat_c, stack_q, stack_c):
    from pkg.modelling.models.tower import forward_acts_pair
    return forward_acts_pair((stack_q, stack_c), (qi, ci), (flat_q, flat_c))


def _pair_backward(ctx, qa, ca, flat_q, flat_c, dq, dc, s, on_tower=None):
    """Both towers' backward as paired launches; on_tower(1, ...) runs in the
    candidate tower's workspace scope (where its update was prepared)."""
    from pkg.modelling.models.tower import backward_acts_pair
    stack_q, stack_c = ctx.stacks
    (gqi, gflat_q), (gci, gflat_c) = backward_acts_pair(
        (stack_q, stack_c), (qa, ca), (flat_q, flat_c), (dq, dc), s,
        (ctx.needs_input_grad[0], ctx.needs_input_grad[1]))
    if on_tower is not None:
        with hip_ops.Workspace.scope(TOWER_C_SCOPE):
            on_tower(1, gci, gflat_c)
        on_tower(0, gqi, gflat_q)
    return gqi, gci, gflat_q, gflat_c


class _TowerFork:
    """Work in this block runs on the candidate tower's stream (forked from the
    current one) and workspace scope; plain on CPU tensors."""

    def __init__(self, like: torch.Tensor):
        self.cuda = _two_streams(like)
        self.dev = like.device

    def __enter__(self):
        self.scope = hip_ops.Workspace.scope(TOWER_C_SCOPE)
        self.scope.__enter__()
        if self.cuda:
            side = _tower_stream(self.dev)
            side.wait_stream(torch.cuda.current_stream())
            self.ctx = torch.cuda.stream(side)
            self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.cuda:
            self.ctx.__exit__(*exc)
        self.scope.__exit__(*exc)
        return False


def _tower_join(like: torch.Tensor) -> None:
    """The current stream waits for the candidate tower's stream (joined from
    the fork's origin: a captured branch must not join a sub-branch itself)."""
    if _two_streams(like):
        torch.cuda.current_stream().wait_stream(_tower_stream(like.device))


def _two_streams(like: torch.Tensor) -> bool:
    return like.is_cuda and GLOBAL_TOWER_STREAMS > 0 and like.shape[0] >= GLOBAL_TOWER_STREAMS


class _TowersInBatchXent(torch.autograd.Function):
    """Both tower MLPs and the in-batch loss as ONE autograd node.  The two
    towers' MLPs are independent chains of small GEMMs, so the candidate
    tower's forward and backward run on a second stream concurrently with
    the query tower's (fork / join with stream waits: captured as parallel
    branches of the step's hipGraph).  The backward hands the loss's incoming
    gradient to the top layers' weight-gradient and input-gradient kernels as
    a device scalar (no separate scaling pass over dQ, dC)."""

    @staticmethod
    def forward(ctx, qi, ci, flat_q, flat_c, logq, stack_q, stack_c, scale, on_tower=None, on_dx=None):
        ctx.pair = _paired(qi, stack_q, stack_c)
        ctx.on_dx = on_dx
        if ctx.pair:
            qa, ca = _pair_forward(qi, ci, flat_q, flat_c, stack_q, stack_c)
            return _TowersInBatchXent._finish(ctx, qa, ca, flat_q, flat_c, logq, stack_q, stack_c, scale, on_tower)
        main = torch.cuda.current_stream()
        side = _tower_stream(qi.device) if TOWER_STREAMS else main
        # SPLIT_PREP: each tower's bf16 copy for the loss is made on its own
        # stream right after its MLP (the workspace is fetched before the fork)
        ws = hip_ops.inbatch_fused_workspace(qi.shape[0], stack_q.out_dim, qi.device) if SPLIT_PREP else None
        side.wait_stream(main)
        with torch.cuda.stream(side), hip_ops.Workspace.scope(TOWER_C_SCOPE):
            ca = stack_c.forward_acts(ci, flat_c)
            if ws is not None:
                hip_ops.inbatch_prep(ca[-1], 1, logq, ws)
        qa = stack_q.forward_acts(qi, flat_q)
        if ws is not None:
            hip_ops.inbatch_prep(qa[-1], 0, None, ws)
        main.wait_stream(side)
        return _TowersInBatchXent._finish(ctx, qa, ca, flat_q, flat_c, logq, stack_q, stack_c, scale, on_tower, ws)

    @staticmethod
    def _finish(ctx, qa, ca, flat_q, flat_c, logq, stack_q, stack_c, scale, on_tower, ws=None):
        ctx.stacks = (stack_q, stack_c)
        ctx.nq = len(qa)
        ctx.scale = scale
        ctx.on_tower = on_tower
        if x3_scores():  # fp32-faithful scores (its own preparation and workspace)
            _, _, dq, dc, loss = hip_ops.inbatch_fused(qa[-1], ca[-1], logq, loss_scale=scale, x3=True)
            ctx.save_for_backward(flat_q, flat_c, dq, dc, *qa, *ca)
            return loss
        if LOSS_IN_COMBINE:  # the loss sum inside the loss entry's last launch
            _, _, dq, dc, loss = hip_ops.inbatch_fused(qa[-1], ca[-1], logq, ws=ws, prepped=ws is not None,
                                                       loss_scale=scale)
            ctx.save_for_backward(flat_q, flat_c, dq, dc, *qa, *ca)
            return loss
        _, row_loss, dq, dc = hip_ops.inbatch_fused(qa[-1], ca[-1], logq, ws=ws, prepped=ws is not None)
        ctx.save_for_backward(flat_q, flat_c, dq, dc, *qa, *ca)
        return hip_ops.loss_sum(row_loss, scale)

    @staticmethod
    def backward(ctx, g):
        flat_q, flat_c, dq, dc, *acts = ctx.saved_tensors
        qa, ca = acts[:ctx.nq], acts[ctx.nq:]
        s = (g * ctx.scale if ctx.scale != 1.0 else g).reshape(1).float().contiguous()
        stack_q, stack_c = ctx.stacks
        if ctx.pair:  # (on_dx unused: on_tower then applies each tower's whole update)
            return (*_pair_backward(ctx, qa, ca, flat_q, flat_c, dq, dc, s, ctx.on_tower),
                    None, None, None, None, None, None)
        on_dx = ctx.on_dx
        main = torch.cuda.current_stream()
        side = _tower_stream(dq.device) if TOWER_STREAMS else main
        side.wait_stream(main)
        with torch.cuda.stream(side), hip_ops.Workspace.scope(TOWER_C_SCOPE):
            # this tower's updates (on_dx: the embedding update once its input
            # gradient exists; on_tower: the rest), beside the other tower's backward
            gci, gflat_c = stack_c.backward_acts(ca, flat_c, dc, s, ctx.needs_input_grad[1],
                                                 on_dx=(lambda dx: on_dx(1, dx)) if on_dx is not None else None)
            if ctx.on_tower is not None:
                ctx.on_tower(1, gci, gflat_c)
        gqi, gflat_q = stack_q.backward_acts(qa, flat_q, dq, s, ctx.needs_input_grad[0],
                                             on_dx=(lambda dx: on_dx(0, dx)) if on_dx is not None else None)
        if ctx.on_tower is not None:
            ctx.on_tower(0, gqi, gflat_q)
        main.wait_stream(side)
        return gqi, gci, gflat_q, gflat_c, None, None, None, None, None, None


def global_inbatch_grads(q: torch.Tensor, c: torch.Tensor, logq: Optional[torch.Tensor], comm,
                         rows=None, cols=None):
    """This rank's share of the in-batch loss over the GLOBAL batch
    (two_tower_model.py:113-122 with the batch split over the ranks: row i's
    negatives are every candidate of every rank).  q, c: this rank's [b, E]
    rows (global rows rank*b ...); comm: all_gather over the ranks (equal b
    everywhere).  Returns (row_loss [b], dq [b, E], dc [b, E]): the loss
    terms of this rank's rows, d loss / d q of its rows, and d (global loss)
    / d c of its candidates.  The rows pass scores the local queries against
    all candidates; the cols pass scores all queries (with their lse) against
    the local candidates, so every gradient is summed inside one kernel in a
    fixed order (no cross-rank reduction of partial sums)."""
    if WORLD1_FUSED and comm.world == 1 and rows is None and cols is None and not getattr(comm, "always", False):
        # one rank: its rows are every row and its columns every column — the
        # single-device entry (one shared preparation of q and c for both passes)
        _, row_loss, dq, dc = hip_ops.inbatch_fused(q, c, logq)
        return row_loss, dq, dc
    rows = rows or hip_ops.inbatch_rows
    cols = cols or hip_ops.inbatch_cols
    b = q.shape[0]
    off = comm.rank * b
    C = comm.all_gather(c)                                     # [G b, E]
    L = comm.all_gather(logq) if logq is not None else None   # [G b]
    lse, row_loss, dq = rows(q, C, L, pos_offset=off)
    Qa = comm.all_gather(q)                                    # [G b, E]
    if comm.world == 1 and not getattr(comm, "always", False):
        lse_a, loss_a = lse, row_loss  # one rank: its rows are every row (no stack / split copies)
    else:
        st = comm.all_gather(torch.stack([lse, row_loss], 1))  # [G b, 2]: every row's lse and loss
        lse_a, loss_a = st[:, 0].contiguous(), st[:, 1].contiguous()
    dc = cols(Qa, lse_a, c, logq, pos_offset=off, row_loss=loss_a)  # local columns, every row
    return row_loss, dq, dc


class _GlobalTowersInBatchXent(torch.autograd.Function):
    """_TowersInBatchXent with global in-batch negatives (global_inbatch_grads):
    the returned loss is this rank's rows' share; the step sums it (and the
    gradients) over the ranks."""

    @staticmethod
    def forward(ctx, qi, ci, flat_q, flat_c, logq, stack_q, stack_c, scale, comm):
        ctx.pair = _paired(qi, stack_q, stack_c)
        if ctx.pair:
            qa, ca = _pair_forward(qi, ci, flat_q, flat_c, stack_q, stack_c)
        else:
            # the two towers' MLPs on two streams, as in _TowersInBatchXent
            with _TowerFork(qi):
                ca = stack_c.forward_acts(ci, flat_c)
            qa = stack_q.forward_acts(qi, flat_q)
            _tower_join(qi)
        row_loss, dq, dc = global_inbatch_grads(qa[-1], ca[-1], logq, comm)
        ctx.stacks = (stack_q, stack_c)
        ctx.nq = len(qa)
        ctx.scale = scale
        ctx.save_for_backward(flat_q, flat_c, dq, dc, *qa, *ca)
        return hip_ops.loss_sum(row_loss, scale)

    @staticmethod
    def backward(ctx, g):
        flat_q, flat_c, dq, dc, *acts = ctx.saved_tensors
        qa, ca = acts[:ctx.nq], acts[ctx.nq:]
        s = (g * ctx.scale if ctx.scale != 1.0 else g).reshape(1).float().contiguous()
        stack_q, stack_c = ctx.stacks
        if ctx.pair:
            return (*_pair_backward(ctx, qa, ca, flat_q, flat_c, dq, dc, s), None, None, None, None, None)
        with _TowerFork(dq):
            gci, gflat_c = stack_c.backward_acts(ca, flat_c, dc, s, ctx.needs_input_grad[1])
        gqi, gflat_q = stack_q.backward_acts(qa, flat_q, dq, s, ctx.needs_input_grad[0])
        _tower_join(dq)
        return gqi, gci, gflat_q, gflat_c, None, None, None, None, None


def global_towers_inbatch_softmax_xent(qi: torch.Tensor, ci: torch.Tensor, stack_q, stack_c, comm,
                                       logq: Optional[torch.Tensor] = None) -> torch.Tensor:
    """towers_inbatch_softmax_xent with the negatives of every rank (SUM
    reduction, the reference's runner.py:78-83)."""
    return _GlobalTowersInBatchXent.apply(qi, ci, stack_q.flat, stack_c.flat, logq, stack_q, stack_c, 1.0, comm)


def towers_inbatch_softmax_xent(qi: torch.Tensor, ci: torch.Tensor, stack_q, stack_c,
                                logq: Optional[torch.Tensor] = None, reduction: str = "sum",
                                on_tower=None, on_dx=None) -> torch.Tensor:
    """Loss of the query tower on qi against the candidate tower on ci (tower
    inputs [B, *]), fused into one autograd node; stack_* are DenseStacks.
    on_tower(i, input_grad, flat_grad), if given, is called in the backward as
    soon as tower i's (0 query, 1 candidate) gradients exist, on the stream and
    workspace scope they were produced in (the fused train step applies the
    optimizer there)."""
    if reduction not in ("sum", "sum_over_batch_size", "mean"):
        raise ValueError(f"unsupported reduction {reduction}")
    scale = 1.0 if reduction == "sum" else 1.0 / qi.shape[0]
    return _TowersInBatchXent.apply(qi, ci, stack_q.flat, stack_c.flat, logq, stack_q, stack_c, scale, on_tower,
                                    on_dx)


def inbatch_softmax_xent(q: torch.Tensor, c: torch.Tensor, logq: Optional[torch.Tensor] = None,
                         reduction: str = "sum") -> torch.Tensor:
    """Loss of query rows q [B,E] against candidates c [B,E] (positive of row
    i is column i), logq [B] the per-candidate log sampling probability."""
    if reduction not in ("sum", "sum_over_batch_size", "mean"):
        raise ValueError(f"unsupported reduction {reduction}")
    scale = 1.0 if reduction == "sum" else 1.0 / q.shape[0]
    if not q.requires_grad and not c.requires_grad:
        lse, row_loss, _ = hip_ops.inbatch_rows(q, c, logq, want_dq=False)
        return hip_ops.loss_sum(row_loss, scale)
    return _InBatchXent.apply(q, c, logq, scale)


class InBatchSoftmaxCrossEntropy:
    """Stand-in for tf.keras.losses.CategoricalCrossentropy(from_logits=True,
    reduction=SUM) as compiled by the reference runner (runner.py:78-83)."""

    def __init__(self, from_logits: bool = True, reduction: str = "sum"):
        if not from_logits:
            raise ValueError("the in-batch loss is defined on logits (from_logits=True)")
        self.reduction = str(reduction).lower().split(".")[-1]

    def __call__(self, q, c, logq=None):
        return inbatch_softmax_xent(q, c, logq, self.reduction)


# Name the reference compiles with.
CategoricalCrossentropy = InBatchSoftmaxCrossEntropy
