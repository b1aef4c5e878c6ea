"""Multi-GPU paths: one process per GPU, torch.distributed over RCCL/xGMI.

SURVEY §8e.  Two pieces the reference's call sites shard naturally:

* ShardedBruteForceIndex — BruteForceIndex with the candidate matrix
  row-sharded over the ranks.  Each rank scores the (replicated) queries
  against its shard with tt_bruteforce_search, indices offset by the shard's
  first global row; the per-shard sorted top-k lists are all-gathered and
  merged with tt_topk_merge (score desc, global index asc), which equals
  tf.math.top_k over the unsharded scores (brute_force.py:76-81).

* DataParallelTrainStep — the reference's train_step
  (two_tower_model.py:94-130) replicated per GPU the way a data-parallel
  Keras run executes it: each replica computes its in-batch loss over its
  own batch (per-replica negatives), dense gradients are summed with one
  all_reduce bucket, and the sparse embedding gradients (the IndexedSlices
  rows + ids) are all-gathered in rank order so every replica applies the
  same global dedup + Adagrad update — replicas stay identical.

Collective and kernel entry points are injectable (`ops=`), so the
orchestration is exercised on CPU with the gloo backend by the tests; the
defaults are the libtt kernels and the product never falls back to them.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Callable, Dict, Iterable, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

__all__ = ["IndexOps", "ShardedBruteForceIndex", "DataParallelTrainStep", "shard_range", "all_gather_cat",
           "EmbeddingOps", "ShardedTables", "ShardedTrainStep"]


def all_gather_cat(t: torch.Tensor, group=None) -> torch.Tensor:
    """Rank-ordered concatenation along a new leading dim [world, *t.shape]
    (all_gather_into_tensor on RCCL; list all_gather elsewhere, e.g. gloo)."""
    world = dist.get_world_size(group)
    t = t.contiguous()
    out = torch.empty((world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, t, group=group)
    else:
        dist.all_gather(list(out.unbind(0)), t, group=group)
    return out


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block [begin, end) of n rows owned by `rank` (sizes differ by <= 1)."""
    base, rem = divmod(n, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


@dataclass
class IndexOps:
    build: Callable[[torch.Tensor], Any]
    search: Callable[..., Tuple[torch.Tensor, torch.Tensor]]
    merge: Callable[[torch.Tensor, torch.Tensor, int], Tuple[torch.Tensor, torch.Tensor]]

    @staticmethod
    def hip() -> "IndexOps":
        from pkg.modelling import hip_ops

        return IndexOps(hip_ops.bruteforce_build,
                        lambda img, cand, q, k, off: hip_ops.bruteforce_search(img, cand, q, k, off),
                        hip_ops.topk_merge)


class ShardedBruteForceIndex:
    """
    Candidate-sharded brute-force index.

    Parameters
    ----------
    k: int
        Results per query.
    query_model: callable
        Query feature dict -> [B, E] embeddings (replicated on every rank).
    local_candidates: [n_local, E] tensor
        This rank's shard of the candidate matrix (rows shard_range(N, world, rank)).
    index_offset: int
        Global row of the shard's first candidate.
    local_identifiers: optional identifiers of the local rows.
    """

    def __init__(self, k: int, query_model, local_candidates: torch.Tensor, index_offset: int,
                 local_identifiers=None, group=None, ops: Optional[IndexOps] = None):
        self.k = int(k)
        self.query_model = query_model
        self.group = group
        self.ops = ops or IndexOps.hip()
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.cand = local_candidates.contiguous()
        self.offset = int(index_offset)
        n_local = torch.tensor([self.cand.shape[0]], dtype=torch.int64, device=self.cand.device)
        sizes = [torch.zeros_like(n_local) for _ in range(self.world)]
        dist.all_gather(sizes, n_local, group=group)
        self.shard_sizes = [int(s.item()) for s in sizes]
        if min(self.shard_sizes) < self.k:
            raise ValueError(f"every shard needs >= k={self.k} candidates, got {self.shard_sizes}")
        self.num_candidates = sum(self.shard_sizes)
        self.image = self.ops.build(self.cand)
        self.local_identifiers = local_identifiers

    def search(self, query_embeddings: torch.Tensor, k: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Global (scores [Q,k], indices [Q,k]) on every rank."""
        k = k or self.k
        s, i = self.ops.search(self.image, self.cand, query_embeddings.contiguous(), k, self.offset)
        all_s = all_gather_cat(s, self.group)
        all_i = all_gather_cat(i, self.group)
        return self.ops.merge(all_s, all_i, k)

    def __call__(self, queries: Dict[str, Any]):
        with torch.no_grad():
            emb = self.query_model(queries)
        return self.search(emb)[1]


class DataParallelTrainStep:
    """One train step per call on every rank (see module docstring).

    `model` is a compiled TwoTowerModel created with the same seed on every
    rank.  The batch passed on each rank is that replica's share of the
    global batch; all replicas must use the same per-replica batch size.
    """

    def __init__(self, model, example_batch: Optional[Dict[str, Any]] = None, group=None):
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group)

    # -- collectives ---------------------------------------------------------
    def allreduce_dense(self) -> None:
        towers = self.model.towers
        grads = [t.dense.flat.grad for t in towers]
        bucket = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(bucket, group=self.group)
        off = 0
        for g in grads:
            g.copy_(bucket[off:off + g.numel()].view_as(g))
            off += g.numel()

    def gather_sparse(self, layer) -> None:
        """Replace the layer's sparse batch (ids per lookup, output grad) by the
        rank-ordered concatenation over all replicas."""
        calls = layer._last_calls
        if not calls or layer.last_grad is None:
            return
        B = layer.last_grad.shape[0]
        ids = torch.stack([c[1] for c in calls], 1).contiguous()  # [B, n_lookups]
        all_ids = all_gather_cat(ids, self.group).reshape(self.world * B, ids.shape[1])
        g = layer.last_grad.contiguous()
        all_g = all_gather_cat(g, self.group).reshape(self.world * B, g.shape[1])
        layer._last_calls = [(name, all_ids[:, j].contiguous(), off) for j, (name, _, off) in enumerate(calls)]
        layer.last_grad = all_g

    def __call__(self, batch: Dict[str, Any]) -> Dict[str, torch.Tensor]:
        m = self.model
        loss = m.compute_loss(batch, training=True)
        for t in m.towers:
            t.dense.flat.grad = None
        loss.backward()
        self.allreduce_dense()
        for t in m.towers:
            self.gather_sparse(t.input_layer)
        m.optimizer.apply_gradients(m.towers)
        total = loss.detach().clone()
        dist.all_reduce(total, group=self.group)
        return {"loss": total}


# --------------------------------------------------------------------------- row-sharded tables
@dataclass
class EmbeddingOps:
    """Kernels of the row-sharded path (defaults: libtt; tests inject CPU ones)."""
    gather_multi: Callable[..., None]
    gather_tagged: Callable[..., torch.Tensor]
    scatter_sum: Callable[..., None]
    sparse_adagrad: Callable[..., None]
    dense_adagrad: Callable[..., None]

    @staticmethod
    def hip() -> "EmbeddingOps":
        from pkg.modelling import hip_ops

        return EmbeddingOps(hip_ops.gather_multi, hip_ops.gather_tagged, hip_ops.sparse_scatter_sum,
                            hip_ops.sparse_adagrad, hip_ops.dense_adagrad)


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits: List[int], in_splits: List[int], group) -> torch.Tensor:
    dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)
    return out


class ShardedTables:
    """
    Embedding tables row-sharded over the ranks: global row r
    lives on rank r % world at local row r // world, so every rank owns ~1/world
    of each table and of its Adagrad accumulator.

    One exchange per step for all sharded tables:
      forward   requests: each rank dedups its lookups per table, buckets the
                distinct (table, row) pairs by owner and sends them with one
                all_to_all; owners answer with one tt_gather_tagged launch and
                one all_to_all of rows back.
      backward  each rank sums its lookup gradients per request
                (tt_sparse_scatter_sum, same order as the single-GPU dedup),
                one all_to_all sends them to the owners, and each owner applies
                tt_sparse_adagrad to its shard (duplicate rows from different
                ranks summed in rank order).
    All sharded tables share one embedding width (rows move as [n, dim]).
    """

    def __init__(self, tables: Dict[str, torch.Tensor], init_accumulator: float = 0.1, group=None,
                 ops: Optional[EmbeddingOps] = None, full_tables: bool = True):
        """tables: name -> full [rows, dim] table (full_tables=True, the shard is
        sliced out) or this rank's shard with a "__rows__" entry giving the
        global row counts (full_tables=False, for tables too big to build)."""
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.ops = ops or EmbeddingOps.hip()
        self.names = [n for n in tables if n != "__rows__"]
        dims = {tables[n].shape[1] for n in self.names}
        if len(dims) != 1:
            raise ValueError(f"sharded tables must share one embedding width, got {sorted(dims)}")
        self.dim = dims.pop()
        self.shard: Dict[str, torch.Tensor] = {}
        self.acc: Dict[str, torch.Tensor] = {}
        self.rows: Dict[str, int] = {}
        for n in self.names:
            t = tables[n]
            if full_tables:
                self.rows[n] = t.shape[0]
                self.shard[n] = t[self.rank::self.world].contiguous().clone()
            else:
                self.rows[n] = int(tables["__rows__"][n])
                self.shard[n] = t.contiguous()
            self.acc[n] = torch.full_like(self.shard[n], init_accumulator)
        self._ctx = None

    def local_rows(self, name: str) -> int:
        return self.shard[name].shape[0]

    # -- forward -----------------------------------------------------------
    def fetch(self, lookups: List[Tuple[str, torch.Tensor]]) -> Tuple[torch.Tensor, List[torch.Tensor]]:
        """lookups: (table name, ids [B] int32) -> (rows [R, dim], row index per
        lookup [B] int32): lookup l's embedding of batch row b is rows[idx_l[b]]."""
        W = self.world
        dev = lookups[0][1].device
        by_table: Dict[str, List[int]] = {}
        for i, (name, _) in enumerate(lookups):
            by_table.setdefault(name, []).append(i)
        req_ids, req_tags, inverse, starts = [], [], {}, {}
        off = 0
        for ti, name in enumerate(self.names):
            if name not in by_table:
                continue
            ids = torch.cat([lookups[i][1].reshape(-1) for i in by_table[name]])
            ids = torch.where((ids >= 0) & (ids < self.rows[name]), ids, torch.full_like(ids, -1))
            uniq, inv = torch.unique(ids, sorted=True, return_inverse=True)
            req_ids.append(uniq.to(torch.int32))
            req_tags.append(torch.full_like(uniq, ti, dtype=torch.int32))
            inverse[name] = inv
            starts[name] = off
            off += uniq.numel()
        req_ids = torch.cat(req_ids)
        req_tags = torch.cat(req_tags)
        R = req_ids.numel()
        owner = torch.remainder(req_ids, W)  # invalid (-1) ids go to rank W-1 and answer zeros
        owner_sorted, perm = torch.sort(owner.to(torch.int64), stable=True)
        send = torch.stack([req_ids[perm], req_tags[perm]], 1).contiguous()
        send_counts = torch.bincount(owner_sorted, minlength=W).to(torch.int64)
        recv_counts = torch.empty_like(send_counts)
        _a2a(recv_counts, send_counts, [1] * W, [1] * W, self.group)
        counts = torch.stack([send_counts, recv_counts]).cpu()  # the one host sync of the step
        s_split, r_split = counts[0].tolist(), counts[1].tolist()
        recv = torch.empty(sum(r_split), 2, dtype=torch.int32, device=dev)
        _a2a(recv, send, r_split, s_split, self.group)
        # owner: answer every request with one launch
        tags = recv[:, 1].contiguous()
        gid = recv[:, 0]
        rows = torch.where(gid >= 0, torch.div(gid, W, rounding_mode="floor"), torch.full_like(gid, -1))
        rows = rows.to(torch.int32).contiguous()
        reply = torch.empty(tags.numel(), self.dim, dtype=torch.float32, device=dev)
        self.ops.gather_tagged([self.shard[n] for n in self.names], tags, rows, reply)
        got = torch.empty(R, self.dim, dtype=torch.float32, device=dev)
        _a2a(got, reply, s_split, r_split, self.group)
        # position of request (table, unique u) in `got`
        inv_perm = torch.empty_like(perm)
        inv_perm[perm] = torch.arange(R, device=dev)
        idx = []
        pos_in_table: Dict[str, int] = {}
        for name, ids in lookups:
            k = pos_in_table.get(name, 0)
            n = ids.numel()
            u = inverse[name][k:k + n]
            pos_in_table[name] = k + n
            idx.append(inv_perm[starts[name] + u].to(torch.int32).contiguous())
        self._ctx = dict(s_split=s_split, r_split=r_split, tags=tags, rows=rows, R=R, dev=dev)
        return got, idx

    # -- backward + update -------------------------------------------------
    def apply(self, grads: List[Tuple[torch.Tensor, List[Tuple[torch.Tensor, int]]]], lr: float, eps: float) -> None:
        """grads: per gradient matrix [B, width] its (row index from fetch, column)
        sources.  Sums per request, returns the sums to the owners, and applies
        Adagrad to the local shards."""
        c = self._ctx
        g_req = torch.zeros(c["R"], self.dim, dtype=torch.float32, device=c["dev"])
        for gmat, sources in grads:
            if not sources:
                continue
            spec = [dict(table=g_req, ids=[s[0] for s in sources], grad_col_offset=[s[1] for s in sources])]
            self.ops.scatter_sum(spec, gmat.shape[0], gmat)
        recv = torch.empty(len(c["tags"]), self.dim, dtype=torch.float32, device=c["dev"])
        _a2a(recv, g_req, c["r_split"], c["s_split"], self.group)
        specs = []
        for ti, name in enumerate(self.names):
            ids = torch.where(c["tags"] == ti, c["rows"], torch.full_like(c["rows"], -1)).contiguous()
            specs.append(dict(table=self.shard[name], slot0=self.acc[name], ids=[ids], grad_col_offset=[0]))
        if recv.shape[0] > 0:
            self.ops.sparse_adagrad(specs, recv.shape[0], recv, lr, eps)
        self._ctx = None

    def gather_full(self, name: str) -> torch.Tensor:
        """The full table reassembled on every rank (checks / export)."""
        rows, W = self.rows[name], self.world
        per = (rows + W - 1) // W
        mine = torch.zeros(per, self.dim, dtype=torch.float32, device=self.shard[name].device)
        mine[:self.shard[name].shape[0]] = self.shard[name]
        parts = all_gather_cat(mine, self.group)
        full = torch.empty(rows, self.dim, dtype=torch.float32, device=mine.device)
        for r in range(W):
            n = len(range(r, rows, W))
            full[r::W] = parts[r, :n]
        return full


class _ShardedGatherFn(torch.autograd.Function):
    """Both towers' input rows from local (replicated) tables and the fetched
    rows of sharded tables, one gather launch; backward keeps the output
    gradients for the explicit sparse step."""

    @staticmethod
    def forward(ctx, step, calls, batch, widths, *anchors):
        step.ops.gather_multi(calls, batch)
        ctx.step = step
        return tuple(out[:, :w] for (_, out), w in zip(calls, widths))

    @staticmethod
    def backward(ctx, *grads):
        ctx.step._out_grads = [g if g is None or g.stride(1) == 1 else g.contiguous() for g in grads]
        return (None, None, None, None) + (None,) * len(grads)


class ShardedTrainStep:
    """
    Data-parallel train step with the large embedding tables row-sharded
    (ShardedTables) and the small ones replicated.  Per-replica in-batch
    negatives, as DataParallelTrainStep.  Per step: the sharded-table exchange
    (3 all_to_all + one tiny count exchange), one all_reduce bucket holding the
    MLP gradients, the dense gradients of the small tables and the loss.
    Sparse work per rank stays ~constant as ranks are added (each owner updates
    only its rows), unlike gathering every replica's sparse gradients.

    Adagrad (the reference's optimizer, main.py:100-101) only.
    """

    def __init__(self, model, shard_min_rows: int = 100_000, group=None, ops: Optional[EmbeddingOps] = None):
        from pkg.modelling.optimizer_factory import Adagrad

        opt = model.optimizer
        if not isinstance(opt, Adagrad):
            raise NotImplementedError("ShardedTrainStep supports the Adagrad optimizer")
        self.model = model
        self.group = group
        self.ops = ops or EmbeddingOps.hip()
        self.world = dist.get_world_size(group)
        self.lr, self.eps, self.init = opt.learning_rate, opt.epsilon, opt.initial_accumulator_value
        big: Dict[str, torch.Tensor] = {}
        self.small: Dict[str, Any] = {}
        for tower in model.towers:
            for name, t in tower.input_layer.embedding_layers.items():
                key = (id(tower), name)
                if t.num_rows >= shard_min_rows:
                    big[f"{len(big)}:{name}"] = t.weight
                    t._shard_key = f"{len(big) - 1}:{name}"
                else:
                    self.small[key] = t
        self.tables = ShardedTables(big, self.init, group, self.ops) if big else None
        for tower in model.towers:  # drop the full copies of sharded tables
            for t in tower.input_layer.embedding_layers.values():
                if hasattr(t, "_shard_key"):
                    t.weight = None
        self._small_acc = {k: torch.full_like(t.weight, self.init) for k, t in self.small.items()}
        self._dense_acc = [torch.full_like(t.dense.flat, self.init) for t in model.towers]
        self._out_grads = None

    def __call__(self, batch: Dict[str, Any]) -> Dict[str, torch.Tensor]:
        m = self.model
        q, c = m._split(batch)
        layers = [t.input_layer for t in m.towers]
        xs = [q, c]
        B = None
        calls, widths, sharded_srcs = [], [], []
        lookups = []
        for li, (layer, x) in enumerate(zip(layers, xs)):
            for f, off in zip(layer.categorical_features, layer.column_offsets()):
                t = layer.embedding_layers[f.name]
                if hasattr(t, "_shard_key"):
                    lookups.append((t._shard_key, layer._ids(x[f.name]), li, off))
        got, idx = (self.tables.fetch([(k, ids) for k, ids, _, _ in lookups]) if lookups else (None, []))
        small_srcs = []
        for li, (layer, x) in enumerate(zip(layers, xs)):
            segs, srcs_big, srcs_small = [], [], []
            for f in layer.numerical_features:
                v = x[f.name]
                v = (v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v, np.float32)))
                v = v.reshape(-1).to(device=layer.device, dtype=torch.float32).contiguous()
                segs.append((v, None, len(segs)))
            for f, off in zip(layer.categorical_features, layer.column_offsets()):
                t = layer.embedding_layers[f.name]
                if hasattr(t, "_shard_key"):
                    j = next(i for i, lk in enumerate(lookups) if lk[2] == li and lk[3] == off)
                    segs.append((got, idx[j], off))
                    srcs_big.append((idx[j], off))
                else:
                    ids = layer._ids(x[f.name])
                    segs.append((t.weight, ids, off))
                    srcs_small.append((f.name, ids, off))
            B = segs[0][1].numel() if segs[0][1] is not None else segs[0][0].numel()
            out = torch.empty(B, layer.row_stride, dtype=torch.float32, device=layer.device)
            calls.append((segs, out))
            widths.append(layer.output_dim)
            sharded_srcs.append(srcs_big)
            small_srcs.append(srcs_small)
        anchors = [layer._anchor for layer in layers]
        qi, ci = _ShardedGatherFn.apply(self, calls, B, widths, *anchors)
        loss = m.tower_loss(qi, ci, m.candidate_logq(batch))
        for t in m.towers:
            t.dense.flat.grad = None
        loss.backward()
        grads = self._out_grads
        # sharded tables: per-request sums -> owners -> Adagrad on the shards
        if self.tables is not None:
            self.tables.apply([(g, srcs) for g, srcs in zip(grads, sharded_srcs)], self.lr, self.eps)
        # one all_reduce bucket: MLP grads, small-table dense grads, loss
        parts = [t.dense.flat.grad.reshape(-1) for t in m.towers]
        small_grads = []
        for li, (layer, srcs) in enumerate(zip(layers, small_srcs)):
            by_name: Dict[str, List[Tuple[torch.Tensor, int]]] = {}
            for name, ids, off in srcs:
                by_name.setdefault(name, []).append((ids, off))
            specs = []
            for name, s in by_name.items():
                t = layer.embedding_layers[name]
                gdense = torch.zeros_like(t.weight)
                small_grads.append(((id(m.towers[li]), name), t, gdense))
                specs.append(dict(table=gdense, ids=[x[0] for x in s], grad_col_offset=[x[1] for x in s]))
            if specs:
                self.ops.scatter_sum(specs, grads[li].shape[0], grads[li])
        parts += [g.reshape(-1) for _, _, g in small_grads]
        parts.append(loss.detach().reshape(1))
        bucket = torch.cat(parts)
        dist.all_reduce(bucket, group=self.group)
        off = 0
        for ti, t in enumerate(m.towers):
            n = t.dense.flat.numel()
            self.ops.dense_adagrad(t.dense.flat.data, self._dense_acc[ti], bucket[off:off + n].view_as(t.dense.flat),
                                   self.lr, self.eps)
            off += n
        for key, t, g in small_grads:
            n = g.numel()
            self.ops.dense_adagrad(t.weight, self._small_acc[key], bucket[off:off + n].view_as(g), self.lr, self.eps)
            off += n
        return {"loss": bucket[off:off + 1].reshape(())}
