"""Multi-GPU paths: one process per GPU, torch.distributed over RCCL/xGMI.

SURVEY §8e.  Three pieces the reference's call sites shard naturally:

* ShardedBruteForceIndex — BruteForceIndex with the candidate matrix
  row-sharded over the ranks: each rank holds only its block of rows and
  computes the exact top-k of its shard (tt_bruteforce_search, indices offset
  by the block's first global row); the per-shard lists of each query block
  go to its owner (all_to_all) and are merged with tt_topk_merge (score desc,
  global index asc), which equals tf.math.top_k over the unsharded scores
  (brute_force.py:76-81).

* ShardedTables / ShardedTrainStep — the reference's train_step
  (two_tower_model.py:94-130) over G ranks: each large embedding table
  (Embedding, input_layer.py:37-40) row-sharded (global row r at rank r mod G),
  lookups routed to their owners with all_to_all (tt_route_requests,
  tt_gather_tagged), the gradient rows returned the same way and applied by
  the owner (tt_sparse_scatter_sum, tt_sparse_adagrad); the batch split over
  the ranks with global in-batch negatives (C and logq all-gathered for the
  rows pass, Q and lse for the cols pass, gradients reduce_scattered), small
  tables and the tower MLPs replicated and all_reduced in one bucket.

* QueryShardedBruteForceIndex — replicated candidates, each rank answers its
  block of the queries (no exchange); bench.py's query-parallel leg.

Collective and kernel entry points are injectable (`ops=`), so the
orchestration is exercised on CPU with the gloo backend by the tests; the
defaults are the libtt kernels and the product never falls back to them.
"""
from __future__ import annotations

import logging
import os
import time
import weakref
from dataclasses import dataclass
from typing import Any, Callable, Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

# world-1 sharded step: the route on a side stream beside the forward (1) or
# on the compute stream ahead of it (0): 0.311 vs 0.320 ms at 2048 rows,
# 0.584-0.586 vs 0.636-0.647 ms at 16384 (profiles/r05_step_ab.txt)
ROUTE_SIDE = os.environ.get("TT_SHARDED_ROUTE_SIDE", "1") == "1"
logger = logging.getLogger(__name__)

__all__ = ["IndexOps", "BatchComm", "ShardedBruteForceIndex", "QueryShardedBruteForceIndex", "shard_range", "all_gather_cat",
           "EmbeddingOps", "ShardedTables", "ShardedTrainStep", "destroy_process_group"]

# every ShardedTrainStep alive: its captured graph may hold RCCL collectives
# and must be destroyed while their communicator still exists
_LIVE_STEPS: "weakref.WeakSet" = weakref.WeakSet()


def destroy_process_group(group=None) -> None:
    """torch.distributed.destroy_process_group, after releasing the captured
    graphs of every live ShardedTrainStep (ShardedTrainStep.close).  A hipGraph
    holding RCCL collectives that is destroyed after its communicator corrupted
    the host heap: a later, unrelated graph replay segfaulted inside
    hipGraphLaunch on a freed vector of the runtime."""
    for step in list(_LIVE_STEPS):
        step.close()
    dist.destroy_process_group(group)


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
    """Kernels of the sharded indices (tt.h: tt_bruteforce_build,
    tt_bruteforce_search with a global index offset, tt_topk_merge).
    Injectable so the orchestration below runs on CPU over gloo in the tests
    (oracle.bruteforce_topk / topk_merge); the defaults are libtt."""
    build: Callable[[torch.Tensor], Any]
    search: Callable[..., Tuple[torch.Tensor, torch.Tensor]]
    merge: Callable[[torch.Tensor, torch.Tensor, int], Tuple[torch.Tensor, torch.Tensor]]
    # (image, rows, queries, k, offset, reduce_max, chunk) -> this shard's exact
    # top-k of the rows that can reach the global k-th score (padded), one
    # reduce_max per chunk of queries; None: search
    shard_search: Optional[Callable[..., Tuple[torch.Tensor, torch.Tensor]]] = None
    # (n_queries, shard sizes of ALL ranks, dim, k) -> the common query chunk
    shard_chunk: Optional[Callable[[int, Sequence[int], int, int], int]] = None

    @staticmethod
    def hip() -> "IndexOps":
        from pkg.modelling import hip_ops

        return IndexOps(hip_ops.bruteforce_build,
                        lambda img, cand, q, k, off: hip_ops.bruteforce_search(img, cand, q, k, off),
                        hip_ops.topk_merge, hip_ops.bruteforce_shard_search, hip_ops.bruteforce_shard_chunk)


def _staged(group) -> bool:
    """gloo moves host tensors only: device tensors go through the host."""
    return dist.get_backend(group) == "gloo"


def _all_reduce_max(t: torch.Tensor, group) -> None:
    if _staged(group) and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.MAX, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)


def _all_gather_any(t: torch.Tensor, group) -> torch.Tensor:
    if _staged(group) and t.is_cuda:
        return all_gather_cat(t.cpu(), group).to(t.device)
    return all_gather_cat(t, group)


def _gather_query_blocks(s: torch.Tensor, i: torch.Tensor, Q: int, world: int, group) -> Tuple[torch.Tensor, torch.Tensor]:
    """Rank-ordered concatenation of the per-rank query blocks
    shard_range(Q, world, r) of (scores, indices) [block, k] -> [Q, k]."""
    k = s.shape[1]
    per = -(-Q // world)
    pad_s = torch.full((per, k), float("-inf"), dtype=s.dtype, device=s.device)
    pad_i = torch.full((per, k), -1, dtype=i.dtype, device=i.device)
    pad_s[:s.shape[0]] = s
    pad_i[:i.shape[0]] = i
    all_s, all_i = _all_gather_any(pad_s, group), _all_gather_any(pad_i, group)
    blocks = [shard_range(Q, world, r) for r in range(world)]
    return (torch.cat([all_s[r, :e - b] for r, (b, e) in enumerate(blocks)]),
            torch.cat([all_i[r, :e - b] for r, (b, e) in enumerate(blocks)]))


# index of a padding entry of a shard with fewer than k rows: sorts after
# every real entry, -inf scores included (tt_topk_merge's (score, -index) key)
PAD_INDEX = 0x7FFFFFFF


class ShardedBruteForceIndex:
    """
    Candidate-sharded brute-force index (north star: "shards the
    candidate matrix across the 8 GPUs ... merges per-shard top-K").
    BruteForceIndex.call (brute_force.py:75-83: matmul -> top_k -> gather)
    with the candidate matrix row-sharded: rank g holds ONLY its contiguous
    block C[b_g:e_g] (fp32 rows + their bf16 screening image), the blocks in
    rank order.

    Per search (queries replicated on every rank):
      1. per chunk of queries, tt_bruteforce_shard_screen on the local rows:
         a lower bound on each query's k-th exact score among them; one
         all_reduce(MAX) makes it a bound on the GLOBAL k-th score (floor);
         tt_bruteforce_shard_finalize rescores only the entries that can reach
         the floor: the exact top-k of the shard among them, indices global
         (index_offset = b_g, ties -> lower index), padded past the survivors
         (so each shard rescores ~1/G of the rows the global top-k needs);
      2. all_to_all: the lists of query block r (shard_range(Q, G, r)) go to
         rank r — Q·k·8 B sent per rank, 1/G of it kept;
      3. tt_topk_merge of the G lists -> the owner's exact global top-k.
    Exact: a candidate of the global top-k outranks every other candidate of
    its own shard that it beats globally, so it is in its shard's top-k, and
    it scores >= the global k-th score >= floor, so it survives the cut; the
    merge orders by the same (score desc, index asc) key top_k uses, and the
    scores are the same fp32 chains wherever a row lives.  search() then
    all-gathers the owners' blocks so every rank holds the whole answer.

    Parameters
    ----------
    k: int
        Results per query.
    query_model: callable
        Query feature dict -> [B, E] embeddings (replicated on every rank).
    candidates: [n_g, E] tensor
        THIS rank's rows; the global matrix is the rank-ordered concatenation
        (ShardedBruteForceIndex.from_full slices it from a full matrix).
    identifiers: optional identifiers of all N rows (small; replicated).
    """

    def __init__(self, k: int, query_model, candidates: torch.Tensor, identifiers=None, group=None,
                 ops: Optional[IndexOps] = None):
        self.k = int(k)
        self.query_model = query_model
        self.group = group
        self.ops = ops or IndexOps.hip()
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.shard = candidates.contiguous()
        n = int(self.shard.shape[0])
        sizes = _all_gather_any(torch.tensor([n], dtype=torch.int64, device=self.shard.device), group)
        self.sizes = [int(x) for x in sizes.reshape(-1).cpu().tolist()]
        self.offset = sum(self.sizes[:self.rank])
        self.num_candidates = sum(self.sizes)
        self.rows = (self.offset, self.offset + n)
        if min(self.sizes) < 1:
            raise ValueError(f"every rank needs >= 1 candidate row, got shard sizes {self.sizes}")
        if self.num_candidates < self.k:
            raise ValueError(f"need >= k={self.k} candidates, got {self.num_candidates}")
        if self.num_candidates >= 2 ** 31 - 64:
            raise ValueError("global candidate indices must fit int32")
        self.image = self.ops.build(self.shard)
        self.identifiers = identifiers

    @classmethod
    def from_full(cls, k: int, query_model, candidates: torch.Tensor, identifiers=None, group=None,
                  ops: Optional[IndexOps] = None) -> "ShardedBruteForceIndex":
        """This rank's block shard_range(N, G, rank) copied out of a full
        matrix (which the caller may then free)."""
        b, e = shard_range(int(candidates.shape[0]), dist.get_world_size(group), dist.get_rank(group))
        return cls(k, query_model, candidates[b:e].clone(), identifiers, group, ops)

    def search_shard(self, query_embeddings: torch.Tensor, k: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """This shard's exact top-k of every query, global indices, padded
        with (-inf, PAD_INDEX) past its row count: ([Q, k], [Q, k] int32)."""
        k = k or self.k
        if k > self.num_candidates:
            raise ValueError(f"k={k} exceeds the number of candidates {self.num_candidates}")
        q = query_embeddings.contiguous()
        kl = min(k, int(self.shard.shape[0]))
        # collective decision: every rank takes the same branch (its all_reduce)
        if self.world > 1 and self.ops.shard_search is not None and min(self.sizes) >= k:
            # two-phase: the shards' lower bounds on their k-th scores, max-reduced,
            # cut each shard's exact rescoring to what can reach the global top-k.
            # The query chunk is computed from ALL shard sizes, so every rank makes
            # the same all_reduce calls (same count, same lengths).
            chunk = self.ops.shard_chunk(int(q.shape[0]), self.sizes, int(q.shape[1]), k)
            return self.ops.shard_search(self.image, self.shard, q, k, self.offset,
                                         lambda t: _all_reduce_max(t, self.group), chunk)
        s, i = self.ops.search(self.image, self.shard, q, kl, self.offset)
        if kl < k:
            ps = torch.full((q.shape[0], k), float("-inf"), dtype=s.dtype, device=s.device)
            pi = torch.full((q.shape[0], k), PAD_INDEX, dtype=i.dtype, device=i.device)
            ps[:, :kl], pi[:, :kl] = s, i
            s, i = ps, pi
        return s, i

    def search_owned(self, query_embeddings: torch.Tensor, k: Optional[int] = None
                     ) -> Tuple[Tuple[int, int], torch.Tensor, torch.Tensor]:
        """Exact global top-k of this rank's query block: ((begin, end),
        scores [end-begin, k], indices [end-begin, k] int32)."""
        k = k or self.k
        Q, G = int(query_embeddings.shape[0]), self.world
        s, i = self.search_shard(query_embeddings, k)
        blocks = [shard_range(Q, G, r) for r in range(G)]
        mb, me = blocks[self.rank]
        if G == 1:
            return (mb, me), s, i
        nb = me - mb
        in_splits = [(e - b) * k for b, e in blocks]
        rs = torch.empty(G * nb * k, dtype=s.dtype, device=s.device)
        ri = torch.empty(G * nb * k, dtype=i.dtype, device=i.device)
        _a2a(rs, s.reshape(-1), [nb * k] * G, in_splits, self.group)
        _a2a(ri, i.reshape(-1), [nb * k] * G, in_splits, self.group)
        if nb == 0:
            return (mb, me), s[:0], i[:0]
        ms, mi = self.ops.merge(rs.view(G, nb, k), ri.view(G, nb, k), k)
        return (mb, me), ms, mi

    def search(self, query_embeddings: torch.Tensor, k: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Global (scores [Q,k], indices [Q,k]) on every rank (blocks all-gathered)."""
        Q = int(query_embeddings.shape[0])
        _, s, i = self.search_owned(query_embeddings, k)
        if self.world == 1:
            return s, i
        return _gather_query_blocks(s, i, Q, self.world, self.group)

    def __call__(self, queries: Dict[str, Any]):
        with torch.no_grad():
            emb = self.query_model(queries)
        return self.search(emb)[1]


class QueryShardedBruteForceIndex:
    """
    Query-parallel brute-force index: every rank keeps the WHOLE candidate
    matrix (C4: 105,542 x 128 fp32 = 54 MB + a 27 MB bf16 image, nothing
    against 288 GB of HBM) and answers its block of the queries,
    shard_range(Q, world, rank).  No merge and no exchange on the search path,
    so QPS scales with the ranks; ShardedBruteForceIndex (candidate-sharded,
    the layout the north star names) is the one that scales the candidate
    count instead.  Results are identical to the single-GPU search (the same
    kernel on the same candidates).
    """

    def __init__(self, k: int, query_model, candidates: torch.Tensor, identifiers=None, group=None,
                 ops: Optional[IndexOps] = None):
        self.k = int(k)
        self.query_model = query_model
        self.group = group
        self.ops = ops or IndexOps.hip()
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.cand = candidates.contiguous()
        if self.cand.shape[0] < self.k:
            raise ValueError(f"need >= k={self.k} candidates, got {self.cand.shape[0]}")
        self.num_candidates = self.cand.shape[0]
        self.image = self.ops.build(self.cand)
        self.identifiers = identifiers

    def search_owned(self, query_embeddings: torch.Tensor, k: Optional[int] = None
                     ) -> Tuple[Tuple[int, int], torch.Tensor, torch.Tensor]:
        """((begin, end), scores [end-begin, k], indices) of this rank's query block."""
        k = k or self.k
        b, e = shard_range(int(query_embeddings.shape[0]), self.world, self.rank)
        s, i = self.ops.search(self.image, self.cand, query_embeddings[b:e].contiguous(), k, 0)
        return (b, e), s, i

    def search(self, query_embeddings: torch.Tensor, k: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Global (scores [Q,k], indices [Q,k]) on every rank (blocks all-gathered)."""
        Q = int(query_embeddings.shape[0])
        _, s, i = self.search_owned(query_embeddings, k)
        return _gather_query_blocks(s, i, Q, self.world, self.group)

    def __call__(self, queries: Dict[str, Any]):
        with torch.no_grad():
            emb = self.query_model(queries)
        return self.search(emb)[1]


# --------------------------------------------------------------------------- row-sharded tables
@dataclass
class EmbeddingOps:
    """Kernels of the row-sharded path (defaults: libtt; tests inject CPU ones)."""
    gather_multi: Callable[..., None]
    gather_tagged: Callable[..., torch.Tensor]
    scatter_sum: Callable[..., None]
    sparse_adagrad: Callable[..., None]
    dense_adagrad: Callable[..., None]
    # the compact route (tt_route_requests / tt_route_owner / tt_route_pad);
    # libtt's in EmbeddingOps.hip(), the CPU tests inject restatements
    route_requests: Optional[Callable[..., Any]] = None
    route_owner: Optional[Callable[..., Any]] = None
    route_pad: Optional[Callable[..., Any]] = None
    # Adagrad on distinct rows (a one-rank owner's requests); None: sparse_adagrad
    sparse_adagrad_rows: Optional[Callable[..., None]] = None
    # per-request sums / Adagrad keyed by the route's own sort (no second
    # sort; needs route_requests(..., ordered=True)); None: scatter_sum
    sparse_routed: Optional[Callable[..., None]] = None
    # the whole fixed route in one call (tt_route_fixed); None: route_requests
    # + route_pad + route_owner
    route_fixed: Optional[Callable[..., Any]] = None
    # dense_adagrad on several (param, accum, grad) buffers in one launch
    dense_adagrad_many: Optional[Callable[..., None]] = None
    # scatter_sum in two stages: the key sort (ids only) early, the sums later
    scatter_sort: Optional[Callable[..., None]] = None
    scatter_sum_sorted: Optional[Callable[..., None]] = None

    def need(self, name: str) -> Callable[..., Any]:
        fn = getattr(self, name)
        if fn is None:
            raise ValueError(f"EmbeddingOps.{name} is not set (EmbeddingOps.hip() provides libtt's)")
        return fn

    @staticmethod
    def hip() -> "EmbeddingOps":
        from pkg.modelling import hip_ops

        # distinct workspaces: the scatter-sum runs inside the captured middle of
        # ShardedTrainStep (fixed size), the owner-side Adagrad outside it with
        # a size that varies per step — it must never move the graph's buffer
        return EmbeddingOps(hip_ops.gather_multi, hip_ops.gather_tagged,
                            lambda specs, b, g: hip_ops.sparse_scatter_sum(specs, b, g, ws_tag="sparse_mid"),
                            lambda specs, b, g, lr, eps: hip_ops.sparse_adagrad(specs, b, g, lr, eps,
                                                                                ws_tag="sparse_owner"),
                            hip_ops.dense_adagrad, hip_ops.route_requests, hip_ops.route_owner,
                            hip_ops.route_pad, hip_ops.sparse_adagrad_rows, hip_ops.sparse_routed,
                            hip_ops.route_fixed, hip_ops.dense_adagrad_many,
                            lambda specs, b: hip_ops.sparse_sort(specs, b, ws_tag="sparse_mid", slots=False),
                            lambda specs, b, g: hip_ops.sparse_scatter_sum(specs, b, g, ws_tag="sparse_mid",
                                                                           presorted=True))


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits: List[int], in_splits: List[int], group,
         force: bool = False) -> torch.Tensor:
    if dist.get_world_size(group) == 1 and not force:  # one rank: the exchange is the identity
        if out.numel():
            out.copy_(inp)
        return out
    if _staged(group) and inp.is_cuda:  # gloo: through the host
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(h, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(h)
        return out
    dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)
    return out


def _all_reduce_sum(t: torch.Tensor, group, force: bool = False) -> None:
    if dist.get_world_size(group) == 1 and not force:  # one rank: the sum is the tensor
        return
    if _staged(group) and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, group=group)


class BatchComm:
    """all_gather / reduce_scatter of equal per-rank blocks along dim 0, for
    the global-negatives loss (losses.global_inbatch_grads): RCCL
    all_gather_into_tensor / reduce_scatter_tensor; over gloo (CPU tests, or
    several ranks sharing one GPU) through the host."""

    def __init__(self, group=None, always: bool = False):
        """always: run the collectives at world 1 too (one-rank RCCL calls;
        the tests use it to put real collectives into a captured step)."""
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.always = bool(always)

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        if self.world == 1 and not self.always:
            return t
        out = _all_gather_any(t.contiguous(), self.group)
        return out.reshape((self.world * t.shape[0],) + tuple(t.shape[1:]))

    def reduce_scatter(self, t: torch.Tensor) -> torch.Tensor:
        if self.world == 1 and not self.always:
            return t
        n = t.shape[0] // self.world
        if _staged(self.group):  # gloo has no reduce_scatter: sum everywhere, keep this rank's block
            h = t.detach().cpu().contiguous()
            dist.all_reduce(h, group=self.group)
            return h[self.rank * n:(self.rank + 1) * n].to(t.device)
        out = torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.reduce_scatter_tensor(out, t.contiguous(), group=self.group)
        return out


class _Route:
    """Where one batch's sharded lookups go and come back from; depends only on
    the ids, so it can be computed a step ahead (ShardedTables.route)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def tensors(self) -> List[torch.Tensor]:
        return [self.tags, self.rows, *self.table_ids, *self.idx]


class ShardedTables:
    """
    Embedding tables row-sharded over the ranks: global row r
    lives on rank r % world at local row r // world, so every rank owns ~1/world
    of each table and of its Adagrad accumulator.

    One exchange per step for all sharded tables:
      routing   (ids only: can run a step ahead, on a side stream, over its
                own process group) each rank dedups its lookups per table,
                buckets the distinct (table, row) requests by owner and sends
                them with one all_to_all (plus one tiny count exchange — the
                step's only host sync);
      forward   owners answer with one tt_gather_tagged launch and one
                all_to_all of rows back;
      backward  each rank sums its lookup gradients per request
                (tt_sparse_scatter_sum, same order as the single-GPU dedup),
                one all_to_all sends them to the owners, and each owner applies
                tt_sparse_adagrad to its shard (duplicate rows from different
                ranks summed in rank order).
    All sharded tables share one embedding width (rows move as [n, dim]).
    """

    def __init__(self, tables: Dict[str, torch.Tensor], init_accumulator: float = 0.1, group=None,
                 ops: Optional[EmbeddingOps] = None, full_tables: bool = True, always: bool = False):
        """tables: name -> full [rows, dim] table (full_tables=True, the shard is
        sliced out) or this rank's shard with a "__rows__" entry giving the
        global row counts (full_tables=False, for tables too big to build).
        always: take the multi-rank path at world 1 too — the request, row and
        gradient all_to_alls run as real one-rank collectives instead of being
        skipped (tests: the N > 1 step's exchanges inside a captured graph on
        one GPU, as BatchComm(always=True) does for the global negatives)."""
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.always = bool(always)
        self.exchange = self.world > 1 or self.always  # the exchanges run (else: identities, skipped)
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

    # -- routing (ids only) ------------------------------------------------
    def route(self, lookups: List[Tuple[str, torch.Tensor]], group=None) -> _Route:
        """lookups: (table name, ids [B] int32).  Collectives run on `group`
        (default: the tables' group) and on the current stream."""
        return self.route_finish(self.route_begin(lookups, group))

    def route_begin(self, lookups: List[Tuple[str, torch.Tensor]], group=None) -> dict:
        """First half of route(), no host sync: dedup + owner bucketing and the
        count exchange are enqueued on the current stream, the counts copied
        to pinned host memory behind an event.  route_finish() completes it
        (by then the counts have long landed, so its wait is free)."""
        group = self.group if group is None else group
        W, T = self.world, len(self.names)
        dev = lookups[0][1].device
        tagged = [(ids.reshape(-1), self.rows[name], self.names.index(name)) for name, ids in lookups]
        send, send_counts, _, idx = self.ops.need("route_requests")(tagged, W, T)
        recv_counts = torch.empty_like(send_counts)
        _a2a(recv_counts, send_counts, [1] * W, [1] * W, group)
        both = torch.stack([send_counts, recv_counts])
        pinned = dev.type == "cuda"
        host = torch.empty(both.shape, dtype=both.dtype, pin_memory=pinned)
        host.copy_(both, non_blocking=pinned)
        ev = None
        if pinned:
            ev = torch.cuda.Event()
            ev.record()
        return dict(group=group, dev=dev, send=send, idx=idx, host=host, event=ev, keep=(both, send_counts))

    def route_finish(self, pend: dict) -> _Route:
        W, T = self.world, len(self.names)
        t0 = time.perf_counter()
        if pend["event"] is not None:
            pend["event"].synchronize()  # the step's one host sync, normally long complete
        pend["sync_s"] = time.perf_counter() - t0
        s_split, r_split = pend["host"][0].tolist(), pend["host"][1].tolist()
        R = int(sum(s_split))
        recv = torch.empty(sum(r_split), 2, dtype=torch.int32, device=pend["dev"])
        _a2a(recv, pend["send"][:R], r_split, s_split, pend["group"])
        tags, rows, tids = self.ops.need("route_owner")(recv, W, T)
        return _Route(s_split=s_split, r_split=r_split, R=R, n_recv=int(sum(r_split)), tags=tags, rows=rows,
                      table_ids=list(tids.unbind(0)), idx=list(pend["idx"].unbind(0)), idx_all=pend["idx"],
                      dev=pend["dev"])

    def route_capacity(self, num_lookups: int, batch: int) -> int:
        """Requests one rank can send one owner, at most: every lookup
        distinct, capped by the rows a table can have on one owner."""
        return max(1, num_lookups * batch)

    def route_fixed(self, lookups: List[Tuple[str, torch.Tensor]], cap: int, group=None,
                    overflow: Optional[torch.Tensor] = None, idx_out: Optional[torch.Tensor] = None) -> _Route:
        """route() with `cap` fixed request slots per owner (tt_route_pad):
        every exchange has split sizes [cap] * world, known on the host
        before the step, so routing, fetch and apply run with no host sync
        and can be captured into a hipGraph.  Unused slots carry (-1, -1):
        owners answer them with zero rows and apply nothing to them.  With
        cap = route_capacity(...) no request is ever dropped; a smaller cap
        counts dropped requests in `overflow`.  idx_out ([L, B] int32):
        where the lookups' slots are written (rt.idx_all is then idx_out)."""
        group = self.group if group is None else group
        W, T = self.world, len(self.names)
        dev = lookups[0][1].device
        tagged = [(ids.reshape(-1), self.rows[name], self.names.index(name)) for name, ids in lookups]
        order = own = None
        ordered = self.ops.sparse_routed is not None  # keep the route's sort for apply_lookups
        if self.ops.route_fixed is not None:  # one call (one launch for small batches)
            send_p, idx_p, counts, order, own = self.ops.route_fixed(tagged, W, T, cap, overflow, ordered=ordered,
                                                                     owner=not self.exchange, idx_out=idx_out)
        else:
            if ordered:
                send, counts, _, idx, order = self.ops.need("route_requests")(tagged, W, T, ordered=True)
            else:
                send, counts, _, idx = self.ops.need("route_requests")(tagged, W, T)
            send_p, idx_p = self.ops.need("route_pad")(send, counts, idx, W, cap, overflow)
            if idx_out is not None:
                idx_out.copy_(idx_p)
                idx_p = idx_out
        split = [cap] * W
        recv = send_p  # world 1: the exchange is the identity
        if self.exchange:
            recv = torch.empty(W * cap, 2, dtype=torch.int32, device=dev)
            _a2a(recv, send_p, split, split, group, self.always)
        tags, rows, tids = own if own is not None else self.ops.need("route_owner")(recv, W, T)
        return _Route(s_split=split, r_split=split, R=W * cap, n_recv=W * cap, tags=tags, rows=rows,
                      table_ids=list(tids.unbind(0)), idx=list(idx_p.unbind(0)), idx_all=idx_p, dev=dev,
                      counts=counts, order=order, cap=cap, lookup_tags=[t for _, _, t in tagged])

    # -- forward -----------------------------------------------------------
    def fetch_routed(self, rt: _Route, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Rows of the routed requests, [R, dim] (into out[:R] when given)."""
        got = out[:rt.R] if out is not None else torch.empty(rt.R, self.dim, dtype=torch.float32, device=rt.dev)
        if not self.exchange:  # one rank: the owner's answer IS the fetched rows
            self.ops.gather_tagged([self.shard[n] for n in self.names], rt.tags, rt.rows, got)
            return got
        reply = torch.empty(rt.n_recv, self.dim, dtype=torch.float32, device=rt.dev)
        self.ops.gather_tagged([self.shard[n] for n in self.names], rt.tags, rt.rows, reply)
        _a2a(got, reply, rt.s_split, rt.r_split, self.group, self.always)
        return got

    def fetch(self, lookups: List[Tuple[str, torch.Tensor]], capacity: Optional[int] = None,
              overflow: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, List[torch.Tensor]]:
        """lookups: (table name, ids [B] int32) -> (rows [R, dim], row index per
        lookup [B] int32): lookup l's embedding of batch row b is rows[idx_l[b]].
        capacity: route with that many fixed slots per owner (route_fixed: no
        host sync; "full" = route_capacity, never overflows)."""
        if capacity is not None:
            if capacity == "full":
                capacity = self.route_capacity(len(lookups), lookups[0][1].numel())
            rt = self.route_fixed(lookups, int(capacity), overflow=overflow)
            self._ctx = rt
            return self.fetch_routed(rt), rt.idx
        rt = self.route(lookups)
        self._ctx = rt
        return self.fetch_routed(rt), rt.idx

    # -- one rank: nothing to exchange --------------------------------------
    def fetch_local(self, lookups: List[Tuple[str, torch.Tensor]], out: torch.Tensor) -> torch.Tensor:
        """World 1 (this rank owns every row): the rows of each lookup (table
        name, ids [B]) read from the shard by id, lookup l into out[l] ([L, B,
        dim]) — one gather launch, no route.  The rows route_fixed +
        fetch_routed would return, per lookup."""
        if self.world != 1:
            raise ValueError("fetch_local: one rank only (world %d)" % self.world)
        B = lookups[0][1].numel()
        self.ops.gather_multi([([(self.shard[name], ids.reshape(-1), 0)], out[l])
                               for l, (name, ids) in enumerate(lookups)], B)
        return out

    def apply_local(self, lookups: List[Tuple[str, torch.Tensor]], grads: List[Tuple[torch.Tensor, int]],
                    lr: float, eps: float) -> None:
        """World 1: Adagrad on the shards from per-lookup gradients (grads[l]
        = (gradient matrix [B, width], column) of lookup l) keyed by the ids
        themselves — the single-device dedup + update (one sort, the block
        sums, the update), with no route: the same update route_fixed +
        apply_lookups makes at one rank (their world-1 form IS this
        tt_sparse_adagrad on the same keys, bit for bit while every id is in
        range; an out-of-range id sorts first in the route and last here,
        which regroups the block sums within fp32 rounding —
        tests/test_configs_gpu.py)."""
        if self.world != 1:
            raise ValueError("apply_local: one rank only (world %d)" % self.world)
        if len(grads) != len(lookups):
            raise ValueError(f"apply_local: {len(grads)} gradients for {len(lookups)} lookups")
        B = lookups[0][1].numel()
        specs: Dict[str, dict] = {}
        for (name, ids), (gmat, col) in zip(lookups, grads):
            sp = specs.setdefault(name, dict(table=self.shard[name], slot0=self.acc[name], ids=[],
                                             grad_col_offset=[], grad=gmat))
            if sp["grad"] is not gmat:
                raise ValueError("apply_local: the lookups of one table must share one gradient matrix")
            sp["ids"].append(ids.reshape(-1))
            sp["grad_col_offset"].append(int(col))
        self.ops.sparse_adagrad(list(specs.values()), B, None, lr, eps)

    # -- backward + update -------------------------------------------------
    def apply_routed(self, rt: _Route, g_req: torch.Tensor, lr: float, eps: float) -> None:
        """g_req[:R]: the per-request gradient sums of the routed requests;
        returns them to the owners, which apply Adagrad to their shards."""
        if not self.exchange:  # one rank: the per-request sums are already the owner's
            recv = g_req[:rt.R]
            if self.ops.sparse_adagrad_rows is not None:
                # one rank's requests are distinct (tag, row) pairs: no sort, no sums
                self.ops.sparse_adagrad_rows([(self.shard[n], self.acc[n]) for n in self.names], rt.tags, rt.rows,
                                             recv, lr, eps)
                return
        else:
            recv = torch.empty(rt.n_recv, self.dim, dtype=torch.float32, device=rt.dev)
            _a2a(recv, g_req[:rt.R], rt.r_split, rt.s_split, self.group, self.always)
        specs = [dict(table=self.shard[name], slot0=self.acc[name], ids=[rt.table_ids[ti]], grad_col_offset=[0])
                 for ti, name in enumerate(self.names)]
        if recv.shape[0] > 0:
            self.ops.sparse_adagrad(specs, recv.shape[0], recv, lr, eps)

    def apply_lookups(self, rt: _Route, grads: List[Tuple[torch.Tensor, int]], lr: float, eps: float,
                      g_req: Optional[torch.Tensor] = None) -> None:
        """Adagrad on the shards from the gradients of a route_fixed batch's
        lookups: grads[l] = (gradient matrix [B, width], column) of routed
        lookup l.  With ops.sparse_routed (libtt) the per-request sums reuse
        the route's sort (tt_sparse_routed): at world 1 they go straight into
        the Adagrad update of the shard (the single-GPU tt_sparse_adagrad on the
        same keys, no per-request buffer), otherwise into g_req (default: a
        fresh [world*cap, dim] buffer) for apply_routed.  Without it:
        scatter_sum, then apply_routed."""
        if len(grads) != len(rt.idx):
            raise ValueError(f"apply_lookups: {len(grads)} gradients for {len(rt.idx)} routed lookups")
        B = rt.idx[0].numel()
        specs, tables_of_tag, lk_table, lk_source = [], {}, [], []
        for l, (gmat, col) in enumerate(grads):
            tag = rt.lookup_tags[l]
            if tag not in tables_of_tag:
                tables_of_tag[tag] = len(specs)
                specs.append(dict(ids=[], grad_col_offset=[], grad=gmat, tag=tag))
            sp = specs[tables_of_tag[tag]]
            if sp["grad"] is not gmat:
                raise ValueError("apply_lookups: the lookups of one table must share one gradient matrix")
            lk_table.append(tables_of_tag[tag])
            lk_source.append(len(sp["ids"]))
            sp["ids"].append(rt.idx[l])
            sp["grad_col_offset"].append(int(col))
        routed = self.ops.sparse_routed is not None and getattr(rt, "order", None) is not None
        if g_req is None and not (not self.exchange and routed):
            g_req = torch.zeros(rt.R, self.dim, dtype=torch.float32, device=rt.dev)
        if not routed:
            for sp in specs:
                sp["table"] = g_req
            self.ops.scatter_sum([{k: v for k, v in sp.items() if k != "tag"} for sp in specs], B, grads[0][0])
            self.apply_routed(rt, g_req, lr, eps)
            return
        route = dict(order=rt.order[0], grp_first=rt.order[1], grp_last=rt.order[2], slot=rt.idx_all, cap=rt.cap,
                     world=self.world, num_tags=len(self.names), lookup_tag=rt.lookup_tags, lookup_table=lk_table,
                     lookup_source=lk_source)
        if not self.exchange:  # the owner is this rank: Adagrad on the shard, keyed by local row
            route["slot_row"] = rt.rows
            for sp in specs:
                name = self.names[sp["tag"]]
                sp["table"], sp["slot0"] = self.shard[name], self.acc[name]
            self.ops.sparse_routed([{k: v for k, v in sp.items() if k != "tag"} for sp in specs], B, None, route,
                                   "adagrad", lr, eps)
            return
        for sp in specs:
            sp["table"] = g_req
        self.ops.sparse_routed([{k: v for k, v in sp.items() if k != "tag"} for sp in specs], B, None, route, "sum")
        self.apply_routed(rt, g_req, lr, eps)

    def apply(self, grads: List[Tuple[torch.Tensor, List[Tuple[torch.Tensor, int]]]], lr: float, eps: float) -> None:
        """grads: per gradient matrix [B, width] its (row index from fetch, column)
        sources.  Sums per request, returns the sums to the owners, and applies
        Adagrad to the local shards."""
        rt = self._ctx
        g_req = torch.zeros(rt.R, self.dim, dtype=torch.float32, device=rt.dev)
        for gmat, sources in grads:
            if not sources:
                continue
            spec = [dict(table=g_req, ids=[s[0] for s in sources], grad_col_offset=[s[1] for s in sources])]
            self.ops.scatter_sum(spec, gmat.shape[0], gmat)
        self.apply_routed(rt, g_req, lr, eps)
        self._ctx = None

    def gather_full(self, name: str, accumulator: bool = False) -> torch.Tensor:
        """The full table (or its Adagrad accumulator) reassembled on every
        rank (checks / export)."""
        rows, W = self.rows[name], self.world
        src = self.acc[name] if accumulator else self.shard[name]
        per = (rows + W - 1) // W
        mine = torch.zeros(per, self.dim, dtype=torch.float32, device=src.device)
        mine[:src.shape[0]] = src
        parts = _all_gather_any(mine, self.group)
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
    (ShardedTables) and the small ones replicated; in-batch negatives from
    the global batch by default (below).  Sparse work per rank stays ~constant
    as ranks are added (each owner updates only its rows), unlike gathering
    every replica's sparse gradients.

    Per step, one hipGraph replay (over RCCL; the first call runs eagerly and
    warms every buffer) on the compute stream, with no host work but the
    batch copy:
      1. routing: the rank's sharded lookups deduplicated and bucketed by
         owner (tt_route_requests), laid into `route_capacity` fixed slots per
         owner (tt_route_pad, no host sync), one all_to_all of the requests
         with split sizes known before the step, the owners' local rows
         (tt_route_owner);
      2. fetch: owners answer (tt_gather_tagged), one all_to_all brings the
         rows back into a static buffer;
      3. the middle — both towers' gathers (one tt_gather_multi), the MLPs +
         fused in-batch loss forward and backward, the per-request gradient
         sums of the sharded tables and the dense gradients of the small ones
         (ONE tt_sparse_scatter_sum: one sort), packed with the MLP gradients
         and the loss into one bucket, one all_reduce of the bucket, then
         tt_dense_adagrad on the two tower MLP buffers and on ONE flat buffer
         holding every small table;
      4. one all_to_all returns the per-request sums to the owners, which
         apply tt_sparse_adagrad to their shards (padding slots: nothing).
    route_capacity (default: num_sharded_lookups x batch, the most one rank
    can ever send one owner) trades exchange bytes for safety: a smaller
    value sends less padding, and a step that overflows it drops requests and
    is reported by check_status().  At world 1 the exchanges are identities
    and the bucket's all_reduce is skipped.

    global_negatives=True (the reference's semantics, two_tower_model.py:
    113-122: every query row's negatives are the candidates of the GLOBAL
    batch): the towers run on this rank's rows, the candidate embeddings and
    logq are all-gathered, the rows pass scores this rank's queries against
    all of them (positive of local row i = global column rank*b + i); the
    query embeddings and their lse are all-gathered and the cols pass scores
    all of them against this rank's candidates (dC of its columns).  The
    loss and every gradient are those of the global batch (tests:
    test_distributed_gloo global loss, test_distributed_gpu step).  This is
    the default.  Over RCCL the middle's all_gathers and reduce_scatters are
    captured into its hipGraph with the kernels (test_model_gpu: a captured
    world-1 step with forced one-rank RCCL collectives is bit-identical to
    the eager one); over gloo it runs eagerly.
    global_negatives=False keeps per-replica negatives (a labelled variant:
    each rank's loss over its own batch).

    Adagrad (the reference's optimizer, main.py:100-101) only.
    """

    def __init__(self, model, shard_min_rows: int = 100_000, group=None, ops: Optional[EmbeddingOps] = None,
                 use_graph: bool = True, global_negatives: bool = True, comm: Optional[BatchComm] = None,
                 route_capacity: Optional[int] = None, always_exchange: bool = False):
        """always_exchange: the multi-rank structure at world 1 too (the
        sharded tables' all_to_alls and the bucket's all_reduce as real
        one-rank collectives, ShardedTables(always=True)) — how one GPU runs
        the N > 1 step's graph over RCCL (tests)."""
        from pkg.modelling.optimizer_factory import Adagrad

        opt = model.optimizer
        if not isinstance(opt, Adagrad):
            raise NotImplementedError("ShardedTrainStep supports the Adagrad optimizer")
        self.model = model
        self.group = group
        self.ops = ops or EmbeddingOps.hip()
        self.world = dist.get_world_size(group)
        self.lr, self.eps, self.init = opt.learning_rate, opt.epsilon, opt.initial_accumulator_value
        self.global_negatives = bool(global_negatives)
        self.comm = (comm or BatchComm(group)) if self.global_negatives else None
        # the step holds collectives (the route's and the rows' all_to_alls,
        # the bucket's all_reduce; the global negatives' all_gathers and
        # reduce_scatters): over RCCL they are captured into the step's
        # hipGraph with the kernels (the default; TT_SHARDED_EAGER=1 runs the
        # step eagerly); over gloo, whose host staging synchronises, the step
        # runs eagerly.  At world 1 every exchange is skipped.
        self.route_capacity = None if route_capacity is None else int(route_capacity)
        self.always = bool(always_exchange)
        self.exchange = self.world > 1 or self.always
        collectives = self.exchange or (self.global_negatives and self.comm.always)
        self.use_graph = use_graph and os.environ.get("TT_SHARDED_EAGER") != "1" and not (
            collectives and _staged(group))
        big: Dict[str, torch.Tensor] = {}
        self.small: Dict[Any, Any] = {}
        for tower in model.towers:
            for name, t in tower.input_layer.embedding_layers.items():
                key = (id(tower), name)
                if t.num_rows >= shard_min_rows:
                    big[f"{len(big)}:{name}"] = t.weight
                    t._shard_key = f"{len(big) - 1}:{name}"
                else:
                    self.small[key] = t
        self.tables = ShardedTables(big, self.init, group, self.ops, always=self.always) if big else None
        for tower in model.towers:  # drop the full copies of sharded tables
            for t in tower.input_layer.embedding_layers.values():
                if hasattr(t, "_shard_key"):
                    t.weight = None
        # every small (replicated) table becomes a view of ONE flat buffer, so
        # its dense gradient is one zero-fill and its update one launch
        dev = model.device
        n_small = sum(t.weight.numel() for t in self.small.values())
        self._small_flat = torch.empty(max(n_small, 1), dtype=torch.float32, device=dev)
        self._small_grad = torch.zeros_like(self._small_flat)
        self._small_views: Dict[Any, Tuple[torch.Tensor, torch.Tensor]] = {}
        off = 0
        for key, t in self.small.items():
            n = t.weight.numel()
            self._small_flat[off:off + n].copy_(t.weight.reshape(-1))
            t.weight = self._small_flat[off:off + n].view(t.num_rows, t.dim)
            self._small_views[key] = (t.weight, self._small_grad[off:off + n].view(t.num_rows, t.dim))
            off += n
        self._small_acc = torch.full_like(self._small_flat, self.init)
        self._dense_acc = [torch.full_like(t.dense.flat, self.init) for t in model.towers]
        self._static = None      # static batch / request buffers (set up on the first call)
        self._graph = None
        self._calls = 0
        self._out_grads = None
        self.host_times: Optional[Dict[str, float]] = {} if os.environ.get("TT_HOST_PROFILE") else None
        _LIVE_STEPS.add(self)

    def close(self) -> None:
        """Release the captured step graph (the next call captures again).
        Call it before the process group is destroyed
        (distributed.destroy_process_group does): the graph holds the
        group's RCCL collectives."""
        if self._graph is not None:
            torch.cuda.synchronize(self.model.device)
            self._graph.reset()
            self._graph = None
            self._graph_events = []

    def __enter__(self) -> "ShardedTrainStep":
        return self

    def __exit__(self, *exc) -> bool:
        self.close()
        return False

    def _tick(self, name: str, t0: float) -> float:
        t1 = time.perf_counter()
        if self.host_times is not None:
            self.host_times[name] = self.host_times.get(name, 0.0) + (t1 - t0)
        return t1

    # -- static buffers ----------------------------------------------------
    def _lookups(self, batch) -> List[Tuple[str, torch.Tensor, int, int]]:
        """(shard key, ids, tower index, column offset) of every sharded lookup."""
        m = self.model
        q, c = m._split(batch)
        out = []
        for li, (layer, x) in enumerate(zip([t.input_layer for t in m.towers], [q, c])):
            for f, off in zip(layer.categorical_features, layer.column_offsets()):
                t = layer.embedding_layers[f.name]
                if hasattr(t, "_shard_key"):
                    out.append((t._shard_key, layer._ids(x[f.name]), li, off))
        return out

    def _setup(self, batch) -> None:
        m = self.model
        dev = m.device
        # the batch lives in one int32 [K, B] and one fp32 [F, B] buffer, loaded
        # with one stacking launch each
        self._static = {}
        kinds = {}
        for k, v in batch.items():
            t = v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))
            kinds[k] = torch.float32 if t.is_floating_point() else torch.int32
            B0 = t.numel()
        self._int_keys = sorted(k for k, d in kinds.items() if d == torch.int32)
        self._float_keys = sorted(k for k, d in kinds.items() if d == torch.float32)
        self._ibuf = torch.empty(max(len(self._int_keys), 1), B0, dtype=torch.int32, device=dev)
        self._fbuf = torch.empty(max(len(self._float_keys), 1), B0, dtype=torch.float32, device=dev)
        self._static.update({k: self._ibuf[i] for i, k in enumerate(self._int_keys)})
        self._static.update({k: self._fbuf[i] for i, k in enumerate(self._float_keys)})
        lk = self._lookups(self._static)
        B = next(iter(self._static.values())).numel()
        self._B = B
        full = self.tables.route_capacity(len(lk), B) if self.tables is not None else 1
        self._cap = full if self.route_capacity is None else max(1, min(self.route_capacity, full))
        slots = self.world * self._cap
        dim = self.tables.dim if self.tables is not None else 1
        # the fetched rows (world 1: unused, the middle reads the shard)
        self._got = torch.zeros(slots if self.exchange else 1, dim, dtype=torch.float32, device=dev)
        self._g_req = torch.zeros(slots, dim, dtype=torch.float32, device=dev)
        # dropped requests (capacity); TT_SHARDED_DEBUG=1: between two canary words
        self._canary = torch.full((3,), 0x7EADBEEF, dtype=torch.int32, device=dev)
        self._canary[1] = 0
        self._overflow = self._canary[1:2]
        self._idx_all = torch.zeros(max(len(lk), 1), B, dtype=torch.int32, device=dev)  # route_fixed writes the slots here
        self._idx = list(self._idx_all[:len(lk)].unbind(0))
        self._loss = torch.zeros((), dtype=torch.float32, device=dev)
        n_bucket = sum(t.dense.flat.numel() for t in m.towers) + self._small_grad.numel() + 1
        self._bucket = torch.zeros(n_bucket, dtype=torch.float32, device=dev)

    def _load(self, batch) -> None:
        dev = self._ibuf.device

        def col(k, dtype):
            v = batch[k]
            t = v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))
            return t.reshape(-1).to(device=dev, dtype=dtype)

        if self._int_keys:
            torch.stack([col(k, torch.int32) for k in self._int_keys], out=self._ibuf)
        if self._float_keys:
            torch.stack([col(k, torch.float32) for k in self._float_keys], out=self._fbuf)

    # -- the static middle (graph-captured) --------------------------------
    def _middle(self) -> None:
        m = self.model
        x = self._static
        q, c = m._split(x)
        layers = [t.input_layer for t in m.towers]
        calls, widths = [], []
        j = 0
        for li, (layer, xx) in enumerate(zip(layers, [q, c])):
            segs = []
            for f in layer.numerical_features:
                segs.append((xx[f.name].to(torch.float32), None, len(segs)))
            for f, off in zip(layer.categorical_features, layer.column_offsets()):
                t = layer.embedding_layers[f.name]
                if hasattr(t, "_shard_key"):
                    if not self.exchange:  # one rank: the shard IS the fetched rows, read by id directly
                        segs.append((self.tables.shard[t._shard_key], layer._ids(xx[f.name]), off))
                    else:
                        segs.append((self._got, self._idx[j], off))
                    j += 1
                else:
                    segs.append((t.weight, layer._ids(xx[f.name]), off))
            out = torch.empty(self._B, layer.row_stride, dtype=torch.float32, device=layer.device)
            calls.append((segs, out))
            widths.append(layer.output_dim)
        anchors = [layer._anchor for layer in layers]
        qi, ci = _ShardedGatherFn.apply(self, calls, self._B, widths, *anchors)
        if self.global_negatives:
            from pkg.modelling.losses import global_towers_inbatch_softmax_xent

            if m.loss.reduction != "sum":
                raise NotImplementedError("global negatives: the reference's SUM reduction only")
            loss = global_towers_inbatch_softmax_xent(qi, ci, m.query_tower.dense, m.candidate_tower.dense,
                                                      self.comm, m.candidate_logq(x))
        else:
            loss = m.tower_loss(qi, ci, m.candidate_logq(x))
        for t in m.towers:
            t.dense.flat.grad = None
        if getattr(self, "_one", None) is None:
            self._one = torch.ones((), dtype=loss.dtype, device=loss.device)
        loss.backward(self._one)  # a persistent seed: no ones-fill launch per step
        grads = self._out_grads
        # one scatter-sum call: per-request sums of the sharded tables' lookups
        # (rows of g_req, disjoint per table) and dense small-table gradients
        self._small_grad.zero_()
        specs = [dict(sp, grad=grads[li]) for sp, li in self._scatter_specs()]
        self._join_route()  # the per-request sums read the route's slots (and its sorted keys)
        if specs:
            if self._presorted:
                self.ops.scatter_sum_sorted(specs, self._B, grads[0])
            else:
                self.ops.scatter_sum(specs, self._B, grads[0])
        self._dense_update([t.dense.flat.grad for t in m.towers], loss.detach())

    def _scatter_specs(self) -> List[Tuple[dict, int]]:
        """(scatter-sum table spec without its gradient, tower index) of every
        table the step's sums write: the sharded tables' per-request sums
        (ids = the lookups' slots) and the small tables' dense gradients
        (ids = the batch's ids).  Static buffers only, so computed once."""
        if getattr(self, "_sspecs", None) is not None:
            return self._sspecs
        m = self.model
        q, c = m._split(self._static)
        big_srcs, small_srcs = {}, {}
        j = 0
        for li, (layer, xx) in enumerate(zip([t.input_layer for t in m.towers], [q, c])):
            for f, off in zip(layer.categorical_features, layer.column_offsets()):
                t = layer.embedding_layers[f.name]
                if hasattr(t, "_shard_key"):
                    big_srcs.setdefault(t._shard_key, (li, []))[1].append((self._idx[j], off))
                    j += 1
                else:
                    small_srcs.setdefault((id(m.towers[li]), f.name), (li, []))[1].append(
                        (layer._ids(xx[f.name]), off))
        specs = []
        for key, (li, srcs) in big_srcs.items():
            specs.append((dict(table=self._g_req, ids=[s[0] for s in srcs], grad_col_offset=[s[1] for s in srcs]),
                          li))
        for key, (li, srcs) in small_srcs.items():
            specs.append((dict(table=self._small_views[key][1], ids=[s[0] for s in srcs],
                               grad_col_offset=[s[1] for s in srcs]), li))
        # cached only while every id tensor is a view of the static buffers
        # (the batch's int32 rows, the route's slots): a categorical column
        # staged as floats makes _ids return a fresh copy per call
        static = {t.untyped_storage().data_ptr() for t in (self._ibuf, self._idx_all)}
        if all(ids.untyped_storage().data_ptr() in static for sp, _ in specs for ids in sp["ids"]):
            self._sspecs = specs
        return specs

    def _dense_update(self, flat_grads: List[torch.Tensor], loss: torch.Tensor) -> None:
        """The tail of the middle: the towers' MLP gradients, the flat
        small-table gradient and the loss packed into one bucket, one
        all_reduce of it (world 1: no bucket, the gradients are used in
        place), then tt_dense_adagrad_many on both towers' MLP buffers and the
        flat small-table buffer, and the loss into its static scalar — fixed
        shapes, captured into the step's hipGraph."""
        m = self.model
        if not self.exchange:
            grads, small, loss_out = [g.view_as(t.dense.flat) for g, t in zip(flat_grads, m.towers)], \
                self._small_grad, loss.reshape(())
        else:
            torch.cat([g.reshape(-1) for g in flat_grads] + [self._small_grad, loss.reshape(1)], out=self._bucket)
            _all_reduce_sum(self._bucket, self.group, self.always)
            grads, off = [], 0
            for t in m.towers:
                n = t.dense.flat.numel()
                grads.append(self._bucket[off:off + n].view_as(t.dense.flat))
                off += n
            small = self._bucket[off:off + self._small_grad.numel()]
            loss_out = self._bucket[off + self._small_grad.numel()]
        jobs = [(t.dense.flat.data, self._dense_acc[ti], g) for ti, (t, g) in enumerate(zip(m.towers, grads))]
        if self.small:
            jobs.append((self._small_flat, self._small_acc, small))
        if self.ops.dense_adagrad_many is not None:  # one launch for every buffer
            self.ops.dense_adagrad_many(jobs, self.lr, self.eps)
        else:
            for p, a, g in jobs:
                self.ops.dense_adagrad(p, a, g, self.lr, self.eps)
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            # captured: the graph's own loss scalar (its pool address is fixed
            # and every replay rewrites it) is the step's loss — no 4-byte copy
            # node in the graph (~5 us of a memcpy node per step)
            self._loss_graph = loss_out
        else:
            self._loss.copy_(loss_out)

    # -- one step ----------------------------------------------------------
    def _body(self) -> None:
        """Route, fetch, middle, owner apply on the static batch: fixed shapes
        and no host sync, so the whole of it is captured as one graph."""
        rt = None
        self._route_side = None
        self._presorted = False
        if self.tables is not None:
            lookups = [(k, ids) for k, ids, _, _ in self._lookups(self._static)]
            idx_out = self._idx_all[:len(self._idx)]
            if not self.exchange and idx_out.is_cuda and ROUTE_SIDE:
                # one rank: the route has no collective and the middle reads the
                # shard by id, so the route only feeds the backward's per-request
                # sums and the owner apply — it runs on a side stream beside the
                # forward, joined (from the origin stream) before the sums
                main = torch.cuda.current_stream()
                if getattr(self, "_side", None) is None:
                    self._side = torch.cuda.Stream(device=idx_out.device)
                self._side.wait_stream(main)
                with torch.cuda.stream(self._side):
                    rt = self.tables.route_fixed(lookups, self._cap, overflow=self._overflow, idx_out=idx_out)
                    # ... and the sums' key sort, which reads only the slots and ids
                    if self.ops.scatter_sort is not None and self._scatter_specs():
                        self.ops.scatter_sort([sp for sp, _ in self._scatter_specs()], self._B)
                        self._presorted = True
                self._route_side = (self._side, rt)
            else:
                rt = self.tables.route_fixed(lookups, self._cap, overflow=self._overflow, idx_out=idx_out)
                self._route_joined(rt)
                if self.exchange:
                    self.tables.fetch_routed(rt, out=self._got)  # rt.idx_all IS self._idx_all[:L]
        self._middle()
        if rt is not None:
            self.tables.apply_routed(rt, self._g_req, self.lr, self.eps)

    def _join_route(self) -> None:
        """Join the side-stream route (world 1) before its outputs are read."""
        if getattr(self, "_route_side", None) is None:
            return
        side, rt = self._route_side
        self._route_side = None
        main = torch.cuda.current_stream()
        main.wait_stream(side)
        for t in (rt.tags, rt.rows, rt.counts, *rt.table_ids):
            t.record_stream(main)
        self._route_joined(rt)

    def _route_joined(self, rt: _Route) -> None:
        if os.environ.get("TT_SHARDED_DEBUG") == "2":  # the per-owner counts, for the status report
            self._last_counts = rt.counts
        if os.environ.get("TT_SHARDED_DEBUG") == "2":  # running max of the per-owner counts, in the graph
            if getattr(self, "_cmax", None) is None:
                self._cmax = torch.zeros(1, dtype=torch.int64, device=rt.counts.device)
            torch.maximum(self._cmax, rt.counts.max().reshape(1), out=self._cmax)

    def prefetch(self, batch) -> None:
        """Kept for API compatibility: routing runs inside the step's graph."""

    def __call__(self, batch: Dict[str, Any], next_batch: Optional[Dict[str, Any]] = None,
                 ahead: Optional[Sequence[Dict[str, Any]]] = None) -> Dict[str, torch.Tensor]:
        """One step on `batch` (next_batch / ahead: accepted for API
        compatibility and ignored — routing is part of the step's graph)."""
        tm = time.perf_counter()
        if self._static is None:
            self._setup(batch)
        self._load(batch)
        tm = self._tick("load", tm)
        if self._graph is None and self.use_graph and self._calls >= 1 and self.model.device.type == "cuda":
            from pkg.modelling import hip_ops

            try:
                g = torch.cuda.CUDAGraph()
                # thread_local: the process group's watchdog thread polls its
                # events during the capture; in the default global mode that
                # poll invalidates the capture and the watchdog aborts the process
                self._graph_events: list = []  # held for the graph's lifetime
                with hip_ops.capture_guard(self._graph_events), torch.cuda.graph(
                        g, capture_error_mode="thread_local"):
                    self._body()
                self._graph = g
                hip_ops.Workspace.snapshot(owner=g)  # its workspaces live as long as the graph
            except Exception as e:  # keep training eagerly (still the HIP kernels)
                logger.warning(f"ShardedTrainStep: graph capture failed ({e!r}); running eagerly")
                self.use_graph = False
        if self._graph is not None:
            self._graph.replay()
        else:
            self._body()
        self._calls += 1
        tm = self._tick("step", tm)
        if os.environ.get("TT_SHARDED_DEBUG") == "1" and self.tables is not None:
            torch.cuda.synchronize()
            c = self._canary.tolist()
            counts = self._last_counts.tolist() if getattr(self, "_last_counts", None) is not None else [0]
            if c[0] != 0x7EADBEEF or c[2] != 0x7EADBEEF or c[1] != 0 or max(counts) > self._cap:
                raise RuntimeError(f"ShardedTrainStep debug: call {self._calls}, canary/overflow {c}, counts {counts}, "
                                   f"cap {self._cap}, graph {self._graph is not None}")
        loss = self._loss_graph if self._graph is not None and getattr(self, "_loss_graph", None) is not None \
            else self._loss
        return {"loss": loss.clone()}

    # workspaces the sharded step's sparse kernels write (EmbeddingOps.hip)
    STATUS_TAGS = ("sparse_owner", "sparse_mid")

    def check_status(self) -> None:
        """Raise if a shard's owner apply or per-request scatter sum since the
        last check refused keys that were not its call's (tt_sparse_status on
        the "sparse_owner" / "sparse_mid" workspaces, every scope); one stream
        sync.  Call it once per epoch, like TwoTowerModel.fit does (the
        reference's legacy apply raises, optimizer_factory.py:15-18)."""
        if self.model.device.type == "cuda":
            from pkg.modelling import hip_ops

            hip_ops.sparse_status_all(self.model.device, self.STATUS_TAGS)
        ov = getattr(self, "_overflow", None)
        if os.environ.get("TT_SHARDED_DEBUG") == "2" and ov is not None:
            torch.cuda.synchronize()
            logger.warning(f"ShardedTrainStep debug: canary/overflow {self._canary.tolist()}, max owner count "
                           f"{int(self._cmax.item())} (cap {self._cap}), last counts {self._last_counts.tolist()}")
        if ov is not None:
            n = int(ov.item())
            ov.zero_()
            if n:
                raise RuntimeError(f"ShardedTrainStep: {n} row requests overflowed route_capacity={self._cap} "
                                   "and were dropped (use the default capacity for exact steps)")
