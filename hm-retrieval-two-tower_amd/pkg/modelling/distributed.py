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

__all__ = ["IndexOps", "ShardedBruteForceIndex", "DataParallelTrainStep", "shard_range", "all_gather_cat"]


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
