"""IndexRecall (mirror of /root/reference/pkg/modelling/metrics/index_recall.py:10-84).

hits[k] += #(true id == any of the first k candidates) per row (every equal
position counts, like the reference's reduce_sum of equal()), seen += rows,
recall@k = hits/seen as float64.  With integer identifiers on the GPU the
count runs in one libtt launch (tt_recall_hits) and stays on the device until
read; string identifiers are compared on the host.
"""
from __future__ import annotations

import logging
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from pkg.modelling import hip_ops

logger = logging.getLogger(__name__)

__all__ = ["IndexRecall"]


class IndexRecall:
    """
    Given an index, calculate a recall@K metric.

    Parameters
    ----------
    index: BruteForceIndex | StaticIndex | callable
        Maps a query feature dict to [B, K] candidate identifiers.
    ks: List[int]
        The top Ks to calculate recall at.
    """

    def __init__(self, index, ks: List[int]):
        self.index = index
        self.ks = list(ks)
        self._host_hits = {k: 0 for k in self.ks}
        self._dev_hits: Optional[torch.Tensor] = None
        self.seen = 0

    def _update(self, true_ids, candidates) -> None:
        if (isinstance(candidates, torch.Tensor) and candidates.device.type == "cuda"
                and candidates.dtype in (torch.int32, torch.int64)):
            t = torch.as_tensor(true_ids).reshape(-1).to(candidates.device, torch.int32).contiguous()
            c = candidates.to(torch.int32).contiguous()
            if self._dev_hits is None:
                self._dev_hits = torch.zeros(len(self.ks), dtype=torch.int64, device=c.device)
            hip_ops.recall_hits(t, c, self.ks, self._dev_hits)
        else:
            c = candidates.cpu().numpy() if isinstance(candidates, torch.Tensor) else np.asarray(candidates)
            t = true_ids.cpu().numpy() if isinstance(true_ids, torch.Tensor) else np.asarray(true_ids, dtype=object)
            t = np.array([x.decode() if isinstance(x, bytes) else x for x in t.reshape(-1)], dtype=object)
            c = np.array([[x.decode() if isinstance(x, bytes) else x for x in row] for row in c], dtype=object)
            eq = t.reshape(-1, 1) == c
            for k in self.ks:
                self._host_hits[k] += int(eq[:, :k].sum())

    def __call__(self, queries: Dict[str, Any], true_candidate_ids) -> Dict[int, np.float64]:
        candidates = self.index(queries)
        n = true_candidate_ids.shape[0] if hasattr(true_candidate_ids, "shape") else len(true_candidate_ids)
        self.seen += int(n)
        self._update(true_candidate_ids, candidates)
        return self.metric

    @property
    def hits(self) -> Dict[int, int]:
        out = dict(self._host_hits)
        if self._dev_hits is not None:
            for k, v in zip(self.ks, self._dev_hits.cpu().tolist()):
                out[k] += int(v)
        return out

    @property
    def metric(self) -> Dict[int, np.float64]:
        h = self.hits
        return {k: np.float64(h[k]) / np.float64(self.seen) if self.seen else np.float64(0.0) for k in self.ks}

    def log_metric(self, epoch: Optional[int] = None, to_tensorboard: bool = True) -> None:
        m = self.metric
        for k in self.ks:
            logger.info(f"Start of epoch {epoch} recall@{k}: {m[k]}")
