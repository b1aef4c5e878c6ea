"""LogQCorrection (mirror of /root/reference/pkg/modelling/layers/logq_correction.py:5-71).

S'_ij = logits_ij - log p(candidate_j): the column of candidate j is shifted
by its log sampling probability; ids missing from the lookup get p = 1.0
(shift 0), as the reference's StaticHashTable default does.  p is stored as
fp32 and the log taken in fp32 (the TF table's value dtype).

On the training hot path the shift is fused into the in-batch softmax kernel
(tt_inbatch_xent_*): this layer only produces the per-candidate log p vector
it consumes.  __call__ keeps the reference's materialised form for API
parity.
"""
from __future__ import annotations

from typing import Dict, Sequence, Union

import numpy as np
import torch

from pkg.schema.features import Feature

__all__ = ["LogQCorrection"]


class LogQCorrection:
    """
    Apply the LogQ Correction to logits.

    Parameters
    ----------
    candidate_prob_lookup: Dict[str, float]
        A dict mapping candidate ids to probs.
    """

    def __init__(self, candidate_prob_lookup: Dict[str, float]):
        self._init_lookup(candidate_prob_lookup)

    def _init_lookup(self, candidate_prob_lookup: Dict[str, float]) -> None:
        self.lookup = {str(k): np.float32(v) for k, v in candidate_prob_lookup.items()}

    def log_probs(self, candidate_ids: Sequence) -> np.ndarray:
        """log p(id) (fp32) for raw candidate ids; missing -> log(1.0) = 0."""
        flat = np.asarray(candidate_ids, dtype=object).reshape(-1)
        p = np.empty(flat.shape[0], np.float32)
        for i, v in enumerate(flat):
            if isinstance(v, bytes):
                v = v.decode()
            p[i] = self.lookup.get(str(v), np.float32(1.0))
        return np.log(p).astype(np.float32)

    def row_table(self, feature: Feature, device: torch.device) -> torch.Tensor:
        """log p per embedding row of the candidate-id feature: row r >= 1 is
        vocab[r-1], row 0 (OOV) gets 0 (p = 1.0).  Used when a batch carries
        encoded rows instead of raw ids."""
        if feature.vocab is None:
            raise ValueError(f"feature {feature.name} has no vocab")
        table = np.zeros(len(feature.vocab) + 1, np.float32)
        table[1:] = self.log_probs(feature.vocab)
        return torch.as_tensor(table, device=device)

    def __call__(self, logits: torch.Tensor, candidate_ids: Union[Sequence, torch.Tensor]) -> torch.Tensor:
        """logits [B,B] minus log p of each column's candidate (broadcast over rows).
        candidate_ids: raw ids (strings) or a [B] float tensor of log p."""
        if isinstance(candidate_ids, torch.Tensor) and candidate_ids.dtype == torch.float32:
            corr = candidate_ids.reshape(1, -1).to(logits.device)
        else:
            corr = torch.as_tensor(self.log_probs(candidate_ids), device=logits.device).reshape(1, -1)
        return logits - corr
