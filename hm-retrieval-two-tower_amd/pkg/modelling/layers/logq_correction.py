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
        self._keys = None

    def log_probs(self, candidate_ids: Sequence) -> np.ndarray:
        """log p(id) (fp32) for raw candidate ids; missing -> log(1.0) = 0.
        The id lookup is libtt's host hash table (pkg.schema.vocab)."""
        from pkg.schema.vocab import NativeVocab

        if self._keys is None:
            self._keys = NativeVocab(list(self.lookup.keys()))
            self._probs = np.concatenate([[np.float32(1.0)], np.asarray(list(self.lookup.values()), np.float32)])
        return np.log(self._probs[self._keys.encode(candidate_ids)]).astype(np.float32)

    def row_table(self, feature: Feature, device: torch.device) -> torch.Tensor:
        """log p per embedding row of the candidate-id feature: row r >= 1 is
        vocab[r-1], row 0 (OOV) gets 0 (p = 1.0).  Used when a batch carries
        encoded rows instead of raw ids.

        Precondition: every id of the probability lookup is in the vocab.  An
        id outside it encodes to the shared OOV row, whose log p is not
        recoverable from the row; the reference (which looks the raw id up)
        would subtract its log p.  Such batches must carry the exact
        per-example column "__logq__" (encode_dataframe(..., logq=...))."""
        if feature.vocab is None:
            raise ValueError(f"feature {feature.name} has no vocab")
        rows = feature.encode(np.asarray(list(self.lookup.keys()), dtype=str)) if self.lookup else np.zeros(0)
        if np.any(rows == 0):
            missing = [k for k, r in zip(self.lookup.keys(), rows.tolist()) if r == 0][:3]
            raise ValueError(
                f"candidate_prob_lookup has ids outside the {feature.name} vocab (e.g. {missing}); their log p "
                "cannot be recovered from encoded rows — encode the batches with their '__logq__' column "
                "(pkg.modelling.dataset.encode_dataframe(..., logq=...))")
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
