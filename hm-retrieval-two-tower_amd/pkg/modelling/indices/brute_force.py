"""BruteForceIndex (mirror of /root/reference/pkg/modelling/indices/brute_force.py:6-114).

The candidate matrix [N, E] (fp32, as computed by the candidate tower) is
prepared once into a bf16 screening image (tt_bruteforce_build).  call()
embeds the queries with the query tower and runs tt_bruteforce_search: bf16
MFMA scoring with a fused, certified top-k screen and an exact fp32 rescoring
of the shortlist, so the returned indices equal tf.math.top_k over the fp32
scores (ties -> lower index) and the scores are the fp32 values.
"""
from __future__ import annotations

from typing import Any, Dict, Iterable, Optional, Tuple

import numpy as np
import torch

from pkg.modelling import hip_ops
from pkg.modelling.device import default_device
from pkg.modelling.models.abstract_keras_model import AbstractKerasModel, TensorSpec

__all__ = ["BruteForceIndex"]


def _as_identifiers(ids) -> Any:
    if isinstance(ids, torch.Tensor):
        return ids.reshape(-1)
    arr = np.asarray(ids).reshape(-1)
    return arr


class BruteForceIndex(AbstractKerasModel):
    """
    Store ids and embeddings for candidates; at inference return the top k ids
    for each query.

    Parameters
    ----------
    k: int
        The number of results the index should return.
    query_model: callable
        Maps a query feature dict to [B, E] embeddings (e.g. a Tower).
    id_candidate_pairs: iterable of (ids [n], embeddings [n, E])
        Batches of candidate identifiers and their embeddings.
    """

    def __init__(self, k: int, query_model, id_candidate_pairs: Iterable[Tuple[Any, Any]],
                 device: Optional[torch.device] = None):
        self.k = int(k)
        self.query_model = query_model
        self.device = device if device is not None else getattr(query_model, "device", None) or default_device()
        self._index(id_candidate_pairs)
        self.initialise_model()

    def _index(self, id_candidate_pairs) -> None:
        identifiers, candidates = self.get_id_embeddings_from_dataset(id_candidate_pairs)
        self._identifiers = identifiers
        self._candidates = candidates.to(self.device, torch.float32).contiguous()
        if self.k > self._candidates.shape[0]:
            raise ValueError(f"k={self.k} exceeds the number of candidates {self._candidates.shape[0]}")
        self._image = hip_ops.bruteforce_build(self._candidates)

    @property
    def num_candidates(self) -> int:
        return self._candidates.shape[0]

    def search(self, query_embeddings: torch.Tensor, k: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """(scores [B,k] fp32, indices [B,k] int32) for query embeddings [B,E]."""
        q = query_embeddings.to(self.device, torch.float32).contiguous()
        return hip_ops.bruteforce_search(self._image, self._candidates, q, k or self.k)

    def lookup_identifiers(self, indices: torch.Tensor):
        if isinstance(self._identifiers, torch.Tensor):
            ident = self._identifiers.to(indices.device)
            return ident.index_select(0, indices.reshape(-1).long()).reshape(indices.shape)
        return self._identifiers[indices.cpu().numpy()]

    def call(self, queries: Dict[str, Any], training: bool = False):
        """Top-k candidate identifiers [B, k] for a query feature dict (brute_force.py:54-83)."""
        with torch.no_grad():
            emb = self.query_model(queries)
        _, idx = self.search(emb)
        return self.lookup_identifiers(idx)

    @staticmethod
    def get_id_embeddings_from_dataset(candidates) -> Tuple[Any, torch.Tensor]:
        """Concatenate (ids, embeddings) batches (brute_force.py:85-106)."""
        ids_list, emb_list = [], []
        for ids, emb in candidates:
            ids_list.append(ids)
            emb_list.append(emb if isinstance(emb, torch.Tensor) else torch.as_tensor(np.asarray(emb, np.float32)))
        emb = torch.cat([e.reshape(-1, e.shape[-1]) for e in emb_list], 0)
        if all(isinstance(i, torch.Tensor) for i in ids_list):
            ids = torch.cat([i.reshape(-1) for i in ids_list], 0)
        else:
            ids = np.concatenate([np.asarray(i.cpu().numpy() if isinstance(i, torch.Tensor) else i).reshape(-1)
                                  for i in ids_list])
        return ids, emb

    def get_input_signature(self) -> Dict[str, TensorSpec]:
        sig = getattr(self.query_model, "get_input_signature", None)
        return sig() if sig else {}

    def state_dict(self) -> Dict[str, Any]:
        ident = self._identifiers
        return {
            "k": torch.tensor(self.k),
            "candidates": self._candidates.detach().cpu(),
            "identifiers": ident.cpu() if isinstance(ident, torch.Tensor)
            else torch.as_tensor(np.arange(len(ident))),
        }

    def save(self, model_path: str) -> None:
        """Candidates, identifiers, k and the query tower (pkg.modelling.export):
        a loaded index answers raw queries on its own (brute_force.py:108-114)."""
        from pkg.modelling import export

        export.save_index(self, model_path[:-3] if model_path.endswith(".pt") else model_path)

    @classmethod
    def load(cls, model_path: str, device: Optional[torch.device] = None) -> "BruteForceIndex":
        from pkg.modelling import export

        return export.load_index(model_path[:-3] if model_path.endswith(".pt") else model_path, device)
