"""StaticIndex (mirror of /root/reference/pkg/modelling/indices/static_index.py:9-95):
the same ordered candidates for every query row (popularity baseline)."""
from __future__ import annotations

from typing import Any, Dict, List, Sequence

import numpy as np
import pandas as pd
import torch

from pkg.schema.features import Feature
from pkg.schema.schema import Schema
from pkg.modelling.models.abstract_keras_model import AbstractKerasModel, TensorSpec

__all__ = ["StaticIndex"]


class StaticIndex(AbstractKerasModel):
    """
    Return a fixed set of candidates in order.

    Parameters
    ----------
    k: int
        The number of candidates to return.
    input_features: List[Feature]
        Input features (only used for the batch size / signature).
    candidates: Sequence or [1, N] array / tensor
        Ordered candidate ids to return.
    """

    def __init__(self, k: int, input_features: List[Feature], candidates):
        self.k = int(k)
        self.input_features = input_features
        if isinstance(candidates, torch.Tensor):
            self.candidates = candidates.reshape(1, -1)
        else:
            self.candidates = np.asarray(candidates).reshape(1, -1)
        self.initialise_model()

    def call(self, x: Dict[str, Any], training: bool = False):
        v = x[self.input_features[0].name]
        n = v.shape[0] if hasattr(v, "shape") else len(v)
        top = self.candidates[:, : self.k]
        if isinstance(top, torch.Tensor):
            return top.expand(n, -1)
        return np.tile(top, (n, 1))

    def get_input_signature(self) -> Dict[str, TensorSpec]:
        return {f.name: TensorSpec((None, 1), f.dtype, f.name) for f in self.input_features}

    @classmethod
    def build_popularity_index_from_series_schema(cls, schema: Schema, s: pd.Series) -> "StaticIndex":
        """Candidates ordered by popularity (value_counts) (static_index.py:67-95)."""
        ids = s.value_counts().index
        return cls(k=max(schema.model_config.ks), input_features=schema.query_features,
                   candidates=np.array([str(i) for i in ids]).reshape(1, -1))
