"""Base class of the models (mirror of
/root/reference/pkg/modelling/models/abstract_keras_model.py:10-131).

The reference attaches a tf.function input signature for SavedModel export;
here the signature documents the expected batch dict (name -> [None, 1]
tensor of a dtype token) and `save` writes a weights-only torch checkpoint.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from dataclasses import dataclass
import logging
import os
from typing import Any, Dict, Tuple

import torch

from pkg import dtypes

logger = logging.getLogger(__name__)


@dataclass(frozen=True)
class TensorSpec:
    shape: Tuple[Any, ...]
    dtype: dtypes.DType
    name: str


class AbstractKerasModel(ABC):
    """Abstract class with the model plumbing shared by towers, the two-tower
    model and the indices."""

    input_signature: Dict[str, TensorSpec] = None

    @abstractmethod
    def get_input_signature(self) -> Dict[str, TensorSpec]:
        """Dict mapping input names to TensorSpec."""

    def set_input_signature(self, input_signature: Dict[str, TensorSpec]) -> None:
        self.input_signature = dict(input_signature)

    @staticmethod
    def _get_default_tensor(dtype) -> Any:
        """Default input per dtype (abstract_keras_model.py:46-68): the OOV
        string b"a" for categorical, 0.0 for numeric."""
        dtype = dtypes.as_dtype(dtype)
        if dtype == dtypes.string:
            return [[b"a"]]
        if dtype == dtypes.float32:
            return torch.zeros(1, 1, dtype=torch.float32)
        raise TypeError(f"Invalid dtype {dtype}")

    def get_default_inputs(self, input_signature: Dict[str, TensorSpec]) -> Dict[str, Any]:
        return {f: self._get_default_tensor(spec.dtype) for f, spec in input_signature.items()}

    @abstractmethod
    def call(self, x: Dict[str, Any], training: bool = True):
        """Pass data through the model."""

    def __call__(self, x: Dict[str, Any], training: bool = False):
        return self.call(x, training=training)

    def initialise_model(self) -> None:
        """Record the input signature (abstract_keras_model.py:109-118).  The
        reference also traces a dummy call; here construction stays host-only
        so models can be configured on machines without a GPU."""
        self.set_input_signature(self.get_input_signature())

    def state_dict(self) -> Dict[str, Any]:  # pragma: no cover - overridden
        return {}

    def save(self, model_path: str) -> None:
        """Save a weights-only checkpoint (loadable with torch.load(weights_only=True))."""
        d = os.path.dirname(model_path)
        if d:
            os.makedirs(d, exist_ok=True)
        logging.info(f"Saving model at path: {model_path}")
        torch.save(self.state_dict(), model_path if model_path.endswith(".pt") else model_path + ".pt")
