from enum import Enum
import logging
from typing import Dict, List, Optional, Sequence

import numpy as np
import pandas as pd

from pkg import dtypes

logger = logging.getLogger(__name__)


class FeatureFamily(Enum):
    """
    The families which features can be part of
    (reference: pkg/schema/features.py:11-18).
    """

    QUERY = "query"
    CANDIDATE = "candidate"


class Feature:
    """
    All of the information for an input feature
    (reference: pkg/schema/features.py:21-127; same arguments and checks).

    Parameters
    ----------
    name: str
        Name of the feature.
    dtype: pkg.dtypes.DType
        ``pkg.dtypes.string`` (categorical, embedded) or ``pkg.dtypes.float32``
        (numeric pass-through).  Strings such as "string" / "tf.string" are
        accepted too.
    feature_family: FeatureFamily
        QUERY or CANDIDATE.
    embedding_size: Optional[int]
        For categorical features, the embedding dimension.
    vocab: Optional[List[str]]
        For categorical features, the values the feature can take.  Unseen
        values map to the OOV row 0.
    max_vocab_size: Optional[int]
        Max size of a vocab built from data (ignored if vocab is given).

    The id -> row mapping is the reference's StringLookup(num_oov_indices=1)
    (input_layer.py:33-36): vocab[i] -> row i+1, anything else -> row 0.
    """

    VALID_DTYPES = [dtypes.string, dtypes.float32]

    def __init__(
        self,
        name: str,
        dtype,
        feature_family: FeatureFamily,
        embedding_size: Optional[int] = None,
        vocab: Optional[List[str]] = None,
        max_vocab_size: Optional[int] = None,
    ):
        self.name = name
        try:
            dtype = dtypes.as_dtype(dtype)
        except TypeError:
            raise TypeError(f"dtype must be one of {self.VALID_DTYPES}, got {dtype}") from None
        if dtype not in self.VALID_DTYPES:
            raise TypeError(f"dtype must be one of {self.VALID_DTYPES}, got {dtype}")
        self.dtype = dtype

        if not isinstance(feature_family, FeatureFamily):
            raise ValueError(
                f"feature_family {feature_family} not valid. "
                f"Must be one of {FeatureFamily._member_names_}"
            )
        self.feature_family = feature_family

        if embedding_size:
            if dtype != dtypes.string:
                raise TypeError(f"Got embedding size, dtype must be tf.string got {dtype}")
        self.embedding_size = embedding_size
        self._lookup: Optional[Dict[str, int]] = None
        self._native = None
        self._init_vocab(vocab)

        if max_vocab_size:
            if not isinstance(max_vocab_size, int):
                raise TypeError(f"max_vocab_size must be an int, got {max_vocab_size}")
        self.max_vocab_size = max_vocab_size

    def _init_vocab(self, vocab: Optional[List[str]] = None) -> None:
        """Check the dtype and init the vocab (features.py:83-104)."""
        if self.dtype != dtypes.string:
            logger.info(f"Ignoring vocab passed for non-string feature {self.name}")
            self.vocab = None
            self.is_built = True
        else:
            if vocab:
                # The reference stores a set (unordered rows); keep the
                # de-duplicated insertion order so rows are reproducible.
                self.vocab = np.array([str(v) for v in dict.fromkeys(vocab)])
                self.is_built = True
            else:
                self.vocab = None
                self.is_built = False
        self._lookup = None
        self._native = None

    def set_vocab_from_dataframe(self, df: pd.DataFrame) -> None:
        """
        Set the vocabulary from a DataFrame (features.py:106-127):
        value_counts() order, optional head(max_vocab_size), str().
        """
        if self.name not in df.columns:
            raise ValueError(f"Feature name {self.name} not found in df cols {df.columns}")
        v_counts = df[self.name].value_counts()
        if self.max_vocab_size:
            vocab = list(v_counts.head(self.max_vocab_size).index)
        else:
            vocab = list(v_counts.index)
        self.vocab = np.array([str(x) for x in vocab])
        self.is_built = True
        self._lookup = None
        self._native = None

    # ---- id encoding (StringLookup) -------------------------------------
    @property
    def num_rows(self) -> int:
        """Embedding table rows: len(vocab) + 1 for the OOV row."""
        if self.vocab is None:
            raise ValueError(f"feature {self.name} has no vocab")
        return len(self.vocab) + 1

    def lookup_table(self) -> Dict[str, int]:
        if self._lookup is None:
            if self.vocab is None:
                raise ValueError(f"feature {self.name} has no vocab")
            self._lookup = {v: i + 1 for i, v in enumerate(self.vocab)}
        return self._lookup

    def encode(self, values: Sequence, num_threads: int = 0) -> np.ndarray:
        """Strings (or anything str()-able) -> int32 rows; OOV -> 0.  Runs in
        libtt's multi-threaded host hash lookup (pkg.schema.vocab), built once
        per vocabulary."""
        if self.vocab is None:
            raise ValueError(f"feature {self.name} has no vocab")
        if self._native is None:
            from pkg.schema.vocab import NativeVocab

            self._native = NativeVocab(self.vocab)
        return self._native.encode(values, num_threads)

    def __getstate__(self):
        state = dict(self.__dict__)
        state["_lookup"] = None
        state["_native"] = None
        return state

    def __setstate__(self, state):
        state.setdefault("_native", None)
        self.__dict__.update(state)

    def __repr__(self) -> str:
        return (f"Feature({self.name!r}, {self.dtype}, {self.feature_family}, "
                f"embedding_size={self.embedding_size})")
