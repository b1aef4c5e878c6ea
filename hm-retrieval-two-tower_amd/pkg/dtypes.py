"""Dtype tokens replacing ``tf.string`` / ``tf.float32`` in the Schema API.

The reference's Feature takes TensorFlow dtypes (pkg/schema/features.py:43,
55-58).  TensorFlow is not part of this framework, so the same two tokens
are provided here; ``pkg.dtypes.string`` marks a categorical (embedded)
feature and ``pkg.dtypes.float32`` a numeric pass-through feature.
"""
from __future__ import annotations


class DType:
    __slots__ = ("name",)

    def __init__(self, name: str):
        self.name = name

    def __repr__(self) -> str:
        return f"pkg.dtypes.{self.name}"

    def __eq__(self, other) -> bool:
        if isinstance(other, DType):
            return self.name == other.name
        if isinstance(other, str):
            return self.name == other
        return NotImplemented

    def __hash__(self) -> int:
        return hash(self.name)

    def __reduce__(self):
        return (_token, (self.name,))


string = DType("string")
float32 = DType("float32")
_TOKENS = {"string": string, "float32": float32}


def _token(name: str) -> DType:
    return _TOKENS[name]


def as_dtype(x) -> DType:
    """Accept a token, its name, or anything whose str() names one ('tf.string')."""
    if isinstance(x, DType):
        return x
    s = str(x).split(".")[-1].strip("<>'\" ")
    if s.startswith("dtype: "):
        s = s[len("dtype: "):]
    if s in _TOKENS:
        return _TOKENS[s]
    raise TypeError(f"dtype must be one of {list(_TOKENS.values())}, got {x}")
