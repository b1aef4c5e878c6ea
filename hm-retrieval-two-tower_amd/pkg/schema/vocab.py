"""Native StringLookup for the input pipeline.

The reference looks every batch's strings up inside the graph with
tf.keras.layers.StringLookup(vocabulary=vocab, num_oov_indices=1)
(/root/reference/pkg/modelling/layers/input_layer.py:33-36).  Here a dataset
is encoded once on the host by libtt's multi-threaded hash lookup
(tt_vocab_create / tt_vocab_encode, csrc/tt_vocab.cpp) over an Arrow string
arena, so no Python object is touched per value; the int32 rows then stay in
HBM (pkg.modelling.dataset.DeviceDataset).

Values are compared as their str() text, as the reference's tf.string
features see them: str / bytes (UTF-8) / integer arrays go to the arena
directly (Arrow's integer -> string cast is Python's str()); anything else
(floats, bools, mixed objects) is converted with str() first.
"""
from __future__ import annotations

import ctypes
from typing import Sequence, Tuple

import numpy as np
import pyarrow as pa

from pkg import _native

__all__ = ["NativeVocab", "string_arena"]


def _arrow_strings(values) -> pa.Array:
    if isinstance(values, pa.ChunkedArray):
        values = values.combine_chunks()
    if isinstance(values, pa.Array):
        arr = values
    else:
        if hasattr(values, "to_numpy") and not isinstance(values, np.ndarray):
            values = values.to_numpy()  # pandas Series / Index
        # Python sequences keep each element's own type (str(True) is "True",
        # not numpy's coerced "1.0")
        a = np.asarray(values, dtype=object) if isinstance(values, (list, tuple)) else np.asarray(values)
        a = a.reshape(-1)
        if a.dtype.kind in "US":
            arr = pa.array(a)
        elif a.dtype.kind in "iu":
            arr = pa.array(a).cast(pa.string())
        elif a.dtype.kind == "O":
            try:  # object arrays of str / bytes convert without a Python loop
                arr = pa.array(a, from_pandas=False)
            except (pa.ArrowInvalid, pa.ArrowTypeError):
                arr = None
            if arr is None or arr.null_count or not (
                    pa.types.is_string(arr.type) or pa.types.is_large_string(arr.type)
                    or pa.types.is_binary(arr.type) or pa.types.is_large_binary(arr.type)):
                # per element str(): None -> "None", as a str()-cast column reads
                arr = pa.array([v.decode() if isinstance(v, bytes) else str(v) for v in a.tolist()],
                               type=pa.large_string())
        else:
            # floats / bools / other numpy scalars: str() of the numpy scalar
            # itself (str(np.float32(0.1)) is "0.1"; tolist() would widen it)
            arr = pa.array([str(v) for v in a], type=pa.large_string())
    if isinstance(arr, pa.ChunkedArray):
        arr = arr.combine_chunks()
    if pa.types.is_integer(arr.type):
        arr = arr.cast(pa.string())
    if arr.null_count:
        raise ValueError("null values cannot be looked up (StringLookup takes strings)")
    if pa.types.is_string(arr.type):
        arr = arr.cast(pa.large_string())
    elif pa.types.is_binary(arr.type):
        arr = arr.cast(pa.large_binary())
    elif not (pa.types.is_large_string(arr.type) or pa.types.is_large_binary(arr.type)):
        raise TypeError(f"cannot look up values of type {arr.type}")
    return arr.combine_chunks() if isinstance(arr, pa.ChunkedArray) else arr


def string_arena(values) -> Tuple[np.ndarray, np.ndarray, int, pa.Array]:
    """(data uint8, offsets int64 [n+1], n, owner) of an Arrow large-string
    view of `values`; `owner` keeps the buffers alive."""
    arr = _arrow_strings(values)
    n = len(arr)
    bufs = arr.buffers()
    off = np.frombuffer(bufs[1], dtype=np.int64, count=n + 1 + arr.offset)[arr.offset:]
    data = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None and bufs[2].size else np.zeros(1, np.uint8)
    return data, off, n, arr


def _ptr(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


class NativeVocab:
    """vocab[i] -> row i + 1, anything else -> 0 (libtt host hash table)."""

    def __init__(self, vocab: Sequence):
        data, off, n, self._owner = string_arena(vocab)
        h = ctypes.c_void_p()
        _native.check(_native.lib().tt_vocab_create(_ptr(data), _ptr(off), n, ctypes.byref(h)))
        self._handle = h
        self.size = int(_native.lib().tt_vocab_size(h))
        del self._owner  # the library copied the arena

    def encode(self, values, num_threads: int = 0) -> np.ndarray:
        data, off, n, owner = string_arena(values)
        out = np.empty(n, dtype=np.int32)
        if n:
            _native.check(_native.lib().tt_vocab_encode(self._handle, _ptr(data), _ptr(off), n, _ptr(out),
                                                        int(num_threads)))
        del owner
        return out

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            try:
                _native.lib().tt_vocab_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self._handle = None
