"""ctypes binding of libtt.so, the gfx950 C ABI declared in include/tt.h.

The library is built in-tree (``make -C hm-retrieval-two-tower_amd/csrc``) and
loaded from this directory.  There is no fallback: if the library is missing
or cannot be loaded, :func:`lib` raises, and every op that needs it fails
loudly.
"""
from __future__ import annotations

import ctypes
import os
import threading
from ctypes import POINTER, c_char_p, c_float, c_int32, c_int64, c_size_t, c_void_p

__all__ = [
    "LIB_PATH",
    "TTError",
    "GatherSegment",
    "GatherCall",
    "RowTable",
    "SparseTable",
    "RouteLookup",
    "MlpPackJob",
    "MlpRowsProblem",
    "MlpWgradProblem",
    "MAX_SEGMENTS",
    "MAX_SOURCES",
    "lib",
    "check",
    "EXPORTED_SYMBOLS",
]

# TT_LIB_PATH: a variant build for timing tools (tools/index_variants.sh); the
# package default is the in-tree libtt.so
LIB_PATH = os.environ.get("TT_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libtt.so")
MAX_SEGMENTS = 32
MAX_SOURCES = 4

TT_OK = 0
TT_ERR_BAD_ARG = 1
TT_ERR_HIP = 2
TT_ERR_UNSUPPORTED = 3
TT_ERR_WORKSPACE = 4


class TTError(RuntimeError):
    """A libtt entry point returned a non-zero status."""

    def __init__(self, code: int, message: str):
        super().__init__(f"libtt error {code}: {message}")
        self.code = code


class GatherSegment(ctypes.Structure):
    _fields_ = [
        ("table", c_void_p),
        ("ids", c_void_p),
        ("num_rows", c_int64),
        ("dim", c_int32),
        ("col_offset", c_int32),
    ]


class GatherCall(ctypes.Structure):
    _fields_ = [
        ("segs", c_void_p),
        ("num_segs", c_int32),
        ("out", c_void_p),
        ("out_stride", c_int64),
    ]


class RowTable(ctypes.Structure):
    _fields_ = [
        ("table", c_void_p),
        ("num_rows", c_int64),
    ]


class RouteLookup(ctypes.Structure):
    _fields_ = [
        ("ids", c_void_p),
        ("num_rows", c_int64),
        ("tag", c_int32),
    ]


class MlpPackJob(ctypes.Structure):
    _fields_ = [
        ("w", c_void_p),
        ("ldw", c_int64),
        ("K", c_int32),
        ("N", c_int32),
        ("trans", c_int32),
        ("img", c_void_p),
        ("img_bytes", c_size_t),
    ]


class MlpRowsProblem(ctypes.Structure):
    _fields_ = [
        ("A", c_void_p),
        ("lda", c_int64),
        ("amask", c_void_p),
        ("ldam", c_int64),
        ("scale", c_void_p),
        ("M", c_int64),
        ("K", c_int32),
        ("img", c_void_p),
        ("N", c_int32),
        ("bias", c_void_p),
        ("relu", c_int32),
        ("cmask", c_void_p),
        ("ldcm", c_int64),
        ("C", c_void_p),
        ("ldc", c_int64),
    ]


class MlpWgradProblem(ctypes.Structure):
    _fields_ = [
        ("A", c_void_p),
        ("lda", c_int64),
        ("G", c_void_p),
        ("ldg", c_int64),
        ("gmask", c_void_p),
        ("ldgm", c_int64),
        ("scale", c_void_p),
        ("M", c_int64),
        ("Ka", c_int32),
        ("N", c_int32),
        ("dwb", c_void_p),
    ]


class SparseTable(ctypes.Structure):
    _fields_ = [
        ("table", c_void_p),
        ("slot0", c_void_p),
        ("slot1", c_void_p),
        ("num_rows", c_int64),
        ("dim", c_int32),
        ("num_sources", c_int32),
        ("ids", c_void_p * MAX_SOURCES),
        ("grad_col_offset", c_int32 * MAX_SOURCES),
        ("grad", c_void_p),      # optional per-table gradient (NULL: the call's)
        ("grad_ld", c_int64),
    ]


class DenseJob(ctypes.Structure):
    _fields_ = [
        ("param", c_void_p),
        ("accum", c_void_p),
        ("grad", c_void_p),
        ("n", c_int64),
    ]


ROUTE_MAX_LOOKUPS = 32  # TT_ROUTE_MAX_LOOKUPS


class RouteSorted(ctypes.Structure):
    _fields_ = [
        ("order", c_void_p),
        ("grp_first", c_void_p),
        ("grp_last", c_void_p),
        ("slot", c_void_p),
        ("slot_row", c_void_p),
        ("cap", c_int64),
        ("world", c_int32),
        ("num_tags", c_int32),
        ("num_lookups", c_int32),
        ("lookup_tag", c_int32 * ROUTE_MAX_LOOKUPS),
        ("lookup_table", c_int32 * ROUTE_MAX_LOOKUPS),
        ("lookup_source", c_int32 * ROUTE_MAX_LOOKUPS),
    ]


# name -> (restype, argtypes); mirrors include/tt.h one to one.
_PROTOS = {
    "tt_version": (c_char_p, []),
    "tt_last_error": (c_char_p, []),
    "tt_probe_arm": (c_int32, [c_int32, c_void_p, c_void_p]),
    "tt_probe_arm_repeat": (c_int32, [c_int32, c_void_p, c_void_p, c_int32]),
    "tt_gather_grouped": (c_int32, [POINTER(GatherSegment), c_int32, c_int64, c_void_p, c_int64, c_void_p]),
    "tt_gather_multi": (c_int32, [POINTER(GatherCall), c_int32, c_int64, c_void_p]),
    "tt_gather_multi_pack": (c_int32, [POINTER(GatherCall), c_int32, c_int64, c_void_p, c_int32, c_void_p]),
    "tt_gather_tagged": (c_int32, [POINTER(RowTable), c_int32, c_int32, c_void_p, c_void_p, c_int64, c_void_p, c_int64,
                                   c_void_p]),
    "tt_sparse_workspace_size": (c_size_t, [POINTER(SparseTable), c_int32, c_int64]),
    "tt_sparse_adagrad": (
        c_int32,
        [POINTER(SparseTable), c_int32, c_int64, c_void_p, c_int64, c_float, c_float, c_void_p, c_size_t, c_void_p],
    ),
    "tt_sparse_adam": (
        c_int32,
        [POINTER(SparseTable), c_int32, c_int64, c_void_p, c_int64, c_float, c_float, c_float, c_float, c_int64,
         c_void_p, c_size_t, c_void_p],
    ),
    "tt_sparse_scatter_sum_sorted": (
        c_int32, [POINTER(SparseTable), c_int32, c_int64, c_void_p, c_int64, c_void_p, c_size_t, c_void_p]),
    "tt_sparse_scatter_sum": (
        c_int32, [POINTER(SparseTable), c_int32, c_int64, c_void_p, c_int64, c_void_p, c_size_t, c_void_p]),
    "tt_dedup_workspace_size": (c_size_t, [c_int64, c_int32]),
    "tt_dedup_sum": (
        c_int32,
        [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
         c_void_p],
    ),
    "tt_sparse_sort": (c_int32, [POINTER(SparseTable), c_int32, c_int64, c_void_p, c_size_t, c_void_p]),
    "tt_sparse_adagrad_sorted": (
        c_int32,
        [POINTER(SparseTable), c_int32, c_int64, c_void_p, c_int64, c_float, c_float, c_void_p, c_size_t, c_void_p]),
    "tt_sparse_status": (c_int32, [c_void_p, c_size_t, c_void_p]),
    "tt_route_workspace_size": (c_size_t, [c_int32, c_int64, c_int32, c_int64, c_int32]),
    "tt_route_requests": (
        c_int32,
        [POINTER(RouteLookup), c_int32, c_int64, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_size_t, c_void_p]),
    "tt_route_requests_ordered": (
        c_int32,
        [POINTER(RouteLookup), c_int32, c_int64, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "tt_route_fixed_workspace_size": (c_size_t, [c_int32, c_int64, c_int32, c_int64, c_int32]),
    "tt_route_fixed": (
        c_int32,
        [POINTER(RouteLookup), c_int32, c_int64, c_int32, c_int32, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "tt_sparse_routed": (
        c_int32,
        [POINTER(SparseTable), c_int32, c_int64, c_void_p, c_int64, POINTER(RouteSorted), c_int32, c_float, c_float,
         c_void_p, c_size_t, c_void_p]),
    "tt_route_owner": (c_int32, [c_void_p, c_int64, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "tt_sparse_adagrad_rows": (c_int32, [c_void_p, c_int32, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_float,
                                         c_float, c_void_p]),
    "tt_route_pad": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int64, c_void_p, c_void_p, c_void_p,
                               c_void_p]),
    "tt_sum": (c_int32, [c_void_p, c_int64, c_float, c_void_p, c_void_p]),
    "tt_dense_adagrad": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float, c_void_p]),
    "tt_dense_adagrad_many": (c_int32, [POINTER(DenseJob), c_int32, c_float, c_float, c_void_p]),
    "tt_dense_adam": (
        c_int32,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float, c_float, c_float, c_int64, c_void_p],
    ),
    "tt_inbatch_workspace_size": (c_size_t, [c_int64, c_int64, c_int32]),
    "tt_inbatch_xent_rows": (
        c_int32,
        [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_int64, c_void_p, c_void_p,
         c_void_p, c_void_p, c_size_t, c_void_p],
    ),
    "tt_inbatch_xent_cols": (
        c_int32,
        [c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_int64,
         c_void_p, c_void_p, c_size_t, c_void_p],
    ),
    "tt_inbatch_fused_workspace_size": (c_size_t, [c_int64, c_int32]),
    "tt_inbatch_softmax_xent": (
        c_int32,
        [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p, c_size_t, c_void_p],
    ),
    "tt_inbatch_prep": (
        c_int32,
        [c_void_p, c_int64, c_int64, c_int32, c_int32, c_void_p, c_void_p, c_size_t, c_void_p],
    ),
    "tt_inbatch_softmax_xent_prepped": (
        c_int32,
        [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p, c_size_t, c_void_p],
    ),
    "tt_inbatch_softmax_xent_loss": (
        c_int32,
        [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_float, c_void_p, c_int32, c_void_p, c_size_t, c_void_p],
    ),
    "tt_inbatch_fused_x3_workspace_size": (c_size_t, [c_int64, c_int32]),
    "tt_inbatch_softmax_xent_x3": (
        c_int32,
        [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_float, c_void_p, c_void_p, c_size_t, c_void_p],
    ),
    "tt_bruteforce_index_bytes": (c_size_t, [c_int64, c_int32]),
    "tt_bruteforce_build": (c_int32, [c_void_p, c_int64, c_int64, c_int32, c_void_p, c_size_t, c_void_p]),
    "tt_bruteforce_workspace_size": (c_size_t, [c_int64, c_int64, c_int32, c_int32]),
    "tt_bruteforce_search": (
        c_int32,
        [c_void_p, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_int64, c_int64, c_int32, c_int64, c_void_p,
         c_void_p, c_void_p, c_size_t, c_void_p],
    ),
    "tt_bruteforce_shard_chunk": (c_int64, [c_int64, c_int64, c_int32, c_int32]),
    "tt_bruteforce_shard_workspace_size": (c_size_t, [c_int64, c_int64, c_int32, c_int32]),
    "tt_bruteforce_shard_screen": (
        c_int32,
        [c_void_p, c_int64, c_int32, c_void_p, c_int64, c_int64, c_int64, c_int32, c_int64, c_void_p, c_void_p,
         c_size_t, c_void_p],
    ),
    "tt_bruteforce_shard_finalize": (
        c_int32,
        [c_void_p, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_int64, c_int64, c_int64, c_int32, c_int64,
         c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p],
    ),
    "tt_topk_merge": (c_int32, [c_void_p, c_void_p, c_int32, c_int64, c_int32, c_int32, c_void_p, c_void_p, c_void_p]),
    "tt_recall_hits": (c_int32, [c_void_p, c_void_p, c_int64, c_int32, POINTER(c_int32), c_int32, c_void_p, c_void_p]),
    "tt_vocab_create": (c_int32, [c_void_p, c_void_p, c_int64, POINTER(c_void_p)]),
    "tt_vocab_size": (c_int64, [c_void_p]),
    "tt_vocab_encode": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int32]),
    "tt_vocab_destroy": (c_int32, [c_void_p]),
    "tt_mlp_pack_bytes": (c_size_t, [c_int32, c_int32]),
    "tt_mlp_pack": (c_int32, [c_void_p, c_int64, c_int32, c_int32, c_int32, c_void_p, c_size_t, c_void_p]),
    "tt_mlp_pack_many": (c_int32, [c_void_p, c_int32, c_void_p]),
    "tt_mlp_rows_workspace_size": (c_size_t, [c_int64, c_int32]),
    "tt_mlp_rows": (
        c_int32,
        [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int32, c_void_p, c_int32, c_void_p, c_int32,
         c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_size_t, c_void_p]),
    "tt_mlp_wgrad_workspace_size": (c_size_t, [c_int64, c_int32, c_int32]),
    "tt_mlp_wgrad": (
        c_int32,
        [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int32, c_int32, c_void_p,
         c_void_p, c_size_t, c_void_p]),
    "tt_mlp_wgrad_adagrad": (
        c_int32,
        [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int32, c_int32, c_void_p,
         c_void_p, c_void_p, c_float, c_float, c_void_p, c_size_t, c_void_p]),
    "tt_mlp_rows_pair": (c_int32, [c_void_p, c_void_p]),
    "tt_mlp_wgrad_pair_workspace_size": (c_size_t, [c_void_p]),
    "tt_mlp_wgrad_pair": (c_int32, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "tt_batch_take": (
        c_int32,
        [c_void_p, c_int64, c_int32, c_void_p, c_int64, c_void_p, c_int64, c_int32, c_void_p, c_int64, c_void_p,
         c_void_p]),
}

EXPORTED_SYMBOLS = tuple(_PROTOS.keys())

_lock = threading.Lock()
_lib = None


def lib() -> ctypes.CDLL:
    """Load (once) and return libtt.so; raises if it is missing or broken."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libtt.so not found at {LIB_PATH}; build it with "
                "`make -C hm-retrieval-two-tower_amd/csrc` (or __graft_entry__.build())"
            )
        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (restype, argtypes) in _PROTOS.items():
            fn = getattr(handle, name)
            fn.restype = restype
            fn.argtypes = argtypes
        _lib = handle
        return _lib


def check(rc: int) -> None:
    """Raise TTError for a non-zero libtt status."""
    if rc != TT_OK:
        msg = lib().tt_last_error()
        raise TTError(rc, msg.decode() if msg else "")
