"""CPU: libtt.so loads, exports every function include/tt.h declares, and
validates arguments on the host (no kernel is launched by these calls)."""
import ctypes
import os
import re

import pytest

from pkg import _native

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "tt.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tt_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert header_functions() == sorted(_native.EXPORTED_SYMBOLS)


def test_library_exports_every_symbol():
    lib = _native.lib()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.tt_version().decode().startswith("tt ")


def test_host_validation_errors():
    lib = _native.lib()
    rc = lib.tt_gather_grouped(None, 0, 10, None, 4, None)
    assert rc == _native.TT_ERR_BAD_ARG
    assert "segs" in lib.tt_last_error().decode()
    rc = lib.tt_bruteforce_search(None, None, 1, 1, 8, None, 8, 1, 4, 0, None, None, None, 0, None)
    assert rc == _native.TT_ERR_BAD_ARG
    rc = lib.tt_inbatch_xent_rows(None, 8, 4, None, 8, 4, 8, None, 0, None, None, None, None, 0, None)
    assert rc == _native.TT_ERR_BAD_ARG
    # dim > 128 is a valid request this build does not implement
    one = ctypes.c_void_p(16)
    rc = lib.tt_inbatch_xent_rows(one, 256, 4, one, 256, 4, 256, None, 0, one, one, None, one, 1 << 30, None)
    assert rc == _native.TT_ERR_UNSUPPORTED
    with pytest.raises(_native.TTError):
        _native.check(rc)


def test_workspace_queries():
    lib = _native.lib()
    assert lib.tt_inbatch_workspace_size(16384, 16384, 128) > 16384 * 128 * 2
    assert lib.tt_inbatch_workspace_size(16, 16, 300) == 0
    assert lib.tt_bruteforce_index_bytes(105542, 128) >= 105542 * 128 * 2
    assert lib.tt_bruteforce_workspace_size(1 << 20, 105542, 128, 100) > 0
    assert lib.tt_dedup_workspace_size(16384, 128) > 16384 * 128 * 4
    t = (_native.SparseTable * 1)()
    t[0].num_rows, t[0].dim, t[0].num_sources = 100, 8, 1
    assert lib.tt_sparse_workspace_size(t, 1, 4096) > 0
