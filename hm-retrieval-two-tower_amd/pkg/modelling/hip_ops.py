"""Torch-tensor wrappers over the libtt C ABI (include/tt.h).

PyTorch is plumbing here: it owns device memory and the current HIP stream.
Every function checks shapes/dtypes/devices on the host, passes raw device
pointers plus torch's current stream to libtt, and raises on error.  There is
no CPU or eager fallback: a CPU tensor or a missing libtt.so is an error.
"""
from __future__ import annotations

import contextlib
import ctypes
import gc
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from pkg import _native
from pkg._native import GatherSegment, SparseTable, check, lib

__all__ = [
    "loss_sum",
    "gather_grouped",
    "sparse_adagrad",
    "sparse_adagrad_rows",
    "sparse_sort",
    "sparse_status",
    "sparse_adam",
    "dedup_sum",
    "dense_adagrad",
    "dense_adagrad_many",
    "dense_adam",
    "inbatch_rows",
    "inbatch_cols",
    "inbatch_fused",
    "inbatch_fused_workspace",
    "inbatch_prep",
    "probe_arm",
    "probe_arm_repeat",
    "route_requests",
    "route_pad",
    "route_fixed",
    "sparse_routed",
    "route_owner",
    "bruteforce_build",
    "bruteforce_search",
    "bruteforce_shard_search",
    "topk_merge",
    "recall_hits",
    "Workspace",
    "capture_guard",
    "CaptureTopology",
    "NestedJoinError",
]


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _req(t: torch.Tensor, name: str, dtype: torch.dtype, ndim: Optional[int] = None) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must live on the GPU (got {t.device}); libtt has no CPU path")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if ndim is not None and t.dim() != ndim:
        raise ValueError(f"{name} must be {ndim}-D, got shape {tuple(t.shape)}")


def _row_major(t: torch.Tensor, name: str) -> int:
    """Leading dimension of a 2-D tensor with unit column stride."""
    if t.dim() != 2 or (t.stride(1) != 1 and t.shape[1] > 1):
        raise ValueError(f"{name} must be 2-D with unit column stride")
    return max(t.stride(0), t.shape[1])


class NestedJoinError(RuntimeError):
    """A captured stream waited on a side branch without being the capture's
    origin stream (CaptureTopology)."""


class CaptureTopology:
    """The fork / join structure of one hipGraph capture, checked as it is
    issued.  ROCm 7.2's hipStreamEndCapture segfaults when a captured side
    branch waits on another side branch — the branch that forked it
    (tools/graph_fork_probe.py nested_join, profiles/r03_graph_fork_probe.txt)
    or a sibling (the round-5 embedding update on the id-sort stream) — so
    here only the capture's origin stream may wait on a branch; a stream
    entering the capture may wait on any captured stream (a fork) and a
    branch may wait on the origin again.  The origin is the stream of the first event
    recorded while capturing (nothing else is in the capture yet).  On a
    violating wait the wait is NOT issued: every branch is joined into the
    origin instead (so the capture can end cleanly) and NestedJoinError is
    raised."""

    def __init__(self):
        self.active = True
        self.depth = 0  # > 0 inside a checked Stream.wait_event (its Event.wait is the same wait)
        self.origin = None
        self.branches: Dict[int, object] = {}  # stream id -> stream (streams that joined by waiting)
        self.source: Dict[int, object] = {}    # id(event) -> stream it was recorded on

    def recorded(self, event, stream) -> None:
        if not self.active:
            return
        if self.origin is None:
            if not torch.cuda.is_current_stream_capturing():
                return
            self.origin = stream
        self.source[id(event)] = stream

    def waiting(self, stream, event) -> None:
        src = self.source.get(id(event)) if self.active else None
        if src is None or self.origin is None or src == stream:
            return
        if stream != self.origin and stream.cuda_stream not in self.branches:
            # a stream entering the capture: a fork (from the origin or from a
            # branch: legal, tools/graph_fork_probe.py origin_join)
            self.branches[stream.cuda_stream] = stream
            return
        if src != self.origin and stream != self.origin:
            origin, branches = self.origin, list(self.branches.values())
            self.active = False  # the repair below is not itself checked, nor anything after it
            for b in branches:
                origin.wait_stream(b)
            raise NestedJoinError(
                f"captured stream {stream} waits on side branch {src}: only the capture's origin stream "
                f"({origin}) may join a branch (ROCm's hipStreamEndCapture crashes on nested joins)")


@contextlib.contextmanager
def capture_guard(keep: Optional[list] = None):
    """Around a hipGraph capture on this thread: Python's garbage collector
    off (collected first) — a collection mid-capture can run a finalizer that
    frees device or pinned host memory or destroys an event, which the
    runtime refuses during capture and the process aborts — and every HIP
    event created during the capture appended to `keep`, so the caller holds
    them for the graph's lifetime (a captured cross-stream wait whose event
    was destroyed after the capture crashed a later replay).  Every event
    record / wait is checked against the nested-join pattern
    (CaptureTopology: raises NestedJoinError instead of reaching a crash in
    hipStreamEndCapture)."""
    import torch.cuda.streams as _streams

    gc.collect()
    was = gc.isenabled()
    gc.disable()
    orig = (torch.cuda.Event, _streams.Event)
    base = orig[0]
    topo = CaptureTopology()
    methods = (base.record, base.wait, _streams.Stream.wait_event)

    def record(ev, stream=None):
        stream = torch.cuda.current_stream() if stream is None else stream
        methods[0](ev, stream)
        topo.recorded(ev, stream)

    def wait(ev, stream=None):
        stream = torch.cuda.current_stream() if stream is None else stream
        if topo.depth == 0:
            topo.waiting(stream, ev)
        methods[1](ev, stream)

    def wait_event(stream, ev):
        topo.waiting(stream, ev)
        topo.depth += 1
        try:
            methods[2](stream, ev)  # torch implements it as ev.wait(stream): checked once, here
        finally:
            topo.depth -= 1

    base.record, base.wait, _streams.Stream.wait_event = record, wait, wait_event
    if keep is not None:

        class _Kept(base):
            def __new__(cls, *a, **k):
                ev = base.__new__(cls, *a, **k)
                keep.append(ev)
                return ev

        torch.cuda.Event = _Kept
        _streams.Event = _Kept
    try:
        yield
    finally:
        torch.cuda.Event, _streams.Event = orig
        base.record, base.wait, _streams.Stream.wait_event = methods
        if was:
            gc.enable()


class Workspace:
    """Grow-only device scratch buffers, one per (device, scope, tag).

    Buffers are reused across calls on the same stream; allocate (warm) them
    before capturing a hipGraph so replays never allocate.  Work issued on a
    concurrent stream runs inside its own `Workspace.scope(name)` so the two
    streams never share a buffer.
    """

    _bufs: Dict[Tuple[int, str], torch.Tensor] = {}
    _scope = ""
    # device addresses each live captured graph may hold (snapshot(owner)), and
    # the buffers a regrowth replaced while such a graph could still address
    # them: kept until no live graph holds their address (the owner's
    # finalizer releases its hold)
    _holds: Dict[int, set] = {}
    _next_hold = 0
    _retired: List[torch.Tensor] = []

    @classmethod
    def _captured(cls) -> set:
        return set().union(*cls._holds.values()) if cls._holds else set()

    @classmethod
    def _release(cls, token: int) -> None:
        cls._holds.pop(token, None)
        live = cls._captured()
        cls._retired = [b for b in cls._retired if b.data_ptr() in live]

    @classmethod
    def get(cls, nbytes: int, device: torch.device, tag: str) -> torch.Tensor:
        key = (device.index if device.index is not None else torch.cuda.current_device(), cls._scope + tag)
        buf = cls._bufs.get(key)
        if buf is None or buf.numel() < nbytes:
            if buf is not None and buf.data_ptr() in cls._captured():
                cls._retired.append(buf)  # a live graph may replay into it
            # zeroed once (a fresh sparse workspace carries no recorded error)
            buf = torch.zeros(max(int(nbytes), 256), dtype=torch.uint8, device=device)
            cls._bufs[key] = buf
        return buf

    @classmethod
    def existing(cls, device: torch.device, tag: str, scope: Optional[str] = None) -> Optional[torch.Tensor]:
        """The buffer of (device, scope, tag) if it was ever allocated."""
        idx = device.index if device.index is not None else torch.cuda.current_device()
        pre = cls._scope if scope is None else (scope + "/" if scope else "")
        return cls._bufs.get((idx, pre + tag))

    @classmethod
    def all_with_tag(cls, device: torch.device, tag: str) -> List[torch.Tensor]:
        """Every buffer of (device, any scope, tag) allocated so far."""
        idx = device.index if device.index is not None else torch.cuda.current_device()
        return [b for (d, k), b in cls._bufs.items() if d == idx and (k == tag or k.endswith("/" + tag))]

    @classmethod
    def clear(cls) -> None:
        """Forget every buffer (those a captured graph may address stay alive)."""
        live = cls._captured()
        cls._retired.extend(b for b in cls._bufs.values() if b.data_ptr() in live)
        cls._bufs.clear()

    @classmethod
    def snapshot(cls, owner=None) -> Dict[Tuple[int, str], int]:
        """{key: device address} of every buffer now allocated.  A captured
        hipGraph holds these addresses: while `owner` (the graph object) is
        alive they are never freed (a regrowth retires the old buffer
        instead); once it is collected its hold is released and retired
        buffers no live graph addresses are freed (owner=None: held for the
        process's lifetime).  Replay the graph only while
        `unchanged(snapshot)` — the host-side readers (sparse_status) look at
        the current buffers."""
        import weakref

        snap = {k: v.data_ptr() for k, v in cls._bufs.items()}
        token = cls._next_hold
        cls._next_hold += 1
        cls._holds[token] = set(snap.values())
        if owner is not None:
            try:
                weakref.finalize(owner, cls._release, token)
            except TypeError:  # not weak-referenceable: held for good
                pass
        return snap

    @classmethod
    def unchanged(cls, snap: Dict[Tuple[int, str], int]) -> bool:
        return all(k in cls._bufs and cls._bufs[k].data_ptr() == p for k, p in snap.items())

    class scope:  # noqa: N801 - context manager named like the operation
        def __init__(self, name: str):
            self.name = name

        def __enter__(self):
            self.prev = Workspace._scope
            Workspace._scope = self.name + "/" if self.name else ""  # "": the root scope
            return self

        def __exit__(self, *exc):
            Workspace._scope = self.prev
            return False


# --------------------------------------------------------------------------
# K2+K3 gather
def _gather_segments(segments, batch: int):
    arr = (GatherSegment * len(segments))()
    for i, (table, ids, off) in enumerate(segments):
        _req(table, f"table[{i}]", torch.float32)
        if not table.is_contiguous():
            raise ValueError(f"table[{i}] must be contiguous")
        if ids is not None:
            _req(ids, f"ids[{i}]", torch.int32)
            if ids.numel() != batch or not ids.is_contiguous():
                raise ValueError(f"ids[{i}] must be a contiguous [{batch}] int32 tensor")
            dim = table.shape[1]
            rows = table.shape[0]
        else:
            if table.numel() != batch:
                raise ValueError(f"numeric column {i} must have {batch} values")
            dim, rows = 1, batch
        arr[i].table = table.data_ptr()
        arr[i].ids = ids.data_ptr() if ids is not None else None
        arr[i].num_rows = rows
        arr[i].dim = dim
        arr[i].col_offset = off
    return arr


def gather_grouped(
    segments: Sequence[Tuple[torch.Tensor, Optional[torch.Tensor], int]],
    batch: int,
    out: torch.Tensor,
) -> torch.Tensor:
    """segments: (table [V,D] or numeric values [B], ids [B] int32 or None, col_offset)."""
    _req(out, "out", torch.float32, 2)
    ld = _row_major(out, "out")
    if len(segments) > _native.MAX_SEGMENTS:
        raise ValueError(f"at most {_native.MAX_SEGMENTS} segments per launch")
    arr = _gather_segments(segments, batch)
    check(lib().tt_gather_grouped(arr, len(segments), batch, out.data_ptr(), ld, _stream()))
    return out


def gather_multi(calls: Sequence[Tuple[Sequence[Tuple[torch.Tensor, Optional[torch.Tensor], int]], torch.Tensor]],
                 batch: int, pack_jobs: Optional[Sequence[Tuple[torch.Tensor, bool, torch.Tensor]]] = None) -> None:
    """Several gather_grouped calls of one batch (e.g. both towers) in one
    launch; pack_jobs (mlp_pack_many's jobs): the weight images packed by the
    same launch (tt_gather_multi_pack)."""
    if sum(len(segs) for segs, _ in calls) > _native.MAX_SEGMENTS:
        raise ValueError(f"at most {_native.MAX_SEGMENTS} segments per launch")
    keep = []
    arr = (_native.GatherCall * len(calls))()
    for i, (segs, out) in enumerate(calls):
        _req(out, f"out[{i}]", torch.float32, 2)
        ld = _row_major(out, f"out[{i}]")
        sa = _gather_segments(segs, batch)
        keep.append(sa)
        arr[i].segs = ctypes.cast(sa, ctypes.c_void_p)
        arr[i].num_segs = len(segs)
        arr[i].out = out.data_ptr()
        arr[i].out_stride = ld
    if pack_jobs:
        check(lib().tt_gather_multi_pack(arr, len(calls), batch, _pack_job_array(pack_jobs), len(pack_jobs),
                                         _stream()))
        return
    check(lib().tt_gather_multi(arr, len(calls), batch, _stream()))


def _sparse_tables(tables: Sequence[dict], batch: int, adam: bool, slots: bool = True):
    arr = (SparseTable * len(tables))()
    for i, t in enumerate(tables):
        table = t["table"]
        _req(table, f"table[{i}]", torch.float32, 2)
        slot0 = t["slot0"] if slots else None
        if not table.is_contiguous():
            raise ValueError(f"table[{i}] must be contiguous")
        if slots:
            _req(slot0, f"slot0[{i}]", torch.float32, 2)
            if not slot0.is_contiguous() or slot0.shape != table.shape:
                raise ValueError(f"table/slot0[{i}] must be contiguous and of equal shape")
        if adam:
            slot1 = t["slot1"]
            _req(slot1, f"slot1[{i}]", torch.float32, 2)
            if not slot1.is_contiguous() or slot1.shape != table.shape:
                raise ValueError(f"slot1[{i}] must be contiguous with the table's shape")
        ids: List[torch.Tensor] = t["ids"]
        offs: List[int] = t["grad_col_offset"]
        if not (1 <= len(ids) <= _native.MAX_SOURCES) or len(ids) != len(offs):
            raise ValueError(f"table[{i}]: 1..{_native.MAX_SOURCES} (ids, col_offset) sources required")
        arr[i].table = table.data_ptr()
        arr[i].slot0 = slot0.data_ptr() if slots else None
        arr[i].slot1 = t["slot1"].data_ptr() if adam else None
        arr[i].num_rows = table.shape[0]
        arr[i].dim = table.shape[1]
        arr[i].num_sources = len(ids)
        for s, (x, o) in enumerate(zip(ids, offs)):
            _req(x, f"ids[{i}][{s}]", torch.int32)
            if x.numel() != batch or not x.is_contiguous():
                raise ValueError(f"ids[{i}][{s}] must be contiguous [{batch}] int32")
            arr[i].ids[s] = x.data_ptr()
            arr[i].grad_col_offset[s] = o
        g = t.get("grad")
        if g is not None:  # per-table gradient buffer (e.g. another tower's input gradient)
            _req(g, f"grad[{i}]", torch.float32, 2)
            if g.shape[0] != batch:
                raise ValueError(f"grad[{i}] must have {batch} rows")
            arr[i].grad = g.data_ptr()
            arr[i].grad_ld = _row_major(g, f"grad[{i}]")
    return arr


def sparse_adagrad(tables: Sequence[dict], batch: int, grad: Optional[torch.Tensor], lr: float,
                   epsilon: float, presorted: bool = False, ws_tag: str = "sparse") -> None:
    """tables: dicts with table, slot0 (accumulator), ids [list], grad_col_offset [list] and an
    optional per-table "grad" [batch, *] that overrides the call's `grad` (which may then be None),
    so one call — one sort — updates the tables of both towers.  presorted: the ids were
    already sorted by sparse_sort(tables, batch) (same tables, stream-ordered before this)."""
    ld = 0
    if grad is not None:
        _req(grad, "grad", torch.float32, 2)
        ld = _row_major(grad, "grad")
    elif any(t.get("grad") is None for t in tables):
        raise ValueError("grad is None but some table has no per-table grad")
    arr = _sparse_tables(tables, batch, adam=False)
    L = lib()
    need = L.tt_sparse_workspace_size(arr, len(tables), batch)
    dev = grad.device if grad is not None else tables[0]["grad"].device
    ws = Workspace.get(need, dev, ws_tag)
    fn = L.tt_sparse_adagrad_sorted if presorted else L.tt_sparse_adagrad
    check(fn(arr, len(tables), batch, grad.data_ptr() if grad is not None else None, ld, lr, epsilon,
             ws.data_ptr(), ws.numel(), _stream()))


def sparse_adagrad_rows(tables: Sequence[Tuple[torch.Tensor, torch.Tensor]], tags: torch.Tensor, rows: torch.Tensor,
                        grad: torch.Tensor, lr: float, epsilon: float) -> None:
    """Adagrad on DISTINCT rows (tt_sparse_adagrad_rows): slot j applies
    grad[j] to row rows[j] of tables[tags[j]] = (table, accumulator);
    invalid tags / rows are skipped.  Each (tag, row) at most once."""
    _req(tags, "tags", torch.int32, 1)
    _req(rows, "rows", torch.int32, 1)
    _req(grad, "grad", torch.float32, 2)
    n = tags.numel()
    if rows.numel() != n or grad.shape[0] < n:
        raise ValueError("tags / rows / grad sizes disagree")
    arr = (SparseTable * len(tables))()
    for i, (t, a) in enumerate(tables):
        _req(t, f"table[{i}]", torch.float32, 2)
        _req(a, f"slot0[{i}]", torch.float32, 2)
        if not (t.is_contiguous() and a.is_contiguous()) or a.shape != t.shape:
            raise ValueError(f"table/slot0[{i}] must be contiguous and of equal shape")
        arr[i].table, arr[i].slot0, arr[i].num_rows, arr[i].dim = t.data_ptr(), a.data_ptr(), t.shape[0], t.shape[1]
    check(lib().tt_sparse_adagrad_rows(arr, len(tables), tags.data_ptr(), rows.data_ptr(), n, grad.data_ptr(),
                                       _row_major(grad, "grad"), lr, epsilon, _stream()))


def sparse_status(device: torch.device, ws_tag: str = "sparse", scope: Optional[str] = None) -> None:
    """Raise TTError if a sparse apply on this workspace recorded an error
    (keys of another call, tt_sparse_status) since the last check.  Synchronises
    the current stream."""
    ws = Workspace.existing(device, ws_tag, scope)
    if ws is None:
        return
    check(lib().tt_sparse_status(ws.data_ptr(), ws.numel(), _stream()))


def sparse_status_all(device: torch.device, ws_tags: Sequence[str]) -> None:
    """sparse_status over every scope's workspace of each tag (all are read
    and cleared; the first recorded error is raised)."""
    err = None
    for tag in ws_tags:
        for ws in Workspace.all_with_tag(device, tag):
            try:
                check(lib().tt_sparse_status(ws.data_ptr(), ws.numel(), _stream()))
            except Exception as e:  # noqa: BLE001 - re-raised below after every workspace is cleared
                err = err or e
    if err is not None:
        raise err


def sparse_sort(tables: Sequence[dict], batch: int, ws_tag: str = "sparse", slots: bool = True) -> None:
    """First stage of sparse_adagrad(..., presorted=True) or
    sparse_scatter_sum(..., presorted=True) (slots=False: tables without
    accumulators): build and sort the lookup keys (reads only the ids; no
    gradient needed), on the current stream."""
    arr = _sparse_tables(tables, batch, adam=False, slots=slots)
    L = lib()
    need = L.tt_sparse_workspace_size(arr, len(tables), batch)
    ws = Workspace.get(need, tables[0]["table"].device, ws_tag)
    check(L.tt_sparse_sort(arr, len(tables), batch, ws.data_ptr(), ws.numel(), _stream()))


def sparse_adam(tables: Sequence[dict], batch: int, grad: torch.Tensor, lr: float, beta1: float, beta2: float,
                epsilon: float, step: int) -> None:
    _req(grad, "grad", torch.float32, 2)
    ld = _row_major(grad, "grad")
    arr = _sparse_tables(tables, batch, adam=True)
    L = lib()
    need = L.tt_sparse_workspace_size(arr, len(tables), batch)
    ws = Workspace.get(need, grad.device, "sparse")
    check(L.tt_sparse_adam(arr, len(tables), batch, grad.data_ptr(), ld, lr, beta1, beta2, epsilon, step,
                           ws.data_ptr(), ws.numel(), _stream()))


def sparse_scatter_sum(tables: Sequence[dict], batch: int, grad: torch.Tensor, ws_tag: str = "sparse",
                       presorted: bool = False) -> None:
    """tables: dicts with table (zero-filled dense gradient [rows, dim]), ids
    [list], grad_col_offset [list]; every touched row receives its
    duplicate-summed gradient (tt_sparse_scatter_sum).  presorted: the keys
    were sorted by sparse_sort(tables, batch, ws_tag, slots=False) earlier
    (tt_sparse_scatter_sum_sorted)."""
    _req(grad, "grad", torch.float32, 2)
    ld = _row_major(grad, "grad")
    arr = _sparse_tables(tables, batch, adam=False, slots=False)
    L = lib()
    need = L.tt_sparse_workspace_size(arr, len(tables), batch)
    ws = Workspace.get(need, grad.device, ws_tag)
    fn = L.tt_sparse_scatter_sum_sorted if presorted else L.tt_sparse_scatter_sum
    check(fn(arr, len(tables), batch, grad.data_ptr(), ld, ws.data_ptr(), ws.numel(), _stream()))


def route_requests(lookups: Sequence[Tuple[torch.Tensor, int, int]], world: int, num_tags: int,
                   ordered: bool = False):
    """lookups: (ids [B] int32, table rows, tag).  Returns (send [L*B, 2] int32
    capacity, counts [world] int64, num_requests [1] int32, idx [L, B] int32)
    from tt_route_requests (owner-major deduplicated requests); ordered=True
    appends the route's sorted order (order [L*B], grp_first / grp_last
    [world*num_tags] int32, tt_route_requests_ordered) for sparse_routed."""
    L = len(lookups)
    B = lookups[0][0].numel()
    dev = lookups[0][0].device
    arr = (_native.RouteLookup * L)()
    max_rows = 1
    for i, (ids, rows, tag) in enumerate(lookups):
        _req(ids, f"ids[{i}]", torch.int32, 1)
        if ids.numel() != B or not ids.is_contiguous():
            raise ValueError("route: every lookup needs a contiguous [B] int32 id tensor")
        arr[i].ids = ids.data_ptr()
        arr[i].num_rows = int(rows)
        arr[i].tag = int(tag)
        max_rows = max(max_rows, int(rows))
    send = torch.empty(L * B, 2, dtype=torch.int32, device=dev)
    counts = torch.empty(world, dtype=torch.int64, device=dev)
    nreq = torch.empty(1, dtype=torch.int32, device=dev)
    idx = torch.empty(L, B, dtype=torch.int32, device=dev)
    lib_ = lib()
    ws = Workspace.get(lib_.tt_route_workspace_size(L, B, world, max_rows, num_tags), dev, "route")
    if not ordered:
        check(lib_.tt_route_requests(arr, L, B, world, num_tags, send.data_ptr(), counts.data_ptr(), nreq.data_ptr(),
                                     idx.data_ptr(), ws.data_ptr(), ws.numel(), _stream()))
        return send, counts, nreq, idx
    order = torch.empty(L * B, dtype=torch.int32, device=dev)
    grp = torch.empty(2, world * num_tags, dtype=torch.int32, device=dev)
    check(lib_.tt_route_requests_ordered(arr, L, B, world, num_tags, send.data_ptr(), counts.data_ptr(),
                                         nreq.data_ptr(), idx.data_ptr(), order.data_ptr(), grp[0].data_ptr(),
                                         grp[1].data_ptr(), ws.data_ptr(), ws.numel(), _stream()))
    return send, counts, nreq, idx, (order, grp[0], grp[1])


def route_fixed(lookups: Sequence[Tuple[torch.Tensor, int, int]], world: int, num_tags: int, cap: int,
                overflow: Optional[torch.Tensor] = None, ordered: bool = False, owner: bool = False,
                idx_out: Optional[torch.Tensor] = None):
    """The fixed-capacity route in one call (tt_route_fixed; one launch for
    <= 16384 lookups): (send_padded [world*cap, 2], idx_padded [L, B],
    counts [world] int64, (order, grp_first, grp_last) if ordered, and at
    world 1 with owner=True (tags, rows, table_ids [num_tags, cap]) of the
    slots) — equal to route_requests + route_pad (+ route_owner).  idx_out:
    an [L, B] int32 buffer for idx_padded (e.g. a captured step's static one)."""
    L = len(lookups)
    B = lookups[0][0].numel()
    dev = lookups[0][0].device
    arr = (_native.RouteLookup * L)()
    max_rows = 1
    for i, (ids, rows, tag) in enumerate(lookups):
        _req(ids, f"ids[{i}]", torch.int32, 1)
        if ids.numel() != B or not ids.is_contiguous():
            raise ValueError("route: every lookup needs a contiguous [B] int32 id tensor")
        arr[i].ids = ids.data_ptr()
        arr[i].num_rows = int(rows)
        arr[i].tag = int(tag)
        max_rows = max(max_rows, int(rows))
    if owner and world != 1:
        raise ValueError("route_fixed: owner=True is the world-1 shortcut")
    slots = world * cap
    send_p = torch.empty(slots, 2, dtype=torch.int32, device=dev)
    if idx_out is not None:
        _req(idx_out, "idx_out", torch.int32, 2)
        if tuple(idx_out.shape) != (L, B) or not idx_out.is_contiguous():
            raise ValueError(f"route_fixed: idx_out must be a contiguous [{L}, {B}] int32 buffer")
    idx_p = idx_out if idx_out is not None else torch.empty(L, B, dtype=torch.int32, device=dev)
    counts = torch.empty(world, dtype=torch.int64, device=dev)
    if overflow is not None:
        _req(overflow, "overflow", torch.int32, 1)
    order = grp = own = None
    if ordered:
        order = torch.empty(L * B, dtype=torch.int32, device=dev)
        grp = torch.empty(2, world * num_tags, dtype=torch.int32, device=dev)
    if owner:
        own = (torch.empty(slots, dtype=torch.int32, device=dev), torch.empty(slots, dtype=torch.int32, device=dev),
               torch.empty(num_tags, slots, dtype=torch.int32, device=dev))
    lib_ = lib()
    ws = Workspace.get(lib_.tt_route_fixed_workspace_size(L, B, world, max_rows, num_tags), dev, "route")
    check(lib_.tt_route_fixed(arr, L, B, world, num_tags, cap, send_p.data_ptr(), idx_p.data_ptr(), counts.data_ptr(),
                              _ptr(overflow), _ptr(order), _ptr(grp[0] if grp is not None else None),
                              _ptr(grp[1] if grp is not None else None), *(_ptr(t) for t in (own or (None,) * 3)),
                              ws.data_ptr(), ws.numel(), _stream()))
    return send_p, idx_p, counts, (order, grp[0], grp[1]) if ordered else None, own


def sparse_routed(tables: Sequence[dict], batch: int, grad: Optional[torch.Tensor], route: dict, op: str,
                  lr: float = 0.0, epsilon: float = 0.0, ws_tag: str = "sparse_routed") -> None:
    """Per-request sums (op "sum", tt_sparse_scatter_sum semantics) or the
    Adagrad update (op "adagrad", tables need slot0) of routed lookups, keyed
    by the route's own sort (tt_sparse_routed: no second sort).  tables: as
    for sparse_scatter_sum / sparse_adagrad (ids = each source lookup's slots).
    route: order, grp_first, grp_last (route_requests(..., ordered=True)),
    slot ([L, B] slots of every routed lookup), slot_row (optional [world*cap]
    keys per slot), cap, world, num_tags and per routed lookup l its
    lookup_tag / lookup_table / lookup_source."""
    ld = 0
    if grad is not None:
        _req(grad, "grad", torch.float32, 2)
        ld = _row_major(grad, "grad")
    elif any(t.get("grad") is None for t in tables):
        raise ValueError("grad is None but some table has no per-table grad")
    if op not in ("sum", "adagrad"):
        raise ValueError(f"sparse_routed: op must be 'sum' or 'adagrad', got {op!r}")
    arr = _sparse_tables(tables, batch, adam=False, slots=op == "adagrad")
    rs = _native.RouteSorted()
    for name in ("order", "grp_first", "grp_last", "slot"):
        t = route[name]
        _req(t, name, torch.int32)
        if not t.is_contiguous():
            raise ValueError(f"sparse_routed: {name} must be contiguous")
        setattr(rs, name, t.data_ptr())
    rs.slot_row = _ptr(route.get("slot_row"))
    rs.cap, rs.world, rs.num_tags = int(route["cap"]), int(route["world"]), int(route["num_tags"])
    L = len(route["lookup_tag"])
    if L > _native.ROUTE_MAX_LOOKUPS:
        raise ValueError(f"sparse_routed: at most {_native.ROUTE_MAX_LOOKUPS} routed lookups, got {L}")
    rs.num_lookups = L
    for i in range(L):
        rs.lookup_tag[i] = int(route["lookup_tag"][i])
        rs.lookup_table[i] = int(route["lookup_table"][i])
        rs.lookup_source[i] = int(route["lookup_source"][i])
    lib_ = lib()
    need = lib_.tt_sparse_workspace_size(arr, len(tables), batch)
    dev = grad.device if grad is not None else tables[0]["grad"].device
    ws = Workspace.get(need, dev, ws_tag)
    check(lib_.tt_sparse_routed(arr, len(tables), batch, grad.data_ptr() if grad is not None else None, ld,
                                ctypes.byref(rs), 1 if op == "adagrad" else 0, lr, epsilon, ws.data_ptr(), ws.numel(),
                                _stream()))


def route_pad(send: torch.Tensor, counts: torch.Tensor, idx: torch.Tensor, world: int, cap: int,
              overflow: Optional[torch.Tensor] = None):
    """The compact requests of route_requests in `cap` fixed slots per owner
    (tt_route_pad): (send_padded [world*cap, 2], idx_padded like idx).  No
    host sync; `overflow` (int32 [1], optional) counts dropped requests."""
    _req(send, "send", torch.int32, 2)
    _req(counts, "counts", torch.int64, 1)
    _req(idx, "idx", torch.int32)
    if counts.numel() != world or not idx.is_contiguous():
        raise ValueError("route_pad: counts must be [world], idx contiguous")
    send_p = torch.empty(world * cap, 2, dtype=torch.int32, device=send.device)
    idx_p = torch.empty_like(idx)
    if overflow is not None:
        _req(overflow, "overflow", torch.int32, 1)
    check(lib().tt_route_pad(send.data_ptr(), counts.data_ptr(), idx.data_ptr(), idx.numel(), world, cap,
                             send_p.data_ptr(), idx_p.data_ptr(), _ptr(overflow), _stream()))
    return send_p, idx_p


def route_owner(recv: torch.Tensor, world: int, num_tags: int):
    """recv [n, 2] int32 requests received by this owner -> (tags [n], local rows
    [n], table_ids [num_tags, n]) from tt_route_owner."""
    _req(recv, "recv", torch.int32, 2)
    n = recv.shape[0]
    tags = torch.empty(n, dtype=torch.int32, device=recv.device)
    rows = torch.empty(n, dtype=torch.int32, device=recv.device)
    tids = torch.empty(num_tags, n, dtype=torch.int32, device=recv.device)
    check(lib().tt_route_owner(recv.contiguous().data_ptr(), n, world, num_tags, tags.data_ptr(), rows.data_ptr(),
                               tids.data_ptr(), _stream()))
    return tags, rows, tids


def gather_tagged(tables: Sequence[torch.Tensor], tags: torch.Tensor, rows: torch.Tensor,
                  out: torch.Tensor) -> torch.Tensor:
    """out[j] = tables[tags[j]][rows[j]] (zero row when invalid); tables share dim."""
    _req(tags, "tags", torch.int32, 1)
    _req(rows, "rows", torch.int32, 1)
    _req(out, "out", torch.float32, 2)
    ld = _row_major(out, "out")
    dim = tables[0].shape[1]
    arr = (_native.RowTable * len(tables))()
    for i, t in enumerate(tables):
        _req(t, f"tables[{i}]", torch.float32, 2)
        if t.shape[1] != dim or not t.is_contiguous():
            raise ValueError("tables must be contiguous and share one dim")
        arr[i].table = t.data_ptr()
        arr[i].num_rows = t.shape[0]
    n = tags.numel()
    if rows.numel() != n or out.shape[0] < n or out.shape[1] < dim:
        raise ValueError("tags/rows/out sizes disagree")
    check(lib().tt_gather_tagged(arr, len(tables), dim, tags.data_ptr(), rows.data_ptr(), n, out.data_ptr(), ld,
                                 _stream()))
    return out


def dedup_sum(ids: torch.Tensor, grad: torch.Tensor, num_rows: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Distinct ids (ascending) and per-id gradient sums (K8)."""
    _req(ids, "ids", torch.int32, 1)
    _req(grad, "grad", torch.float32, 2)
    ld = _row_major(grad, "grad")
    n, dim = ids.numel(), grad.shape[1]
    if grad.shape[0] != n:
        raise ValueError("grad must have one row per id")
    L = lib()
    ws = Workspace.get(L.tt_dedup_workspace_size(n, dim), grad.device, "dedup")
    uniq = torch.empty(n, dtype=torch.int32, device=grad.device)
    summed = torch.empty(n, dim, dtype=torch.float32, device=grad.device)
    count = torch.empty(1, dtype=torch.int32, device=grad.device)
    check(L.tt_dedup_sum(ids.data_ptr(), n, num_rows, grad.data_ptr(), ld, dim, uniq.data_ptr(), summed.data_ptr(),
                         count.data_ptr(), ws.data_ptr(), ws.numel(), _stream()))
    u = int(count.item())
    return uniq[:u], summed[:u]


def loss_sum(x: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    """0-d tensor scale * x.sum() (tt_sum: one deterministic launch)."""
    _req(x, "x", torch.float32)
    if not x.is_contiguous():
        raise ValueError("x must be contiguous")
    out = torch.empty((), dtype=torch.float32, device=x.device)
    check(lib().tt_sum(x.data_ptr(), x.numel(), float(scale), out.data_ptr(), _stream()))
    return out


def dense_adagrad(param: torch.Tensor, accum: torch.Tensor, grad: torch.Tensor, lr: float, epsilon: float) -> None:
    for t, n in ((param, "param"), (accum, "accum"), (grad, "grad")):
        _req(t, n, torch.float32)
        if not t.is_contiguous() or t.numel() != param.numel():
            raise ValueError(f"{n} must be contiguous with param's numel")
    check(lib().tt_dense_adagrad(param.data_ptr(), accum.data_ptr(), grad.data_ptr(), param.numel(), lr, epsilon,
                                 _stream()))


def dense_adagrad_many(jobs: Sequence[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]], lr: float,
                       epsilon: float) -> None:
    """dense_adagrad on up to 8 (param, accum, grad) buffers in one launch
    (tt_dense_adagrad_many; bit-identical to one call each)."""
    arr = (_native.DenseJob * len(jobs))()
    for i, (p, a, g) in enumerate(jobs):
        for name, t in (("param", p), ("accum", a), ("grad", g)):
            _req(t, f"{name}[{i}]", torch.float32)
            if not t.is_contiguous() or t.numel() != p.numel():
                raise ValueError(f"dense_adagrad_many: {name}[{i}] must be contiguous with param's size")
        arr[i].param, arr[i].accum, arr[i].grad, arr[i].n = p.data_ptr(), a.data_ptr(), g.data_ptr(), p.numel()
    check(lib().tt_dense_adagrad_many(arr, len(jobs), lr, epsilon, _stream()))


def dense_adam(param, m, v, grad, lr, beta1, beta2, epsilon, step) -> None:
    for t, n in ((param, "param"), (m, "m"), (v, "v"), (grad, "grad")):
        _req(t, n, torch.float32)
        if not t.is_contiguous() or t.numel() != param.numel():
            raise ValueError(f"{n} must be contiguous with param's numel")
    check(lib().tt_dense_adam(param.data_ptr(), m.data_ptr(), v.data_ptr(), grad.data_ptr(), param.numel(), lr,
                              beta1, beta2, epsilon, step, _stream()))


# --------------------------------------------------------------------------
# K5+K6+K7 fused in-batch softmax cross-entropy
# --------------------------------------------------------------------------
# Measurement hook: time ONE kernel of a multi-launch entry point (tt_probe_arm)
PROBE_INBATCH_ROWS, PROBE_INBATCH_COLS, PROBE_INDEX_SCREEN, PROBE_INDEX_FINALIZE = range(4)


def probe_arm(kernel: int, start: "torch.cuda.Event", stop: "torch.cuda.Event") -> None:
    """The next launch of `kernel` on this thread records `start` / `stop`
    (timing-enabled torch.cuda.Events) on its own launch stream."""
    for ev in (start, stop):
        if not ev.cuda_event:  # torch creates the HIP event on first record
            ev.record()
    check(lib().tt_probe_arm(kernel, start.cuda_event, stop.cuda_event))


def probe_arm_repeat(kernel: int, start: "torch.cuda.Event", stop: "torch.cuda.Event", reps: int) -> None:
    """As probe_arm, and the armed in-batch pass is launched `reps` times back
    to back between the events (tt_probe_arm_repeat)."""
    for ev in (start, stop):
        if not ev.cuda_event:
            ev.record()
    check(lib().tt_probe_arm_repeat(kernel, start.cuda_event, stop.cuda_event, int(reps)))


def _opt_ptr(t: Optional[torch.Tensor], name: str, n: int) -> Optional[int]:
    if t is None:
        return None
    _req(t, name, torch.float32, 1)
    if t.numel() != n or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous [{n}] float32 tensor")
    return t.data_ptr()


def inbatch_rows(q: torch.Tensor, c: torch.Tensor, logq: Optional[torch.Tensor], pos_offset: int = 0,
                 want_dq: bool = True):
    """Row pass: (lse [R], row_loss [R], dq [R,E] or None)."""
    _req(q, "q", torch.float32, 2)
    _req(c, "c", torch.float32, 2)
    ldq, ldc = _row_major(q, "q"), _row_major(c, "c")
    R, E = q.shape
    C = c.shape[0]
    if c.shape[1] != E:
        raise ValueError("q and c must share the embedding size")
    L = lib()
    ws = Workspace.get(L.tt_inbatch_workspace_size(R, C, E), q.device, "inbatch")
    lse = torch.empty(R, dtype=torch.float32, device=q.device)
    row_loss = torch.empty(R, dtype=torch.float32, device=q.device)
    dq = torch.empty(R, E, dtype=torch.float32, device=q.device) if want_dq else None
    check(L.tt_inbatch_xent_rows(q.data_ptr(), ldq, R, c.data_ptr(), ldc, C, E, _opt_ptr(logq, "logq", C),
                                 pos_offset, lse.data_ptr(), row_loss.data_ptr(),
                                 dq.data_ptr() if dq is not None else None, ws.data_ptr(), ws.numel(), _stream()))
    return lse, row_loss, dq


def inbatch_cols(q: torch.Tensor, lse: torch.Tensor, c: torch.Tensor, logq: Optional[torch.Tensor],
                 pos_offset: int = 0, row_loss: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Column pass: dc [C,E] from every row's q [R,E], lse [R] and (optional,
    for the exact 1 - P_pos of confident rows) row_loss [R]."""
    _req(q, "q", torch.float32, 2)
    _req(c, "c", torch.float32, 2)
    ldq, ldc = _row_major(q, "q"), _row_major(c, "c")
    R, E = q.shape
    C = c.shape[0]
    L = lib()
    ws = Workspace.get(L.tt_inbatch_workspace_size(R, C, E), q.device, "inbatch")
    dc = torch.empty(C, E, dtype=torch.float32, device=q.device)
    check(L.tt_inbatch_xent_cols(q.data_ptr(), ldq, R, _opt_ptr(lse, "lse", R), _opt_ptr(row_loss, "row_loss", R),
                                 c.data_ptr(), ldc, C, E,
                                 _opt_ptr(logq, "logq", C), pos_offset, dc.data_ptr(), ws.data_ptr(), ws.numel(),
                                 _stream()))
    return dc


def inbatch_fused_workspace(B: int, E: int, device: torch.device) -> torch.Tensor:
    """The fused entry's workspace in the current scope (fetch it before
    forking per-tower streams so inbatch_prep on either stream and the
    fused call share it)."""
    return Workspace.get(lib().tt_inbatch_fused_workspace_size(B, E), device, "inbatch_fused")


def inbatch_prep(x: torch.Tensor, operand: int, logq: Optional[torch.Tensor], ws: torch.Tensor) -> None:
    """bf16 preparation of one operand of inbatch_fused into `ws` on the
    current stream: operand 0 = q, 1 = c (+ the logQ bias vectors)."""
    _req(x, "x", torch.float32, 2)
    ld = _row_major(x, "x")
    B, E = x.shape
    check(lib().tt_inbatch_prep(x.data_ptr(), ld, B, E, int(operand), _opt_ptr(logq, "logq", B) if operand else None,
                                ws.data_ptr(), ws.numel(), _stream()))


def inbatch_fused(q: torch.Tensor, c: torch.Tensor, logq: Optional[torch.Tensor], ws: Optional[torch.Tensor] = None,
                  prepped: bool = False, loss_scale: Optional[float] = None, x3: bool = False):
    """Single-device loss + gradients (both passes, shared bf16 prep):
    (lse [B], row_loss [B], dq [B,E], dc [B,E]).  prepped: both operands were
    already prepared into `ws` by inbatch_prep (ordered before this call).
    loss_scale: also return the loss loss_scale * sum(row_loss) (a 0-d
    tensor, computed inside the last launch, equal to loss_sum's).
    x3: fp32-faithful products (tt_inbatch_softmax_xent_x3: S and P.V as
    bf16x3 products, ~3x the passes' time; not with prepped)."""
    _req(q, "q", torch.float32, 2)
    _req(c, "c", torch.float32, 2)
    ldq, ldc = _row_major(q, "q"), _row_major(c, "c")
    B, E = q.shape
    if tuple(c.shape) != (B, E):
        raise ValueError("q and c must both be [B, E]")
    if prepped and ws is None:
        raise ValueError("prepped=True needs the workspace the operands were prepared into")
    L = lib()
    if x3:
        if prepped:
            raise ValueError("x3: the fp32-faithful entry prepares its operands itself (prepped=False)")
        ws = Workspace.get(L.tt_inbatch_fused_x3_workspace_size(B, E), q.device, "inbatch_fused_x3")
    if ws is None:
        ws = inbatch_fused_workspace(B, E, q.device)
    lse = torch.empty(B, dtype=torch.float32, device=q.device)
    row_loss = torch.empty(B, dtype=torch.float32, device=q.device)
    dq = torch.empty(B, E, dtype=torch.float32, device=q.device)
    dc = torch.empty(B, E, dtype=torch.float32, device=q.device)
    if x3:
        loss = torch.empty((), dtype=torch.float32, device=q.device) if loss_scale is not None else None
        check(L.tt_inbatch_softmax_xent_x3(q.data_ptr(), ldq, c.data_ptr(), ldc, B, E, _opt_ptr(logq, "logq", B),
                                           lse.data_ptr(), row_loss.data_ptr(), dq.data_ptr(), dc.data_ptr(),
                                           float(loss_scale if loss_scale is not None else 1.0),
                                           loss.data_ptr() if loss is not None else None, ws.data_ptr(), ws.numel(),
                                           _stream()))
        return (lse, row_loss, dq, dc, loss) if loss is not None else (lse, row_loss, dq, dc)
    if loss_scale is not None:
        loss = torch.empty((), dtype=torch.float32, device=q.device)
        check(L.tt_inbatch_softmax_xent_loss(q.data_ptr(), ldq, c.data_ptr(), ldc, B, E, _opt_ptr(logq, "logq", B),
                                             lse.data_ptr(), row_loss.data_ptr(), dq.data_ptr(), dc.data_ptr(),
                                             float(loss_scale), loss.data_ptr(), int(prepped), ws.data_ptr(),
                                             ws.numel(), _stream()))
        return lse, row_loss, dq, dc, loss
    fn = L.tt_inbatch_softmax_xent_prepped if prepped else L.tt_inbatch_softmax_xent
    check(fn(q.data_ptr(), ldq, c.data_ptr(), ldc, B, E, _opt_ptr(logq, "logq", B), lse.data_ptr(), row_loss.data_ptr(),
             dq.data_ptr(), dc.data_ptr(), ws.data_ptr(), ws.numel(), _stream()))
    return lse, row_loss, dq, dc


# --------------------------------------------------------------------------
# K11+K12 brute-force index
def bruteforce_build(cand: torch.Tensor) -> torch.Tensor:
    _req(cand, "cand", torch.float32, 2)
    ld = _row_major(cand, "cand")
    n, d = cand.shape
    L = lib()
    nbytes = L.tt_bruteforce_index_bytes(n, d)
    if nbytes == 0:
        raise ValueError(f"unsupported index shape {tuple(cand.shape)}")
    index = torch.empty(nbytes, dtype=torch.uint8, device=cand.device)
    check(L.tt_bruteforce_build(cand.data_ptr(), ld, n, d, index.data_ptr(), nbytes, _stream()))
    return index


def bruteforce_search(index: torch.Tensor, cand: torch.Tensor, queries: torch.Tensor, k: int,
                      index_offset: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    _req(index, "index", torch.uint8, 1)
    _req(cand, "cand", torch.float32, 2)
    _req(queries, "queries", torch.float32, 2)
    ldc, ldq = _row_major(cand, "cand"), _row_major(queries, "queries")
    n, d = cand.shape
    nq = queries.shape[0]
    if queries.shape[1] != d:
        raise ValueError("queries and candidates must share the embedding size")
    if k > n:
        raise ValueError(f"k={k} exceeds the number of candidates {n}")
    L = lib()
    ws = Workspace.get(L.tt_bruteforce_workspace_size(max(nq, 1), n, d, k), queries.device, "bruteforce")
    out_s = torch.empty(nq, k, dtype=torch.float32, device=queries.device)
    out_i = torch.empty(nq, k, dtype=torch.int32, device=queries.device)
    check(L.tt_bruteforce_search(index.data_ptr(), cand.data_ptr(), ldc, n, d, queries.data_ptr(), ldq, nq, k,
                                 index_offset, out_s.data_ptr(), out_i.data_ptr(), ws.data_ptr(), ws.numel(),
                                 _stream()))
    return out_s, out_i


def bruteforce_shard_chunk(n_queries: int, shard_sizes: Sequence[int], dim: int, k: int) -> int:
    """The query chunk every rank of a candidate-sharded search uses: the
    smallest of the shards' recommendations (tt_bruteforce_shard_chunk), so
    all ranks make the same number of all_reduce calls with the same lengths."""
    L = lib()
    return max(1, min(int(L.tt_bruteforce_shard_chunk(max(int(n_queries), 1), int(n), dim, k)) for n in shard_sizes))


def bruteforce_shard_search(index: torch.Tensor, cand: torch.Tensor, queries: torch.Tensor, k: int,
                            index_offset: int, reduce_max, chunk: Optional[int] = None
                            ) -> Tuple[torch.Tensor, torch.Tensor]:
    """This shard's part of a candidate-sharded exact top-k (tt.h
    tt_bruteforce_shard_*): per chunk of queries, the screen's lower bound on
    the shard's k-th score, `reduce_max(t)` (in place: the max over the shards,
    an all_reduce) as the floor, then the shard's exact top-k of the entries
    that can reach it, padded with (-inf, INT32_MAX).  `chunk` must be the
    same on every rank (bruteforce_shard_chunk over all shard sizes); the
    default, this shard's own recommendation, is only safe for one rank."""
    _req(index, "index", torch.uint8, 1)
    _req(cand, "cand", torch.float32, 2)
    _req(queries, "queries", torch.float32, 2)
    ldc, ldq = _row_major(cand, "cand"), _row_major(queries, "queries")
    n, d = cand.shape
    nq = queries.shape[0]
    if queries.shape[1] != d:
        raise ValueError("queries and candidates must share the embedding size")
    if k > n:
        raise ValueError(f"k={k} exceeds the shard's {n} candidates")
    L = lib()
    out_s = torch.empty(nq, k, dtype=torch.float32, device=queries.device)
    out_i = torch.empty(nq, k, dtype=torch.int32, device=queries.device)
    if nq == 0:
        return out_s, out_i
    chunk = int(chunk) if chunk else int(L.tt_bruteforce_shard_chunk(nq, n, d, k))
    if chunk < 1:
        raise ValueError(f"chunk must be >= 1, got {chunk}")
    ws = Workspace.get(L.tt_bruteforce_shard_workspace_size(chunk, n, d, k), queries.device, "bruteforce_shard")
    kth = torch.empty(chunk, dtype=torch.float32, device=queries.device)
    for q0 in range(0, nq, chunk):
        m = min(chunk, nq - q0)
        qc = queries[q0:q0 + m]
        check(L.tt_bruteforce_shard_screen(index.data_ptr(), n, d, qc.data_ptr(), ldq, m, chunk, k, index_offset,
                                           kth.data_ptr(), ws.data_ptr(), ws.numel(), _stream()))
        reduce_max(kth[:m])
        check(L.tt_bruteforce_shard_finalize(index.data_ptr(), cand.data_ptr(), ldc, n, d, qc.data_ptr(), ldq, m,
                                             chunk, k, index_offset, kth.data_ptr(), out_s[q0:q0 + m].data_ptr(),
                                             out_i[q0:q0 + m].data_ptr(), ws.data_ptr(), ws.numel(), _stream()))
    return out_s, out_i


def topk_merge(scores: torch.Tensor, idx: torch.Tensor, k_out: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """scores/idx: [L, Q, k_in] sorted per list -> global [Q, k_out]."""
    _req(scores, "scores", torch.float32, 3)
    _req(idx, "idx", torch.int32, 3)
    if not (scores.is_contiguous() and idx.is_contiguous()) or scores.shape != idx.shape:
        raise ValueError("scores/idx must be contiguous and of equal shape")
    Ln, Q, k_in = scores.shape
    out_s = torch.empty(Q, k_out, dtype=torch.float32, device=scores.device)
    out_i = torch.empty(Q, k_out, dtype=torch.int32, device=scores.device)
    check(lib().tt_topk_merge(scores.data_ptr(), idx.data_ptr(), Ln, Q, k_in, k_out, out_s.data_ptr(),
                              out_i.data_ptr(), _stream()))
    return out_s, out_i


def recall_hits(true_ids: torch.Tensor, cand_ids: torch.Tensor, ks: Sequence[int], hits: torch.Tensor) -> None:
    """hits [len(ks)] int64 += #{b: true_ids[b] in cand_ids[b,:k]} (every match counts)."""
    _req(true_ids, "true_ids", torch.int32, 1)
    _req(cand_ids, "cand_ids", torch.int32, 2)
    _req(hits, "hits", torch.int64, 1)
    B, K = cand_ids.shape
    if true_ids.numel() != B or not cand_ids.is_contiguous() or not true_ids.is_contiguous():
        raise ValueError("true_ids [B] and cand_ids [B,K] must be contiguous")
    ks_arr = (ctypes.c_int32 * len(ks))(*[int(k) for k in ks])
    check(lib().tt_recall_hits(true_ids.data_ptr(), cand_ids.data_ptr(), B, K, ks_arr, len(ks), hits.data_ptr(),
                               _stream()))


def batch_take(src: torch.Tensor, perm: torch.Tensor, cursor: torch.Tensor, out: torch.Tensor,
               advance: bool = True, status: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[c, b] = src[c, perm[cursor + b]] for the 32-bit word columns of an
    HBM-resident dataset (tt_batch_take); cursor (device int64 [1]) advances by
    the batch when `advance`.  Graph-capturable: nothing is read on the host."""
    _req(src, "src", torch.int32, 2)
    _req(perm, "perm", torch.int64, 1)
    _req(cursor, "cursor", torch.int64, 1)
    _req(out, "out", torch.int32, 2)
    if src.shape[0] != out.shape[0]:
        raise ValueError(f"src has {src.shape[0]} columns, out {out.shape[0]}")
    if perm.numel() != src.shape[1]:
        raise ValueError(f"perm has {perm.numel()} entries for {src.shape[1]} rows")
    if status is not None:
        _req(status, "status", torch.int32, 1)
    check(lib().tt_batch_take(src.data_ptr(), _row_major(src, "src"), src.shape[0], perm.data_ptr(), src.shape[1],
                              cursor.data_ptr(), out.shape[1], int(bool(advance)), out.data_ptr(),
                              _row_major(out, "out"), status.data_ptr() if status is not None else None,
                              _stream()))
    return out


def mlp_pack(w: torch.Tensor, trans: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16 hi/lo MFMA-fragment image of B = w ([K, N]) or B = w^T (trans:
    w is [N, K]) for mlp_rows (tt_mlp_pack)."""
    _req(w, "w", torch.float32, 2)
    K, N = (w.shape[1], w.shape[0]) if trans else (w.shape[0], w.shape[1])
    nbytes = lib().tt_mlp_pack_bytes(K, N)
    if out is None:
        out = torch.empty(nbytes, dtype=torch.uint8, device=w.device)
    if out.numel() < nbytes:
        raise ValueError(f"image buffer of {out.numel()} B < {nbytes} B")
    check(lib().tt_mlp_pack(w.data_ptr(), _row_major(w, "w"), K, N, int(bool(trans)), out.data_ptr(), out.numel(),
                            _stream()))
    out.mlp_kn = (K, N)
    return out


def score_matrix(q: torch.Tensor, c: torch.Tensor, chunk: int = 256) -> torch.Tensor:
    """S = q . c^T [Q, N] fp32 (TwoTowerModel.call, two_tower_model.py:92)
    on libtt's bf16x3 row GEMM: c in column chunks of `chunk` candidates, each
    packed as the B image of one tt_mlp_rows call writing its columns of S."""
    _req(q, "q", torch.float32, 2)
    _req(c, "c", torch.float32, 2)
    Q, E = q.shape
    N = c.shape[0]
    if c.shape[1] != E:
        raise ValueError(f"q {tuple(q.shape)} and c {tuple(c.shape)} must share the embedding size")
    n4 = (N + 3) // 4 * 4
    out = torch.empty(Q, max(n4, 4), dtype=torch.float32, device=q.device)
    if Q == 0 or N == 0:
        return out[:, :N]
    e4 = (E + 3) // 4 * 4
    a = q.contiguous()
    if e4 != E:  # 16-B rows for the kernel's vector loads
        a = torch.zeros(Q, e4, dtype=torch.float32, device=q.device)
        a[:, :E] = q
    cc = c.contiguous()
    for j0 in range(0, N, chunk):
        j1 = min(N, j0 + chunk)
        img = mlp_pack(cc[j0:j1], trans=True)
        mlp_rows(a, img, E, j1 - j0, out[:, j0:j1])
    return out[:, :N]


def matmul_rows(a: torch.Tensor, b: torch.Tensor, chunk: int = 256) -> torch.Tensor:
    """a [M, K] . b [K, N] fp32 on libtt's bf16x3 row GEMM (tt_mlp_rows) for
    any K and N: b in (K-chunk x N-chunk) blocks of <= `chunk`, each packed as
    one B image; the K-chunk partials of an output block are added in chunk
    order (deterministic).  The backward GEMMs of ScoreMatrix."""
    _req(a, "a", torch.float32, 2)
    _req(b, "b", torch.float32, 2)
    M, K = a.shape
    if b.shape[0] != K:
        raise ValueError(f"a {tuple(a.shape)} and b {tuple(b.shape)} do not chain")
    N = b.shape[1]
    out = torch.zeros(M, max((N + 3) // 4 * 4, 4), dtype=torch.float32, device=a.device)
    if M == 0 or N == 0 or K == 0:
        return out[:, :N]
    k4 = (K + 3) // 4 * 4
    aa = a.contiguous()
    if k4 != K:  # 16-B rows (and 16-B aligned column chunks) for the kernel's vector loads
        aa = torch.zeros(M, k4, dtype=torch.float32, device=a.device)
        aa[:, :K] = a
    bb = b.contiguous()
    part = torch.empty(M, min(chunk, (N + 3) // 4 * 4), dtype=torch.float32, device=a.device)
    for n0 in range(0, N, chunk):
        n1 = min(N, n0 + chunk)
        for k0 in range(0, K, chunk):
            k1 = min(K, k0 + chunk)
            img = mlp_pack(bb[k0:k1, n0:n1].contiguous())
            mlp_rows(aa[:, k0:], img, k1 - k0, n1 - n0, part)
            out[:, n0:n1] += part[:, :n1 - n0]
    return out[:, :N]


class ScoreMatrix(torch.autograd.Function):
    """S = q . c^T with its gradients, every product on libtt (score_matrix
    forward; dq = G . c and dc = G^T . q by matmul_rows): the differentiable
    form of TwoTowerModel.call (two_tower_model.py:92, tf.matmul)."""

    @staticmethod
    def forward(ctx, q, c):
        ctx.save_for_backward(q, c)
        return score_matrix(q.detach(), c.detach())

    @staticmethod
    def backward(ctx, g):
        q, c = ctx.saved_tensors
        g = g.contiguous()
        dq = matmul_rows(g, c.detach()) if ctx.needs_input_grad[0] else None
        dc = matmul_rows(g.t().contiguous(), q.detach()) if ctx.needs_input_grad[1] else None
        return dq, dc


def _pack_job_array(jobs: Sequence[Tuple[torch.Tensor, bool, torch.Tensor]]):
    arr = (_native.MlpPackJob * len(jobs))()
    for i, (w, trans, img) in enumerate(jobs):
        _req(w, "w", torch.float32, 2)
        K, N = (w.shape[1], w.shape[0]) if trans else (w.shape[0], w.shape[1])
        arr[i].w, arr[i].ldw, arr[i].K, arr[i].N = w.data_ptr(), _row_major(w, "w"), K, N
        arr[i].trans, arr[i].img, arr[i].img_bytes = int(bool(trans)), img.data_ptr(), img.numel()
    return arr


def mlp_pack_many(jobs: Sequence[Tuple[torch.Tensor, bool, torch.Tensor]]) -> None:
    """Several mlp_pack images in one launch: jobs of (w, trans, image buffer)."""
    check(lib().tt_mlp_pack_many(_pack_job_array(jobs), len(jobs), _stream()))


def _check_rows(a, k, n, out, amask, cmask, bias) -> int:
    """mlp_rows' operand checks; returns M."""
    _req(a, "a", torch.float32, 2)
    _req(out, "out", torch.float32, 2)
    M = a.shape[0]
    if a.shape[1] < k or out.shape[0] != M or out.shape[1] < n:
        raise ValueError(f"mlp_rows: a {tuple(a.shape)}, out {tuple(out.shape)}, k={k}, n={n}")
    for t, nm in ((amask, "amask"), (cmask, "cmask")):
        if t is not None:
            _req(t, nm, torch.float32, 2)
            if t.shape[0] != M:
                raise ValueError(f"{nm} has {t.shape[0]} rows, expected {M}")
    if amask is not None and amask.shape[1] < k:
        raise ValueError("amask narrower than k")
    if cmask is not None and cmask.shape[1] < n:
        raise ValueError("cmask narrower than n")
    if bias is not None and (bias.dtype != torch.float32 or bias.numel() < n or not bias.is_contiguous()):
        raise ValueError("bias must be a contiguous fp32 vector of >= n entries")
    return M


def _ptr(t: Optional[torch.Tensor]):
    return t.data_ptr() if t is not None else None


def mlp_rows(a: torch.Tensor, img: torch.Tensor, k: int, n: int, out: torch.Tensor, *,
             amask: Optional[torch.Tensor] = None, scale: Optional[torch.Tensor] = None,
             bias: Optional[torch.Tensor] = None, relu: bool = False,
             cmask: Optional[torch.Tensor] = None, colsum: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[M, n] = epi(maskA(a[:, :k]) . B) with B packed by mlp_pack (tt_mlp_rows);
    colsum (a contiguous [n] tensor): also the column sums of out."""
    M = _check_rows(a, k, n, out, amask, cmask, bias)
    ws = None
    if colsum is not None:
        if colsum.dtype != torch.float32 or colsum.numel() != n or not colsum.is_contiguous():
            raise ValueError("colsum must be a contiguous fp32 [n] tensor")
        ws = Workspace.get(lib().tt_mlp_rows_workspace_size(M, n), a.device, "mlp_colsum")
    check(lib().tt_mlp_rows(a.data_ptr(), _row_major(a, "a"), _ptr(amask),
                            _row_major(amask, "amask") if amask is not None else 0,
                            _ptr(scale), M, k, img.data_ptr(), n, _ptr(bias), int(bool(relu)), _ptr(cmask),
                            _row_major(cmask, "cmask") if cmask is not None else 0, out.data_ptr(),
                            _row_major(out, "out"), _ptr(colsum), _ptr(ws), ws.numel() if ws is not None else 0,
                            _stream()))
    return out


def mlp_rows_pair(problems: Sequence[dict]) -> None:
    """Two independent mlp_rows problems (the two towers' layers) in ONE
    launch (tt_mlp_rows_pair); each problem is a dict of mlp_rows' arguments
    a, img, k, n, out and optionally amask, scale, bias, relu, cmask (no
    colsum).  Results equal two mlp_rows calls bit for bit."""
    if len(problems) != 2:
        raise ValueError("mlp_rows_pair takes exactly 2 problems")
    arr = (_native.MlpRowsProblem * 2)()
    for i, p in enumerate(problems):
        a, img, k, n, out = p["a"], p["img"], p["k"], p["n"], p["out"]
        amask, cmask, bias = p.get("amask"), p.get("cmask"), p.get("bias")
        M = _check_rows(a, k, n, out, amask, cmask, bias)
        q = arr[i]
        q.A, q.lda, q.amask = a.data_ptr(), _row_major(a, "a"), _ptr(amask)
        q.ldam = _row_major(amask, "amask") if amask is not None else 0
        q.scale, q.M, q.K, q.img, q.N = _ptr(p.get("scale")), M, k, img.data_ptr(), n
        q.bias, q.relu, q.cmask = _ptr(bias), int(bool(p.get("relu", False))), _ptr(cmask)
        q.ldcm = _row_major(cmask, "cmask") if cmask is not None else 0
        q.C, q.ldc = out.data_ptr(), _row_major(out, "out")
    check(lib().tt_mlp_rows_pair(arr, _stream()))


def _check_wgrad(a, g, dwb, gmask) -> Tuple[int, int, int]:
    _req(a, "a", torch.float32, 2)
    _req(g, "g", torch.float32, 2)
    _req(dwb, "dwb", torch.float32, 2)
    M, Ka = a.shape
    N = g.shape[1]
    if g.shape[0] != M or tuple(dwb.shape) != (Ka + 1, N) or not dwb.is_contiguous():
        raise ValueError(f"mlp_wgrad: a {tuple(a.shape)}, g {tuple(g.shape)}, dwb {tuple(dwb.shape)}")
    if gmask is not None:
        _req(gmask, "gmask", torch.float32, 2)
        if tuple(gmask.shape) != (M, N):
            raise ValueError("gmask must match g")
    return M, Ka, N


def mlp_wgrad(a: torch.Tensor, g: torch.Tensor, dwb: torch.Tensor, *, gmask: Optional[torch.Tensor] = None,
              scale: Optional[torch.Tensor] = None, adagrad: Optional[tuple] = None) -> torch.Tensor:
    """dwb [Ka + 1, N] = [a | 1]^T . Gm (weight gradient rows then the bias
    gradient row), Gm = g or (gmask > 0) ? g * scale : 0 (tt_mlp_wgrad).
    adagrad = (param, accum, lr, eps): also the layer's Adagrad step on
    param / accum (contiguous, dwb's shape) from the summed gradient
    (tt_mlp_wgrad_adagrad: dense_adagrad's arithmetic inside the sum launch)."""
    M, Ka, N = _check_wgrad(a, g, dwb, gmask)
    ws = Workspace.get(lib().tt_mlp_wgrad_workspace_size(M, Ka, N), a.device, "mlp_wgrad")
    args = (a.data_ptr(), _row_major(a, "a"), g.data_ptr(), _row_major(g, "g"), _ptr(gmask),
            _row_major(gmask, "gmask") if gmask is not None else 0, _ptr(scale), M, Ka, N, dwb.data_ptr())
    if adagrad is not None:
        param, accum, lr, eps = adagrad
        for t, n in ((param, "param"), (accum, "accum")):
            _req(t, n, torch.float32)
            if t.numel() != dwb.numel() or not t.is_contiguous():
                raise ValueError(f"{n} must be contiguous with dwb's {dwb.numel()} elements")
        check(lib().tt_mlp_wgrad_adagrad(*args, param.data_ptr(), accum.data_ptr(), float(lr), float(eps),
                                         ws.data_ptr(), ws.numel(), _stream()))
        return dwb
    check(lib().tt_mlp_wgrad(*args, ws.data_ptr(), ws.numel(), _stream()))
    return dwb


def mlp_wgrad_pair(problems: Sequence[dict]) -> None:
    """Two mlp_wgrad problems (dicts of a, g, dwb and optionally gmask,
    scale) in one launch plus one partial-sum launch (tt_mlp_wgrad_pair)."""
    if len(problems) != 2:
        raise ValueError("mlp_wgrad_pair takes exactly 2 problems")
    arr = (_native.MlpWgradProblem * 2)()
    for i, p in enumerate(problems):
        a, g, dwb, gmask = p["a"], p["g"], p["dwb"], p.get("gmask")
        M, Ka, N = _check_wgrad(a, g, dwb, gmask)
        q = arr[i]
        q.A, q.lda, q.G, q.ldg = a.data_ptr(), _row_major(a, "a"), g.data_ptr(), _row_major(g, "g")
        q.gmask, q.ldgm = _ptr(gmask), _row_major(gmask, "gmask") if gmask is not None else 0
        q.scale, q.M, q.Ka, q.N, q.dwb = _ptr(p.get("scale")), M, Ka, N, dwb.data_ptr()
    ws = Workspace.get(lib().tt_mlp_wgrad_pair_workspace_size(arr), problems[0]["a"].device, "mlp_wgrad")
    check(lib().tt_mlp_wgrad_pair(arr, ws.data_ptr(), ws.numel(), _stream()))
