"""Torch restatements of libtt's request routing (tt_route_requests,
tt_route_pad, tt_route_owner; csrc/tt_route.hip): test infrastructure only —
the gloo tests inject them into distributed.EmbeddingOps, the GPU tests hold
the kernels to them element for element."""
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch


def torch_route_requests(lookups: List[Tuple[torch.Tensor, int, int]], world: int, num_tags: int,
                         ordered: bool = False):
    """Restatement of tt_route_requests in torch ops (the CPU/gloo tests'
    implementation): (send [R, 2], counts [world] int64, num_requests [1],
    idx [L, B]); ordered=True appends tt_route_requests_ordered's (order,
    grp_first, grp_last)."""
    dev = lookups[0][0].device
    B = lookups[0][0].numel()
    by_tag: Dict[int, List[int]] = {}
    for i, (_, _, tag) in enumerate(lookups):
        by_tag.setdefault(tag, []).append(i)
    req_ids, req_tags, inverse, starts = [], [], {}, {}
    off = 0
    for tag in sorted(by_tag):
        rows = lookups[by_tag[tag][0]][1]
        ids = torch.cat([lookups[i][0].reshape(-1) for i in by_tag[tag]])
        ids = torch.where((ids >= 0) & (ids < rows), ids, torch.full_like(ids, -1))
        uniq, inv = torch.unique(ids, sorted=True, return_inverse=True)
        req_ids.append(uniq.to(torch.int32))
        req_tags.append(torch.full_like(uniq, tag, dtype=torch.int32))
        inverse[tag] = inv
        starts[tag] = off
        off += uniq.numel()
    req_ids = torch.cat(req_ids)
    req_tags = torch.cat(req_tags)
    R = req_ids.numel()
    owner = torch.remainder(req_ids, world)  # invalid (-1) ids go to rank world-1
    owner_sorted, perm = torch.sort(owner.to(torch.int64), stable=True)
    send = torch.stack([req_ids[perm], req_tags[perm]], 1).contiguous()
    counts = torch.bincount(owner_sorted, minlength=world).to(torch.int64)
    inv_perm = torch.empty_like(perm)
    inv_perm[perm] = torch.arange(R, device=dev)
    idx = torch.empty(len(lookups), B, dtype=torch.int32, device=dev)
    pos: Dict[int, int] = {}
    for i, (ids, _, tag) in enumerate(lookups):
        k = pos.get(tag, 0)
        u = inverse[tag][k:k + B]
        pos[tag] = k + B
        idx[i] = inv_perm[starts[tag] + u].to(torch.int32)
    nreq = torch.tensor([R], dtype=torch.int32, device=dev)
    if not ordered:
        return send, counts, nreq, idx
    # the route's sort: lookups by (owner, tag, row + 1), stable in lookup order
    keys = []
    for ids, rows, tag in lookups:
        r = ids.reshape(-1).to(torch.int64)
        ok = (r >= 0) & (r < rows)
        owner = torch.where(ok, torch.remainder(r, world), torch.full_like(r, world - 1))
        keys.append(((owner * num_tags + tag) << 32) | torch.where(ok, r + 1, torch.zeros_like(r)))
    keys = torch.cat(keys)
    order = torch.sort(keys, stable=True)[1]
    g = (keys[order] >> 32).tolist()
    first = torch.zeros(world * num_tags, dtype=torch.int32)
    last = torch.full((world * num_tags,), -1, dtype=torch.int32)
    for p, gg in enumerate(g):
        if p == 0 or g[p - 1] != gg:
            first[gg] = p
        last[gg] = p
    return send, counts, nreq, idx, (order.to(torch.int32).to(dev), first.to(dev), last.to(dev))


def torch_route_pad(send: torch.Tensor, counts: torch.Tensor, idx: torch.Tensor, world: int, cap: int,
                    overflow: Optional[torch.Tensor] = None):
    """Restatement of tt_route_pad in torch ops (the CPU/gloo tests'
    implementation): (send_padded [world*cap, 2], idx_padded)."""
    c = [int(v) for v in counts.tolist()]
    start = np.concatenate([[0], np.cumsum(c)]).astype(np.int64)
    send_p = torch.full((world * cap, 2), -1, dtype=torch.int32, device=send.device)
    for o in range(world):
        n = min(c[o], cap)
        send_p[o * cap:o * cap + n] = send[start[o]:start[o] + n]
    st = torch.as_tensor(start[:-1], device=idx.device)
    u = idx.reshape(-1).to(torch.int64)
    own = torch.searchsorted(st, u, right=True) - 1
    j = u - st[own]
    if overflow is not None:
        overflow += sum(max(0, v - cap) for v in c)
    # a dropped request (j >= cap) gets the sentinel -1 - owner (tt_route_pad)
    slot = torch.where(j < cap, own * cap + j, -1 - own)
    return send_p, slot.to(torch.int32).reshape(idx.shape)


def torch_route_owner(recv: torch.Tensor, world: int, num_tags: int):
    tags = recv[:, 1].contiguous()
    gid = recv[:, 0]
    rows = torch.where(gid >= 0, torch.div(gid, world, rounding_mode="floor"), torch.full_like(gid, -1))
    rows = rows.to(torch.int32).contiguous()
    tids = torch.stack([torch.where(tags == t, rows, torch.full_like(rows, -1)) for t in range(num_tags)])
    return tags, rows, tids.reshape(num_tags, -1)
