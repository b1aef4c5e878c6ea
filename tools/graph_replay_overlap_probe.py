"""Probe: do back-to-back replays of one hipGraph overlap on the device?

A captured graph writes a small temporary t (= 5), folds it into a running
max y, frees it, then allocates a block of the same size (the caching
allocator hands back t's block) and fills it with a large value.  In capture
order nothing ever reads the large value through t.  If replay N+1's first
nodes ran while replay N's last nodes still ran (or the nodes of one replay
ran out of order), y would pick the large value up.  Variants: a linear
graph, and the same with a forked branch (side stream, joined from the
origin) that does unrelated work.  Each variant: 2000 replays back to back,
one sync at the end.  Then the same with the temporary zeroed by a
captured hipMemsetAsync (a memset node) before a kernel adds to it.

usage: python tools/graph_replay_overlap_probe.py
"""
import torch

dev = torch.device("cuda:0")
big = torch.ones(1 << 22, device=dev)  # some real work per replay


def run(fork: bool, reps: int = 2000) -> int:
    y = torch.zeros(1, dtype=torch.int64, device=dev)
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        big.mul_(1.0)
        t = torch.full((1,), 5, dtype=torch.int64, device=dev)
        if fork:
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                big.add_(0.0)
        torch.maximum(y, t, out=y)
        del t
        u = torch.empty(1, dtype=torch.int64, device=dev)  # t's block again
        u.fill_(1 << 40)
        big.mul_(1.0)
        if fork:
            torch.cuda.current_stream().wait_stream(side)
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return int(y.item())


def run_memset(reps: int = 2000, keep: bool = False) -> int:
    """As run(), with the temporary zeroed by hipMemsetAsync (a captured
    memset NODE, as tt_route_requests zeroes its per-owner counts) and then
    incremented by a kernel before it is read."""
    import ctypes
    import os

    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    y = torch.zeros(1, dtype=torch.int64, device=dev)
    g = torch.cuda.CUDAGraph()
    kept = []
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        big.mul_(1.0)
        t = torch.empty(1, dtype=torch.int64, device=dev)
        assert hip.hipMemsetAsync(t.data_ptr(), 0, 8, torch.cuda.current_stream().cuda_stream) == 0
        t.add_(5)
        torch.maximum(y, t, out=y)
        if keep:
            kept.append(t)
        del t
        u = torch.empty(1, dtype=torch.int64, device=dev)  # t's block again (unless kept)
        u.fill_(1 << 40)
        big.mul_(1.0)
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return int(y.item())


for fork in (False, True):
    v = run(fork)
    print(f"fork={fork}: running max {v} ({'OVERLAP / reorder seen' if v != 5 else 'ordered'})", flush=True)
for keep in (True, False):
    v = run_memset(keep=keep)
    print(f"memset node, temporary kept={keep}: running max {v} "
          f"({'memset node mis-ordered' if v != 5 else 'ordered'})", flush=True)
