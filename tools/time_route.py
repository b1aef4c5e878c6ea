"""Times tt_route_fixed (the ShardedTrainStep's route: 3 sharded lookups,
Zipf ids, world 1, owner view + sorted order) with HIP events, and with a
TT_ROUTE_STAMPS build (TT_LIB_PATH) prints the fused kernel's phase times.

usage: [TT_ROUTE_FUSED=0] [TT_LIB_PATH=...] python tools/time_route.py [B] [reps]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd")]
import torch  # noqa: E402

from pkg import _native  # noqa: E402
from pkg.modelling import hip_ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
rows = [1371980, 352899, 105542]
ids = [torch.as_tensor(((rng.zipf(1.05, B) - 1) % r).astype(np.int32), device=dev) for r in rows]
lookups = [(x, r, t) for t, (x, r) in enumerate(zip(ids, rows))]
for variant in ("full", "plain"):
    kw = dict(ordered=True, owner=True) if variant == "full" else {}
    hip_ops.route_fixed(lookups, 1, 3, 3 * B, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        hip_ops.route_fixed(lookups, 1, 3, 3 * B, **kw)
    e1.record()
    torch.cuda.synchronize()
    print(f"route_fixed B={B} {variant} fused={os.environ.get('TT_ROUTE_FUSED', '1')}: "
          f"{e0.elapsed_time(e1) / reps * 1e3:.1f} us per call (back to back, host launch included)")
fn = getattr(_native.lib(), "tt_route_stamps", None) if hasattr(_native.lib(), "tt_route_stamps") else None
if fn is not None:
    st = (ctypes.c_ulonglong * 8)()
    fn(st)
    t = [st[i] for i in range(8)]
    names = ["keys", "sort", "requests+scan", "slot writes", "padding+counts"]
    marks = [t[5], t[0], t[1], t[2], t[3], t[4]]
    print("phases (us, 100 MHz wall clock): " + ", ".join(
        f"{n} {(marks[i + 1] - marks[i]) / 100:.1f}" for i, n in enumerate(names)))
