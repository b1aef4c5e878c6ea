import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd")]
import numpy as np, torch
from pkg.modelling import hip_ops
dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
def t(fn, reps=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3
for n, V, D, a in ((16384, 200, 4, 1.1), (16384, 60000, 128, 1.1), (16384, 1371980, 128, 0.6), (16384, 105542, 128, 1.1), (32768, 131, 4, 1.1)):
    ids = torch.as_tensor(((rng.zipf(1 + a, n) - 1) % V).astype(np.int32), device=dev) if a > 1 else torch.as_tensor(rng.integers(0, V, n).astype(np.int32), device=dev)
    g = torch.randn(n, D, device=dev)
    tab = torch.zeros(V, D, device=dev); acc = torch.full_like(tab, 0.1)
    spec = [dict(table=tab, slot0=acc, ids=[ids], grad_col_offset=[0])]
    us = t(lambda: hip_ops.sparse_adagrad(spec, n, g, 0.05, 1e-7))
    print(f"n={n} V={V} D={D}: sparse_adagrad {us:.1f} us, unique={len(torch.unique(ids))}")
