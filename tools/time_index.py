"""Times tt_bruteforce_search on BASELINE configs[3]'s shape (105,542 x 128
relu(N(0,1)) candidates, 1 % zero queries, top-k) end to end with HIP events
on the current stream, after a warm-up call of the same size (workspace
allocated outside the timed region).

usage: python tools/time_index.py [n_queries] [k] [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd")]
import torch  # noqa: E402

from pkg.modelling import hip_ops  # noqa: E402

nq = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
k = int(sys.argv[2]) if len(sys.argv) > 2 else 100
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
g.manual_seed(1)
C = torch.relu(torch.randn(105542, 128, generator=g, device=dev))
g.manual_seed(2)
Q = torch.relu(torch.randn(nq, 128, generator=g, device=dev))
Q[::100] = 0.0
img = hip_ops.bruteforce_build(C)
s0, i0 = hip_ops.bruteforce_search(img, C, Q, k)  # warm: workspace + code
torch.cuda.synchronize()
ts = []
for _ in range(reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    s, i = hip_ops.bruteforce_search(img, C, Q, k)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e-3)
same = bool(torch.equal(i, i0) and torch.equal(s, s0))
t = min(ts)
tf = 2.0 * nq * 105542 * 128 / t / 1e12
print(f"search nq={nq} k={k}: {t * 1e3:.2f} ms  {nq / t / 1e6:.2f} M QPS  {tf:.0f} TF/s "
      f"({tf / 2500:.3f} of bf16 peak)  consistent={same}", flush=True)
