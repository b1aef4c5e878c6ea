"""Times tt_bruteforce_search on BASELINE configs[3]'s shape (105,542 x 128
relu(N(0,1)) candidates, 262,144 queries, 1 % zero, top-100) with the screen
and finalize kernels bracketed by HIP events (tt_probe_arm)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd")]
import torch  # noqa: E402

from pkg.modelling import hip_ops  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
g.manual_seed(1)
C = torch.relu(torch.randn(105542, 128, generator=g, device=dev))
g.manual_seed(2)
Q = torch.relu(torch.randn(262144, 128, generator=g, device=dev))
Q[::100] = 0.0
img = hip_ops.bruteforce_build(C)
s0, i0 = hip_ops.bruteforce_search(img, C, Q[:65536], 100)
torch.cuda.synchronize()
ts = []
for _ in range(3):
    t0 = time.perf_counter()
    s, i = hip_ops.bruteforce_search(img, C, Q, 100)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
same = bool(torch.equal(i[:65536], i0) and torch.equal(s[:65536], s0))
print(f"search {min(ts) * 1e3:.2f} ms  {262144 / min(ts) / 1e6:.2f} M QPS  consistent={same}", flush=True)
