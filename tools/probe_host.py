"""Host-side cost probe: how long the host spends inside one hipGraph replay
of the C3 train step versus the GPU time of the step, and the host cost of
small torch ops.  Diagnostic only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from pkg.modelling.models.two_tower_model import GraphedTrainStep  # noqa: E402

dev = torch.device("cuda", 0)
model, data = bench.build_model(dev, 0)
pool = [data.batch(16384) for _ in range(2)]
step = GraphedTrainStep(model, pool[0], warmup=2)
torch.cuda.synchronize()
for _ in range(5):
    step.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
hs = []
for _ in range(20):
    a = time.perf_counter()
    step.replay()
    hs.append(time.perf_counter() - a)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"replay host us: min {min(hs)*1e6:.1f} median {sorted(hs)[10]*1e6:.1f}; 20 replays host {(t1-t0)*1e6:.0f} us, "
      f"wall incl sync {(t2-t0)*1e6:.0f} us")
x = torch.zeros(1000, device=dev)
torch.cuda.synchronize()
a = time.perf_counter()
for _ in range(200):
    x.add_(1)
b = time.perf_counter()
torch.cuda.synchronize()
print(f"torch add_ host us/op: {(b-a)/200*1e6:.1f}")
