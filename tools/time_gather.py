"""Times the C3 step's tt_gather_multi (both towers, one launch) with HIP
events over a graph of 50 launches: bench.time_gather on its own."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
model, data = bench.build_model(dev, 0)
r = bench.time_gather(model, data, dev, 16384)
print(f"gather {r['ms_per_launch'] * 1e3:.2f} us  {r['achieved']:.0f} GB/s  frac {r['frac']:.3f}", flush=True)
u = bench.time_gather_uniform(model, dev, 16384, c5_rows=0) if "--uniform" in sys.argv else None
if u:
    print(f"uniform {u['ms_per_launch'] * 1e3:.2f} us  {u['achieved']:.0f} GB/s  frac {u['frac']:.3f}", flush=True)
