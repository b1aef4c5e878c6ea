"""Times the C3 step's fused in-batch entry (tt_inbatch_softmax_xent) and its
two pass kernels with HIP events: bench.time_inbatch_kernel on its own."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
model, data = bench.build_model(dev, 0)
flops, (ms_rows, ms_rows_1), (ms_cols, ms_cols_1), ms_entry = bench.time_inbatch_kernel(model, data, dev, 16384)
print(f"entry {ms_entry * 1e3:.1f} us  rows {ms_rows * 1e3:.1f} us ({flops / ms_rows / 1e9 / 2500:.3f} of peak; "
      f"{ms_rows_1 * 1e3:.1f} with an event pair per launch)  cols {ms_cols * 1e3:.1f} us ({ms_cols_1 * 1e3:.1f})",
      flush=True)
