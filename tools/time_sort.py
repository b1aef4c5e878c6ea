"""Isolated timing of the embedding update's id sort (tt_sparse_sort) on the
bench's C3 tables: every table alone and all of them in one call, HIP events
over graph replays.  usage: python tools/time_sort.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pkg.modelling import hip_ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model, data = bench.build_model(dev, 0)
    B = 16384
    batch = data.batch(B)
    model.train_step(batch)
    torch.cuda.synchronize()
    specs, b = model.optimizer._sparse_specs(model.towers, with_grad=False)
    for s in specs:
        print(f"table rows={s['table'].shape[0]} dim={s['table'].shape[1]} sources={len(s['ids'])}")
    cases = [([s], f"rows={s['table'].shape[0]}x{len(s['ids'])}") for s in specs] + [(specs, "all")]
    for sp, name in cases:
        ms = bench._graph_time(lambda: hip_ops.sparse_sort(sp, b), 50)
        print(f"{name:>22s} {ms * 1e3:8.1f} us")


if __name__ == "__main__":
    main()
