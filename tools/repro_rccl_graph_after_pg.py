"""Reproduction of the round-4 hipGraphLaunch segfault.

1. A one-rank RCCL process group; a ShardedTrainStep whose captured graph
   holds real RCCL collectives (BatchComm(always=True)) takes 4 steps.
2. The process group is destroyed, then the step (and its graph) is
   released:  --order old  with torch.distributed.destroy_process_group and
   the graph destroyed afterwards (what the tests did);  --order fixed  with
   pkg.modelling.distributed.destroy_process_group (graph released first).
3. An unrelated model trains with the graphed DeviceDataset fit (2 epochs).

Usage: python tools/repro_rccl_graph_after_pg.py --order old|fixed
"""
import argparse
import gc
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pkg import dtypes  # noqa: E402
from pkg.modelling import distributed  # noqa: E402
from pkg.modelling.dataset import DeviceDataset  # noqa: E402
from pkg.modelling.models.two_tower_model import TwoTowerModel  # noqa: E402
from pkg.modelling.optimizer_factory import OptimizerFactory  # noqa: E402
from pkg.schema.features import Feature, FeatureFamily  # noqa: E402


def model(dev, seed):
    V = [str(i) for i in range(300)]
    qf = [Feature("cust", dtypes.string, FeatureFamily.QUERY, embedding_size=16, vocab=V),
          Feature("post", dtypes.string, FeatureFamily.QUERY, embedding_size=8, vocab=V[:50])]
    cf = [Feature("art", dtypes.string, FeatureFamily.CANDIDATE, embedding_size=16, vocab=V),
          Feature("ptn", dtypes.string, FeatureFamily.CANDIDATE, embedding_size=8, vocab=V[:20])]
    probs = {str(i): float(p) for i, p in enumerate(np.random.default_rng(seed).dirichlet(np.ones(300)))}
    m = TwoTowerModel(qf, cf, "art", 32, [64], [48], probs, device=dev, seed=seed)
    m.compile(optimizer=OptimizerFactory.get_optimizer("adagrad", {"learning_rate": 0.05}))
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--order", choices=("old", "fixed"), required=True)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    rng = np.random.default_rng(1)
    step = distributed.ShardedTrainStep(model(dev, 5), shard_min_rows=300, global_negatives=True,
                                        comm=distributed.BatchComm(always=True))
    for _ in range(4):
        z = lambda v: torch.as_tensor((rng.zipf(1.3, 4096) % v).astype(np.int32), device=dev)
        step({"cust": z(301), "post": z(51), "art": z(301), "ptn": z(21)})
    torch.cuda.synchronize()
    assert step._graph is not None
    if args.order == "old":
        dist.destroy_process_group()
    else:
        distributed.destroy_process_group()
    del step
    gc.collect()
    print(f"[{args.order}] sharded step released; graphed DeviceDataset fit next", flush=True)
    n = 2600
    cols = {"cust": (rng.zipf(1.3, n) % 301).astype(np.int32), "post": (rng.zipf(1.3, n) % 51).astype(np.int32),
            "art": (rng.zipf(1.3, n) % 301).astype(np.int32), "ptn": rng.integers(0, 21, n).astype(np.int32)}
    h = model(dev, 3).fit(DeviceDataset(cols, 512, 1000, seed=7, device=dev), epochs=2, use_graph=True)
    torch.cuda.synchronize()
    print(f"[{args.order}] fit ok: {h['loss']}", flush=True)


if __name__ == "__main__":
    main()
