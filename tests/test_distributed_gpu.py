"""Candidate-sharded index on the GPU with the libtt kernels under real
sharding: world 1, 2 and 3 processes on cuda:0 (gloo, collectives staged
through the host), each rank screening its own candidate rows; every rank's
answer must equal the single-GPU search bit for bit, and the oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, c, q, k, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "hm-retrieval-two-tower_amd")]
    from pkg.modelling.distributed import ShardedBruteForceIndex

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    idx = ShardedBruteForceIndex(k, None, torch.as_tensor(c, device=dev))
    s, i = idx.search(torch.as_tensor(q, device=dev))
    (b, e), os_, oi = idx.search_owned(torch.as_tensor(q, device=dev))
    torch.cuda.synchronize()
    out[rank] = (s.cpu().numpy(), i.cpu().numpy(), (b, e), os_.cpu().numpy(), oi.cpu().numpy(), idx.rows)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,signed", [(1, False), (2, False), (3, False), (2, True)])
def test_candidate_sharded_index_hip(cuda, world, signed):
    from oracle import oracle
    from pkg.modelling import hip_ops

    rng = np.random.default_rng(40 + world)
    N, Q, E, k = 20011, 1500, 128, 100
    c = rng.standard_normal((N, E)).astype(np.float32)
    q = rng.standard_normal((Q, E)).astype(np.float32)
    if not signed:
        c, q = np.maximum(c, 0), np.maximum(q, 0)
    c[15000:15030] = c[20:50]  # exact ties across shards resolve by global index
    q[::50] = 0.0              # zero queries: every score ties at 0
    tc = torch.as_tensor(c, device=cuda)
    ref_s, ref_i = hip_ops.bruteforce_search(hip_ops.bruteforce_build(tc), tc, torch.as_tensor(q, device=cuda), k)
    ref_s, ref_i = ref_s.cpu().numpy(), ref_i.cpu().numpy()
    sel = np.arange(0, Q, 7)
    os_, oi_, _ = oracle.bruteforce_topk(q[sel], c, k)
    assert np.array_equal(ref_i[sel], oi_) and np.array_equal(ref_s[sel], os_)
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _free_port(), c, q, k, out), nprocs=world, join=True)
    rows = []
    for r in range(world):
        s, i, (b, e), bs, bi, rr = out[r]
        rows.append(rr)
        assert np.array_equal(i, ref_i) and np.array_equal(s, ref_s)
        assert np.array_equal(bi, ref_i[b:e]) and np.array_equal(bs, ref_s[b:e])
    assert rows[0][0] == 0 and rows[-1][1] == N


def _small_model(dev, seed):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "hm-retrieval-two-tower_amd")]
    from pkg import dtypes
    from pkg.modelling.models.two_tower_model import TwoTowerModel
    from pkg.modelling.optimizer_factory import OptimizerFactory
    from pkg.schema.features import Feature, FeatureFamily

    V = [str(i) for i in range(300)]
    qf = [Feature("cust", dtypes.string, FeatureFamily.QUERY, embedding_size=16, vocab=V),
          Feature("post", dtypes.string, FeatureFamily.QUERY, embedding_size=8, vocab=V[:50])]
    cf = [Feature("art", dtypes.string, FeatureFamily.CANDIDATE, embedding_size=16, vocab=V),
          Feature("ptn", dtypes.string, FeatureFamily.CANDIDATE, embedding_size=8, vocab=V[:20])]
    rng = np.random.default_rng(seed)
    probs = {str(i): float(p) for i, p in enumerate(rng.dirichlet(np.ones(300)))}
    m = TwoTowerModel(qf, cf, "art", 32, [64], [64], probs, device=dev, seed=seed)
    m.compile(optimizer=OptimizerFactory.get_optimizer("adagrad", {"learning_rate": 0.05}))
    return m


def _global_batches(steps, B):
    rng = np.random.default_rng(11)
    z = lambda v: (rng.zipf(1.3, B) % v).astype(np.int32)
    return [{"cust": z(301), "post": z(51), "art": z(301), "ptn": z(21)} for _ in range(steps)]


def _step_worker(rank, world, port, batches, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    m = _small_model(dev, 3)
    from pkg.modelling.distributed import ShardedTrainStep

    step = ShardedTrainStep(m, shard_min_rows=300, global_negatives=True)
    losses = []
    for gb in batches:
        b = len(gb["cust"]) // world
        local = {k: torch.as_tensor(v[rank * b:(rank + 1) * b], device=dev) for k, v in gb.items()}
        losses.append(float(step(local)["loss"].item()))
    tables = {}
    for ti, t in enumerate(m.towers):
        for name, e in t.input_layer.embedding_layers.items():
            full = step.tables.gather_full(e._shard_key) if hasattr(e, "_shard_key") else e.weight
            tables[(ti, name)] = full.cpu().numpy()
    out[rank] = (losses, [t.dense.flat.detach().cpu().numpy() for t in m.towers], tables)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_global_negatives_sharded_step_matches_full_batch(cuda, world):
    """ShardedTrainStep(global_negatives=True) on `world` ranks (libtt
    kernels, row-sharded tables, gloo through the host, all on cuda:0) trains
    like ONE model on the concatenated global batch: the loss of every step
    and the final MLP and embedding parameters match the single-GPU step
    within fp32 summation-order rounding (the reduce_scatter / all_reduce sum
    the same terms in another order)."""
    steps, B = 3, 64 * world
    batches = _global_batches(steps, B)
    ref = _small_model(cuda, 3)
    ref_losses = [float(ref.train_step({k: torch.as_tensor(v, device=cuda) for k, v in gb.items()})["loss"].item())
                  for gb in batches]
    out = mp.Manager().dict()
    mp.spawn(_step_worker, args=(world, _free_port(), batches, out), nprocs=world, join=True)
    for r in range(world):
        losses, flats, tables = out[r]
        np.testing.assert_allclose(losses, ref_losses, rtol=2e-5)
        for fl, t in zip(flats, ref.towers):
            np.testing.assert_allclose(fl, t.dense.flat.detach().cpu().numpy(), rtol=1e-4, atol=2e-6)
        for ti, t in enumerate(ref.towers):
            for name, e in t.input_layer.embedding_layers.items():
                np.testing.assert_allclose(tables[(ti, name)], e.weight.cpu().numpy(), rtol=1e-4, atol=2e-6)
