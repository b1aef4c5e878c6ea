"""Candidate-sharded index on the GPU with the libtt kernels under real
sharding: world 1, 2, 3 and 8 processes on cuda:0 (gloo, collectives staged
through the host), each rank handed ONLY its block of candidate rows; every
rank's answer must equal the single-GPU search bit for bit, and the oracle.
The 8-way case is configs[3]'s layout (N = 105,542 H&M articles, top-100)."""
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
    from pkg.modelling.distributed import ShardedBruteForceIndex, shard_range

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    b, e = shard_range(c.shape[0], world, rank)
    idx = ShardedBruteForceIndex(k, None, torch.as_tensor(c[b:e], device=dev))  # this rank's rows only
    s, i = idx.search(torch.as_tensor(q, device=dev))
    (qb, qe), os_, oi = idx.search_owned(torch.as_tensor(q, device=dev))
    torch.cuda.synchronize()
    out[rank] = (s.cpu().numpy(), i.cpu().numpy(), (qb, qe), os_.cpu().numpy(), oi.cpu().numpy(), idx.rows,
                 int(idx.shard.shape[0]), idx.num_candidates)
    dist.destroy_process_group()


def _check_sharded(cuda, world, c, q, k):
    from oracle import oracle
    from pkg.modelling import hip_ops

    N, Q = c.shape[0], q.shape[0]
    tc = torch.as_tensor(c, device=cuda)
    ref_s, ref_i = hip_ops.bruteforce_search(hip_ops.bruteforce_build(tc), tc, torch.as_tensor(q, device=cuda), k)
    ref_s, ref_i = ref_s.cpu().numpy(), ref_i.cpu().numpy()
    sel = np.arange(0, Q, 7)
    os_, oi_, _ = oracle.bruteforce_topk(q[sel], c, k)
    assert np.array_equal(ref_i[sel], oi_) and np.array_equal(ref_s[sel], os_)
    del tc
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _free_port(), c, q, k, out), nprocs=world, join=True)
    rows = []
    for r in range(world):
        s, i, (b, e), bs, bi, rr, held, n = out[r]
        rows.append(rr)
        assert n == N and held == rr[1] - rr[0] and (world == 1 or held < N)
        assert np.array_equal(i, ref_i) and np.array_equal(s, ref_s)
        assert np.array_equal(bi, ref_i[b:e]) and np.array_equal(bs, ref_s[b:e])
    assert rows[0][0] == 0 and rows[-1][1] == N


@pytest.mark.parametrize("world,signed", [(1, False), (2, False), (3, False), (2, True)])
def test_candidate_sharded_index_hip(cuda, world, signed):
    rng = np.random.default_rng(40 + world)
    N, Q, E, k = 20011, 1500, 128, 100
    c = rng.standard_normal((N, E)).astype(np.float32)
    q = rng.standard_normal((Q, E)).astype(np.float32)
    if not signed:
        c, q = np.maximum(c, 0), np.maximum(q, 0)
    c[15000:15030] = c[20:50]  # exact ties across shards resolve by global index
    q[::50] = 0.0              # zero queries: every score ties at 0
    _check_sharded(cuda, world, c, q, k)


def test_candidate_sharded_index_c4_eight_shards(cuda):
    """configs[3] at its stated 8-way candidate sharding: N = 105,542
    candidates (relu(N(0,1)), the towers' final ReLU), 2048 queries with 1 %
    all-zero rows, top-100; eight processes on cuda:0, ~13.2k rows each."""
    rng = np.random.default_rng(8)
    N, Q, E, k = 105542, 2048, 128, 100
    c = np.maximum(rng.standard_normal((N, E)), 0).astype(np.float32)
    q = np.maximum(rng.standard_normal((Q, E)), 0).astype(np.float32)
    q[rng.choice(Q, Q // 100, replace=False)] = 0.0
    c[13200:13240] = c[40:80]  # duplicate rows straddling the first shard boundary
    _check_sharded(cuda, 8, c, q, k)


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


def _sharded_state(step, m):
    """Every parameter and Adagrad accumulator of the sharded step's model,
    reassembled full-size on every rank: tower MLP buffers, small tables
    (views of the step's flat buffers), row-sharded tables (gather_full)."""
    flats = [(t.dense.flat.detach().cpu().numpy().copy(), step._dense_acc[ti].cpu().numpy().copy())
             for ti, t in enumerate(m.towers)]
    tables = {}
    for ti, t in enumerate(m.towers):
        for name, e in t.input_layer.embedding_layers.items():
            if hasattr(e, "_shard_key"):
                w = step.tables.gather_full(e._shard_key)
                a = step.tables.gather_full(e._shard_key, accumulator=True)
            else:
                off = (e.weight.data_ptr() - step._small_flat.data_ptr()) // 4
                w = e.weight
                a = step._small_acc[off:off + w.numel()].view_as(w)
            tables[(ti, name)] = (w.cpu().numpy().copy(), a.cpu().numpy().copy())
    return flats, tables


def _step_worker(rank, world, port, batches, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    m = _small_model(dev, 3)
    from pkg.modelling.distributed import ShardedTrainStep

    step = ShardedTrainStep(m, shard_min_rows=300, global_negatives=True)
    states, losses = [_sharded_state(step, m)], []
    for gb in batches:
        b = len(gb["cust"]) // world
        local = {k: torch.as_tensor(v[rank * b:(rank + 1) * b], device=dev) for k, v in gb.items()}
        losses.append(float(step(local)["loss"].item()))
        states.append(_sharded_state(step, m))
    out[rank] = (losses, states)
    dist.destroy_process_group()


def _load_state(ref, state):
    """The single-GPU model `ref` set to a state of the sharded step
    (parameters and Adagrad accumulators)."""
    flats, tables = state
    opt = ref.optimizer
    with torch.no_grad():
        for ti, t in enumerate(ref.towers):
            t.dense.flat.copy_(torch.as_tensor(flats[ti][0]))
            opt._slots[id(t.dense.flat)] = [torch.as_tensor(flats[ti][1], device=t.dense.flat.device)]
            for name, e in t.input_layer.embedding_layers.items():
                w, a = tables[(ti, name)]
                e.weight.copy_(torch.as_tensor(w))
                opt._slots[id(e.weight)] = [torch.as_tensor(a, device=e.weight.device)]


@pytest.mark.parametrize("world", [2, 4])
def test_global_negatives_sharded_step_matches_full_batch(cuda, world):
    """ShardedTrainStep(global_negatives=True) on `world` ranks (libtt
    kernels, row-sharded tables, gloo through the host, all on cuda:0) trains
    like ONE model on the concatenated global batch, step by step: the
    single-GPU model, set to the sharded step's full state (parameters and
    Adagrad accumulators, reassembled) before step s, takes one train step on
    the global batch, and the sharded step's loss and state after step s must
    match it.  The two differ only in fp32 summation order (the in-batch
    passes' column splits, the MLP weight gradients' row splits, the
    all_reduce): ~1e-7 relative per gradient.  One Adagrad update moves a
    parameter by lr g / sqrt(a + g^2), whose slope in g is at most
    lr / sqrt(a) <= 0.05 / sqrt(0.1) = 0.16, so the updates differ by
    ~1e-8-1e-7 for the O(0.1-1) gradients here: atol 2e-6 per step.  Every
    step restarts the reference from the sharded state, so nothing compounds
    (a trajectory comparison would measure the drift of two chaotic runs)."""
    steps, B = 3, 64 * world
    batches = _global_batches(steps, B)
    out = mp.Manager().dict()
    mp.spawn(_step_worker, args=(world, _free_port(), batches, out), nprocs=world, join=True)
    losses0, states0 = out[0]
    for r in range(1, world):  # every rank reassembles the same state
        losses, states = out[r]
        assert losses == losses0
        for (fa, ta), (fb, tb) in zip(states, states0):
            assert all(np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]) for x, y in zip(fa, fb))
            assert all(np.array_equal(ta[k][0], tb[k][0]) and np.array_equal(ta[k][1], tb[k][1]) for k in ta)
    ref = _small_model(cuda, 3)
    for s, gb in enumerate(batches):
        _load_state(ref, states0[s])
        ref_loss = float(ref.train_step({k: torch.as_tensor(v, device=cuda) for k, v in gb.items()})["loss"].item())
        np.testing.assert_allclose(losses0[s], ref_loss, rtol=2e-5)
        flats, tables = states0[s + 1]
        opt = ref.optimizer
        for ti, t in enumerate(ref.towers):
            np.testing.assert_allclose(flats[ti][0], t.dense.flat.detach().cpu().numpy(), rtol=0, atol=2e-6)
            np.testing.assert_allclose(flats[ti][1], opt._slots[id(t.dense.flat)][0].cpu().numpy(), rtol=1e-5)
            for name, e in t.input_layer.embedding_layers.items():
                np.testing.assert_allclose(tables[(ti, name)][0], e.weight.cpu().numpy(), rtol=0, atol=2e-6)
                np.testing.assert_allclose(tables[(ti, name)][1], opt._slots[id(e.weight)][0].cpu().numpy(),
                                           rtol=1e-5)


def _integration_worker(rank, world, port, code, C, batches, qemb, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    model = _small_model(dev, 3)
    b = len(batches["cust"]) // world
    env = {"model": model, "C": torch.as_tensor(C), "N": C.shape[0],
           "local_batch": {k: torch.as_tensor(v[rank * b:(rank + 1) * b], device=dev) for k, v in batches.items()},
           "query_embeddings": torch.as_tensor(qemb, device=dev)}
    exec(code, env)
    torch.cuda.synchronize()
    out[rank] = (env["scores"].cpu().numpy(), env["ids"].cpu().numpy(), float(env["out"]["loss"].item()),
                 int(env["index"].shard.shape[0]))
    dist.destroy_process_group()


def test_integration_example(cuda):
    """INTEGRATION.md §4's code block, run as written on 2 ranks (gloo, one
    GPU): the index answers like the single-GPU search, and the sharded step's
    loss is the single-GPU loss of the global batch."""
    import re

    from pkg.modelling import hip_ops

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    text = open(os.path.join(root, "INTEGRATION.md")).read()
    sec = text[text.index("## 4. Multi-GPU"):]
    code = re.search(r"```python\n(.*?)```", sec, re.S).group(1)
    rng = np.random.default_rng(5)
    C = np.maximum(rng.standard_normal((1000, 32)), 0).astype(np.float32)
    qemb = np.maximum(rng.standard_normal((64, 32)), 0).astype(np.float32)
    gb = _global_batches(1, 128)[0]
    tc = torch.as_tensor(C, device=cuda)
    ref_s, ref_i = hip_ops.bruteforce_search(hip_ops.bruteforce_build(tc), tc, torch.as_tensor(qemb, device=cuda), 100)
    ref = _small_model(cuda, 3)
    ref_loss = float(ref.train_step({k: torch.as_tensor(v, device=cuda) for k, v in gb.items()})["loss"].item())
    out = mp.Manager().dict()
    mp.spawn(_integration_worker, args=(2, _free_port(), code, C, gb, qemb, out), nprocs=2, join=True)
    for r in range(2):
        s, i, loss, held = out[r]
        assert held == 500
        assert np.array_equal(i, ref_i.cpu().numpy()) and np.array_equal(s, ref_s.cpu().numpy())
        np.testing.assert_allclose(loss, ref_loss, rtol=2e-5)


# --------------------------------------------------------------------------- C5 at its 8-way layout
C5_ROWS, C5_DIM, C5_BATCH, C5_WORLD = 100_000_000, 128, 65536, 8
_C5_SCALE = np.float32(0.05 / 32768)


def _c5_values_np(rows: np.ndarray) -> np.ndarray:
    """Initial value of global rows `rows` (int64): a hash of (row, column),
    restated by _c5_fill on the GPU with the same fp32 operations."""
    h = (rows.astype(np.int64)[:, None] * 2654435761 + np.arange(C5_DIM, dtype=np.int64)[None, :] * 97) % 65536
    return (h - 32768).astype(np.float32) * _C5_SCALE


def _c5_fill(shard: torch.Tensor, rank: int, world: int, chunk: int = 1 << 20) -> None:
    k = torch.arange(C5_DIM, dtype=torch.int64, device=shard.device)[None, :] * 97
    scale = torch.tensor(_C5_SCALE, device=shard.device)
    for s in range(0, shard.shape[0], chunk):
        n = min(chunk, shard.shape[0] - s)
        g = (torch.arange(s, s + n, dtype=torch.int64, device=shard.device) * world + rank)[:, None]
        shard[s:s + n] = ((g * 2654435761 + k) % 65536 - 32768).to(torch.float32) * scale


def _c5_ids() -> np.ndarray:
    rng = np.random.default_rng(3)
    ids = (((rng.zipf(1.8, C5_BATCH) - 1) % C5_ROWS) * 7919 % C5_ROWS).astype(np.int32)  # Zipf-like, spread
    ids[::7] = rng.integers(0, C5_ROWS, len(ids[::7]))  # plus uniform ids
    return ids


def _c5_grad(rank: int, b: int) -> np.ndarray:
    return np.random.default_rng(100 + rank).standard_normal((b, C5_DIM)).astype(np.float32)


def _c5_worker(rank, world, port, ids, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "hm-retrieval-two-tower_amd")]
    from pkg.modelling.distributed import ShardedTables

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n_local = len(range(rank, C5_ROWS, world))
    shard = torch.empty(n_local, C5_DIM, device=dev)  # ONLY this rank's rows: 12.5M x 128 (6.4 GB)
    _c5_fill(shard, rank, world)
    st = ShardedTables({"big": shard, "__rows__": {"big": C5_ROWS}}, full_tables=False)
    b = C5_BATCH // world
    mine = ids[rank * b:(rank + 1) * b]
    rows, (idx,) = st.fetch([("big", torch.as_tensor(mine, device=dev))])
    got = rows[idx.long()].cpu().numpy()
    fetch_ok = bool(np.array_equal(got, _c5_values_np(mine)))
    st.apply([(torch.as_tensor(_c5_grad(rank, b), device=dev), [(idx, 0)])], 0.05, 1e-7)
    torch.cuda.synchronize()
    owned = np.unique(ids[ids % world == rank]).astype(np.int64)  # this rank's touched rows, global ids
    loc = torch.as_tensor(owned // world, device=dev)
    out[rank] = (fetch_ok, idx.cpu().numpy(), owned, st.shard["big"][loc].cpu().numpy(),
                 st.acc["big"][loc].cpu().numpy(), int(st.shard["big"].shape[0]))
    dist.destroy_process_group()


def test_c5_row_sharded_table_eight_ranks(cuda):
    """configs[4] at its stated layout: a 100M x 128 fp32 table row-sharded
    over 8 ranks (eight processes on cuda:0, gloo; global row r on rank r % 8,
    each rank building ONLY its 12.5M rows and their accumulator), a global
    batch of 65,536 Zipf + uniform ids split over the ranks.
      * fetched rows (all_to_all of requests and rows) bit-exact;
      * one Adagrad apply bit-exact against the restatement of the sharded
        order: each rank's per-request sums (oracle.dedup_sum: the GPU dedup's
        block order, tt_sparse_scatter_sum), sent to the owners, the owner's
        sparse Adagrad over the requests in source-rank order
        (oracle.sparse_adagrad on the owner's touched rows, compacted in
        order)."""
    from oracle import oracle

    ids = _c5_ids()
    out = mp.Manager().dict()
    mp.spawn(_c5_worker, args=(C5_WORLD, _free_port(), ids, out), nprocs=C5_WORLD, join=True)
    W, b = C5_WORLD, C5_BATCH // C5_WORLD
    recv = {o: ([], []) for o in range(W)}  # owner -> (global rows, gradient rows) in arrival order
    for s in range(W):
        fetch_ok, idx, *_ = out[s]
        assert fetch_ok, s
        mine = ids[s * b:(s + 1) * b].astype(np.int64)
        uniq, sums = oracle.dedup_sum(idx, _c5_grad(s, b), oracle.GPU_DEDUP_CHUNK)  # per-request sums
        req_row = np.empty(len(uniq), np.int64)
        req_row[idx] = mine  # request j <- the global row of its lookups
        assert np.array_equal(uniq, np.arange(len(uniq)))
        for o in range(W):  # requests are bucketed by owner, in request order within a bucket
            sel = np.nonzero(req_row % W == o)[0]
            recv[o][0].append(req_row[sel])
            recv[o][1].append(sums[sel])
    for o in range(W):
        _, _, owned, t_got, a_got, n_local = out[o]
        assert n_local == len(range(o, C5_ROWS, W)) and n_local < C5_ROWS
        rows = np.concatenate(recv[o][0])
        grads = np.concatenate(recv[o][1])
        assert np.array_equal(np.unique(rows), owned)
        t_ref = _c5_values_np(owned)
        a_ref = np.full_like(t_ref, 0.1)
        oracle.sparse_adagrad(t_ref, a_ref, np.searchsorted(owned, rows).astype(np.int32), grads, 0.05)
        assert np.array_equal(t_got, t_ref), o
        assert np.array_equal(a_got, a_ref), o
