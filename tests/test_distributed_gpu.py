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
