"""CPU, world_size 2 over gloo: the multi-GPU orchestration of
pkg.modelling.distributed with the kernels replaced by the CPU restatement
(injected `ops`; the product's defaults are the libtt kernels)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _oracle_ops(two_phase=False):
    from oracle import oracle
    from pkg.modelling.distributed import IndexOps

    def search(img, cand, q, k, off):
        s, i, _ = oracle.bruteforce_topk(q.numpy(), cand.numpy(), k)
        return torch.from_numpy(s), torch.from_numpy(i + off)

    def merge(s, i, k):
        ms, mi = oracle.topk_merge(s.numpy(), i.numpy(), k)
        return torch.from_numpy(np.ascontiguousarray(ms)), torch.from_numpy(np.ascontiguousarray(mi))

    def shard_search(img, cand, q, k, off, reduce_max, chunk):
        # the two-phase contract with the loosest legal screen, per chunk of
        # queries like tt_bruteforce_shard_screen/_finalize: a lower bound on
        # the shard's k-th score, max-reduced, then the exact top-k of the
        # entries scoring >= the floor, padded with (-inf, INT32_MAX)
        s, i, _ = oracle.bruteforce_topk(q.numpy(), cand.numpy(), k)
        kth = torch.from_numpy(s[:, k - 1] - np.abs(s[:, k - 1]) * 0.25 - 0.5)
        for q0 in range(0, q.shape[0], chunk):
            reduce_max(kth[q0:q0 + chunk])  # a view: reduced in place
        keep = s >= kth.numpy()[:, None]
        s = np.where(keep, s, -np.inf).astype(np.float32)
        i = np.where(keep, i + off, 0x7FFFFFFF).astype(np.int32)
        return torch.from_numpy(s), torch.from_numpy(i)

    def shard_chunk(nq, sizes, dim, k):
        # a recommendation that differs per shard size (like plan_search's),
        # reduced over every shard: ranks that used their own would issue
        # different numbers of all_reduce calls and gloo would fail
        return min(3 + n % 5 for n in sizes)

    return IndexOps(build=lambda c: None, search=search, merge=merge,
                    shard_search=shard_search if two_phase else None, shard_chunk=shard_chunk)


def _index_worker(rank, world, port, q, c, k, out):
    _init(rank, world, port)
    from pkg.modelling.distributed import QueryShardedBruteForceIndex, ShardedBruteForceIndex, shard_range

    qidx = QueryShardedBruteForceIndex(k, None, torch.from_numpy(c), ops=_oracle_ops())
    qs_s, qs_i = qidx.search(torch.from_numpy(q))
    out[("q", rank)] = (qs_s.numpy(), qs_i.numpy())

    # each rank is handed ONLY its rows: the even split, and a ragged split
    # whose first shard has fewer rows than k (its list is padded)
    N = c.shape[0]
    ragged = [3] + [(N - 3) // (world - 1) + (1 if r < (N - 3) % (world - 1) else 0) for r in range(world - 1)]
    # ragged with every shard >= k (two-phase path) and shard sizes whose chunk
    # recommendations differ: more than one query chunk, same on every rank
    ragged_big = [k + 1] + [(N - k - 1) // (world - 1) + (1 if r < (N - k - 1) % (world - 1) else 0)
                            for r in range(world - 1)]
    for mode in ("even", "ragged", "ragged_big"):
        if mode == "even":
            b, e = shard_range(N, world, rank)
        else:
            sz = ragged if mode == "ragged" else ragged_big
            b = sum(sz[:rank])
            e = b + sz[rank]
        idx = ShardedBruteForceIndex(k, None, torch.from_numpy(c[b:e].copy()), ops=_oracle_ops())
        s, i = idx.search(torch.from_numpy(q))
        blk, os_, oi = idx.search_owned(torch.from_numpy(q))
        out[(mode, rank)] = (s.numpy(), i.numpy(), idx.num_candidates, blk, os_.numpy(), oi.numpy(),
                             idx.rows, int(idx.shard.shape[0]))
        # two-phase (screen floor all-reduced, cut rescoring): same answer
        idx2 = ShardedBruteForceIndex(k, None, torch.from_numpy(c[b:e].copy()), ops=_oracle_ops(True))
        s2, i2 = idx2.search(torch.from_numpy(q))
        out[(mode + "2", rank)] = (s2.numpy(), i2.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_index_equals_unsharded(world):
    from oracle import oracle

    rng = np.random.default_rng(0)
    c = np.maximum(rng.standard_normal((301, 16)), 0).astype(np.float32)
    c[100:140] = c[99]  # cross-shard ties must resolve by global index
    q = np.maximum(rng.standard_normal((20, 16)), 0).astype(np.float32)
    q[3] = 0.0
    q[7] = rng.standard_normal(16).astype(np.float32)  # mixed signs
    k = 25
    out = mp.Manager().dict()
    mp.spawn(_index_worker, args=(world, _free_port(), q, c, k, out), nprocs=world, join=True)
    rs, ri, _ = oracle.bruteforce_topk(q, c, k)
    for mode in ("even", "ragged", "ragged_big"):
        covered, rows = [], []
        for r in range(world):
            s, i, n, (b, e), os_, oi, (r0, r1), held = out[(mode, r)]
            assert n == 301 and held == r1 - r0 < 301  # no rank holds every row
            rows.append((r0, r1))
            assert np.array_equal(i, ri) and np.array_equal(s, rs), mode
            s2, i2 = out[(mode + "2", r)]
            assert np.array_equal(i2, ri) and np.array_equal(s2, rs), mode + " two-phase"
            # search_owned: this rank's query block only, same global lists
            assert np.array_equal(oi, ri[b:e]) and np.array_equal(os_, rs[b:e]), mode
            covered += list(range(b, e))
        assert covered == list(range(q.shape[0]))
        assert rows[0][0] == 0 and rows[-1][1] == 301 and all(rows[j][1] == rows[j + 1][0] for j in range(world - 1))
    for r in range(world):
        qs_s, qs_i = out[("q", r)]  # query-sharded: every rank holds the full answer
        assert np.array_equal(qs_i, ri) and np.array_equal(qs_s, rs)


# --------------------------------------------------------------------------- row-sharded tables (C5)
def _cpu_embedding_ops(routed: bool = False):
    """CPU restatement of the libtt kernels the sharded path calls (test-only);
    routed: with the route-keyed sparse op (tt_sparse_routed's semantics)."""
    from pkg.modelling.distributed import EmbeddingOps

    def gather_multi(calls, batch):
        for segs, out in calls:
            for table, ids, off in segs:
                if ids is None:
                    out[:, off] = table
                    continue
                d = table.shape[1]
                ii = ids.long()
                ok = (ii >= 0) & (ii < table.shape[0])
                rows = torch.zeros(batch, d)
                rows[ok] = table[ii[ok]]
                out[:, off:off + d] = rows

    def gather_tagged(tables, tags, rows, out):
        out.zero_()
        for j in range(tags.numel()):
            t, r = int(tags[j]), int(rows[j])
            if 0 <= t < len(tables) and 0 <= r < tables[t].shape[0]:
                out[j, :tables[t].shape[1]] = tables[t][r]
        return out

    def scatter_sum(specs, batch, grad):
        for s in specs:
            tab = s["table"]
            d = tab.shape[1]
            acc = torch.zeros_like(tab, dtype=torch.float64)
            touched = torch.zeros(tab.shape[0], dtype=torch.bool)
            g_s = s.get("grad") if s.get("grad") is not None else grad
            for ids, off in zip(s["ids"], s["grad_col_offset"]):
                ii = ids.long()
                ok = (ii >= 0) & (ii < tab.shape[0])
                acc.index_add_(0, ii[ok], g_s[ok, off:off + d].double())
                touched[ii[ok]] = True
            tab[touched] = acc[touched].float()

    def sparse_adagrad(specs, batch, grad, lr, eps):
        for s in specs:
            tab, accum = s["table"], s["slot0"]
            d = tab.shape[1]
            g = torch.zeros_like(tab, dtype=torch.float64)
            touched = torch.zeros(tab.shape[0], dtype=torch.bool)
            g_s = s.get("grad") if s.get("grad") is not None else grad
            for ids, off in zip(s["ids"], s["grad_col_offset"]):
                ii = ids.long()
                ok = (ii >= 0) & (ii < tab.shape[0])
                g.index_add_(0, ii[ok], g_s[ok, off:off + d].double())
                touched[ii[ok]] = True
            gt = g[touched]
            a = accum[touched].double() + gt * gt
            accum[touched] = a.float()
            tab[touched] = (tab[touched].double() - lr * gt / (a.sqrt() + eps)).float()

    def dense_adagrad(p, acc, g, lr, eps):
        a = acc.double() + g.double() ** 2
        acc.copy_(a.float())
        p.copy_((p.double() - lr * g.double() / (a.sqrt() + eps)).float())

    def sparse_routed(specs, batch, grad, route, op, lr=0.0, eps=0.0):
        # keyed by slot: the per-request sums; keyed by slot_row (world 1):
        # the owner's Adagrad on its local rows
        if op == "sum":
            return scatter_sum(specs, batch, grad)
        rows = route["slot_row"]
        # a dropped request's lookups carry the sentinel -1 - owner: no row
        key = lambda i: torch.where(i >= 0, rows[i.long().clamp(min=0)], torch.full_like(i, -1))
        return sparse_adagrad([dict(sp, ids=[key(i) for i in sp["ids"]]) for sp in specs], batch, grad, lr, eps)

    from torch_route import torch_route_owner, torch_route_pad, torch_route_requests

    return EmbeddingOps(gather_multi, gather_tagged, scatter_sum, sparse_adagrad, dense_adagrad,
                        torch_route_requests, torch_route_owner, torch_route_pad,
                        sparse_routed=sparse_routed if routed else None)


def _sharded_worker(rank, world, port, tables, lookups, grads, out):
    _init(rank, world, port)
    from pkg.modelling.distributed import ShardedTables

    lk = [(name, torch.from_numpy(ids[rank])) for name, ids in lookups]
    g = torch.from_numpy(grads[rank])  # this rank's [B, 16 * L] gradients, lookup l at column 16 l
    res = {}
    # compact routing (host-known counts), the fixed-capacity routing at the
    # never-overflowing capacity, and at a capacity too small for the batch
    for mode, cap in (("compact", None), ("fixed", "full"), ("small", 5)):
        st = ShardedTables({k: torch.from_numpy(v) for k, v in tables.items()}, 0.1, ops=_cpu_embedding_ops())
        ov = torch.zeros(1, dtype=torch.int32)
        got, idx = st.fetch(lk, capacity=cap, overflow=ov)
        # a dropped request's lookups carry the slot sentinel -1 - owner: zero rows
        fwd = [torch.where((i >= 0)[:, None], got[i.long().clamp(min=0)], torch.zeros(())).numpy() for i in idx]
        st.apply([(g, [(idx[l], 16 * l) for l in range(len(lk))])], lr=0.05, eps=1e-7)
        res[mode] = (fwd, {k: st.gather_full(k).numpy() for k in tables}, int(ov.item()))
    # route_fixed + fetch_routed + apply_lookups (per-lookup gradients): the
    # same update as apply() on the fixed route
    for mode, routed in (("lookups", False), ("routed", True)):
        st = ShardedTables({k: torch.from_numpy(v) for k, v in tables.items()}, 0.1, ops=_cpu_embedding_ops(routed))
        rt = st.route_fixed(lk, st.route_capacity(len(lk), lk[0][1].numel()))
        got = st.fetch_routed(rt)
        st.apply_lookups(rt, [(g, 16 * l) for l in range(len(lk))], lr=0.05, eps=1e-7)
        res[mode] = ([got[i.long()].numpy() for i in rt.idx], {k: st.gather_full(k).numpy() for k in tables}, 0)
    if world == 1:  # one rank: fetch_local + apply_local (by id, no route)
        st = ShardedTables({k: torch.from_numpy(v) for k, v in tables.items()}, 0.1, ops=_cpu_embedding_ops())
        B = lk[0][1].numel()
        got = st.fetch_local(lk, torch.empty(len(lk), B, st.dim))
        st.apply_local(lk, [(g, 16 * l) for l in range(len(lk))], lr=0.05, eps=1e-7)
        res["local"] = ([got[l].numpy() for l in range(len(lk))], {k: st.gather_full(k).numpy() for k in tables}, 0)
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_tables_match_unsharded_adagrad(world):
    rng = np.random.default_rng(1)
    B, D = 40, 16
    tables = {"cust": rng.uniform(-0.05, 0.05, (97, D)).astype(np.float32),
              "art": rng.uniform(-0.05, 0.05, (31, D)).astype(np.float32)}
    # per rank ids (with duplicates, out-of-range ids and one table looked up twice)
    ids = lambda n: rng.integers(-2, n + 3, (world, B)).astype(np.int32)
    lookups = [("cust", ids(97)), ("art", ids(31)), ("cust", ids(97))]
    grads = rng.standard_normal((world, B, 16 * len(lookups))).astype(np.float32)
    out = mp.Manager().dict()
    mp.spawn(_sharded_worker, args=(world, _free_port(), tables, lookups, grads, out), nprocs=world, join=True)
    # reference: unsharded tables, global batch = all ranks' lookups, one Adagrad step
    ref = {k: v.astype(np.float64) for k, v in tables.items()}
    acc = {k: np.full_like(v, 0.1) for k, v in ref.items()}
    gsum = {k: np.zeros_like(v) for k, v in ref.items()}
    for r in range(world):
        for l, (name, idsl) in enumerate(lookups):
            ok = (idsl[r] >= 0) & (idsl[r] < tables[name].shape[0])
            # forward rows equal the unsharded gather (zeros for invalid ids)
            exp = np.zeros((B, D), np.float32)
            exp[ok] = tables[name][idsl[r][ok]]
            assert np.array_equal(out[r]["compact"][0][l], exp)
            np.add.at(gsum[name], idsl[r][ok], grads[r][ok, 16 * l:16 * l + D])
    for k in ref:
        touched = np.abs(gsum[k]).sum(1) > 0
        a = acc[k] + gsum[k] ** 2
        upd = ref[k] - 0.05 * gsum[k] / (np.sqrt(a) + 1e-7)
        ref[k] = np.where(touched[:, None], upd, ref[k])
        for r in range(world):
            np.testing.assert_allclose(out[r]["compact"][1][k], ref[k], rtol=0, atol=2e-6)
    for r in range(world):
        # fixed slots per owner, no host-known counts: the same rows and updates, bit for bit
        fc, ff = out[r]["compact"], out[r]["fixed"]
        assert ff[2] == 0
        assert all(np.array_equal(x, y) for x, y in zip(ff[0], fc[0]))
        assert all(np.array_equal(ff[1][k], fc[1][k]) for k in tables)
        for mode in ("lookups", "routed") + (("local",) if world == 1 else ()):
            fl = out[r][mode]
            assert all(np.array_equal(x, y) for x, y in zip(fl[0], fc[0]))
            if mode in ("routed", "local") and world == 1:
                # one rank: the routed op / the local apply IS the owner's Adagrad (this CPU
                # restatement sums in fp64 without the per-request fp32 buffer;
                # on the GPU both are fp32 in one order: test_kernels_gpu)
                assert all(np.allclose(fl[1][k], fc[1][k], rtol=0, atol=1e-7) for k in tables)
            else:
                assert all(np.array_equal(fl[1][k], fc[1][k]) for k in tables)
        # a capacity of 5 slots per owner drops requests and counts them: the
        # distinct (table, row) requests of this rank per owner, minus 5
        reqs = {}
        for name, idsl in lookups:
            n = tables[name].shape[0]
            for v in np.unique(idsl[r]):
                key = (name, int(v)) if 0 <= v < n else (name, -1)
                reqs[key] = (int(v) % world) if 0 <= v < n else world - 1
        per_owner = np.bincount(list(reqs.values()), minlength=world)
        assert out[r]["small"][2] == int(np.maximum(per_owner - 5, 0).sum()) > 0
    # ... and the dropped requests' lookups read zero rows and add no gradient,
    # while the kept requests (per owner the first 5 in the route's (tag, row)
    # order, an invalid id first) and every untouched row stay exact
    names = list(tables)
    kept_g = {k: np.zeros_like(v) for k, v in ref.items()}
    for r in range(world):
        per = {}
        for name, idsl in lookups:
            n = tables[name].shape[0]
            for v in np.unique(idsl[r]):
                ok = 0 <= v < n
                o = int(v) % world if ok else world - 1
                per.setdefault(o, set()).add((names.index(name), int(v) + 1 if ok else 0))
        kept = {(names[t], rp - 1) for o in per for t, rp in sorted(per[o])[:5]}
        for l, (name, idsl) in enumerate(lookups):
            ok = np.array([(name, int(v)) in kept for v in idsl[r]]) & (idsl[r] >= 0)
            exp = np.zeros((B, D), np.float32)
            exp[ok] = tables[name][idsl[r][ok]]
            assert np.array_equal(out[r]["small"][0][l], exp)
            np.add.at(kept_g[name], idsl[r][ok], grads[r][ok, 16 * l:16 * l + D])
    for k in tables:
        touched = np.abs(kept_g[k]).sum(1) > 0
        a = 0.1 + kept_g[k] ** 2
        exp = np.where(touched[:, None], tables[k] - 0.05 * kept_g[k] / (np.sqrt(a) + 1e-7), tables[k])
        for r in range(world):
            np.testing.assert_allclose(out[r]["small"][1][k], exp, rtol=0, atol=2e-6)
            assert np.array_equal(out[r]["small"][1][k][~touched], tables[k][~touched])


def _global_loss_worker(rank, world, port, q, c, logq, out):
    _init(rank, world, port)
    from oracle import oracle
    from pkg.modelling.distributed import BatchComm
    from pkg.modelling.losses import global_inbatch_grads

    def rows(qq, C, L, pos_offset):
        r = oracle.inbatch_softmax_xent(qq.numpy(), C.numpy(), None if L is None else L.numpy(), pos_offset)
        return torch.from_numpy(r["lse"]), torch.from_numpy(r["row_loss"]), torch.from_numpy(r["dq"])

    def cols(Qa, lse, cl, L, pos_offset, row_loss=None):  # all rows (with their lse) against the local columns
        S = Qa.numpy() @ cl.numpy().T - (0.0 if L is None else L.numpy()[None, :])
        P = np.exp(S - lse.numpy()[:, None])
        P[pos_offset + np.arange(cl.shape[0]), np.arange(cl.shape[0])] -= 1.0
        return torch.from_numpy(P.T @ Qa.numpy())

    b = q.shape[0] // world
    sl = slice(rank * b, (rank + 1) * b)
    row_loss, dq, dc = global_inbatch_grads(torch.from_numpy(q[sl]), torch.from_numpy(c[sl]),
                                            torch.from_numpy(logq[sl]), BatchComm(), rows, cols)
    out[rank] = (row_loss.numpy(), dq.numpy(), dc.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_global_negatives_loss_equals_full_batch(world):
    """Global in-batch negatives split over the ranks (all_gather of the
    candidates and logq, rows pass with the positive at rank*b + i, cols pass
    share reduce-scattered) equal the reference loss over the whole batch
    (two_tower_model.py:113-122): every row's loss term, dQ, and dC.
    (The CPU ops restate the rows / cols passes; comm is the real gloo one.)"""
    from oracle import oracle

    rng = np.random.default_rng(1)
    B, E = 12 * world, 8
    q = rng.standard_normal((B, E))
    c = rng.standard_normal((B, E))
    logq = np.log(rng.dirichlet(np.ones(B)))
    ref = oracle.inbatch_softmax_xent(q, c, logq)
    out = mp.Manager().dict()
    mp.spawn(_global_loss_worker, args=(world, _free_port(), q, c, logq, out), nprocs=world, join=True)
    b = B // world
    total = 0.0
    for r in range(world):
        rl, dq, dc = out[r]
        sl = slice(r * b, (r + 1) * b)
        np.testing.assert_allclose(rl, ref["row_loss"][sl], rtol=1e-12)
        np.testing.assert_allclose(dq, ref["dq"][sl], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(dc, ref["dc"][sl], rtol=1e-10, atol=1e-12)
        total += rl.sum()
    assert abs(total - ref["loss"]) <= 1e-10 * abs(ref["loss"])
