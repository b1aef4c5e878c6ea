"""CPU: the restatement (oracle/) against the reference's own test vectors
(tests/golden/reference_tests.json), plus internal consistency of the paths
no reference test pins (documented as "parity unpinned" in DESIGN.md)."""
import json
import os

import numpy as np
import pytest

from oracle import oracle

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_tests.json")))


def test_logq_matches_reference_test_layers():
    g = GOLD["logq"]
    out = oracle.logq_correction(g["logits"], g["candidate_ids"], g["candidate_prob_lookup"])
    exp = np.asarray(g["expected"], np.float32)
    assert np.array_equal(np.round(out, g["round_decimals"]), np.round(exp, g["round_decimals"]))


def test_logq_missing_id_defaults_to_p1():
    out = oracle.logq_correction([[1.0, 2.0]], ["known", "missing"], {"known": 0.5})
    assert out[0, 1] == 2.0 and np.isclose(out[0, 0], 1.0 - np.log(np.float32(0.5)))


def test_bruteforce_matches_reference_test_indices():
    g = GOLD["bruteforce"]
    rows = oracle.string_lookup(g["query_vocab"], g["queries"])
    assert rows.tolist() == g["derived_query_rows"] == [1, 2, 3, 0, 1]
    q = np.asarray(g["query_embeddings"], np.float32)[rows]
    s, i, _ = oracle.bruteforce_topk(q, np.asarray(g["candidate_embeddings"], np.float32), g["k"])
    assert [[g["candidate_ids"][j] for j in r] for r in i] == g["expected"]
    assert i.tolist() == g["derived_topk_indices"]


def test_recall_matches_reference_test_recall():
    g = GOLD["recall"]
    acc = oracle.RecallAccumulator(g["ks"])
    t = g["true_candidate_ids"]
    for s in range(0, len(t), g["batch_size"]):
        part = t[s:s + g["batch_size"]]
        acc.update(part, oracle.static_index(g["static_candidates"], g["k"], len(part)))
    for k, v in g["expected"].items():
        assert acc.metric[int(k)] == np.float64(v)
        assert isinstance(acc.metric[int(k)], np.float64)


def test_topk_tie_rule_lower_index_first():
    c = np.array([[1.0, 0.0], [1.0, 0.0], [0.0, 1.0], [1.0, 0.0]], np.float32)
    q = np.array([[1.0, 0.0], [0.0, 0.0]], np.float32)
    s, i, _ = oracle.bruteforce_topk(q, c, 3)
    assert i.tolist() == [[0, 1, 3], [0, 1, 2]]
    # -0.0 ties with +0.0
    c2 = np.array([[-1.0, 0.0], [1.0, 0.0]], np.float32)
    s, i, _ = oracle.bruteforce_topk(np.array([[0.0, 1.0]], np.float32), c2, 2)
    assert i.tolist() == [[0, 1]]


def test_fmaf_chain_scores_match_float64_closely():
    rng = np.random.default_rng(0)
    q = rng.standard_normal((7, 128)).astype(np.float32)
    c = rng.standard_normal((50, 128)).astype(np.float32)
    s = oracle.fmaf_scores(q, c)
    np.testing.assert_allclose(s, q.astype(np.float64) @ c.T.astype(np.float64), rtol=1e-5, atol=1e-4)


def test_dedup_sequential_vs_chunked_orders():
    ids = np.array([5, 3, 5, 5, 3, 9], np.int32)
    g = np.arange(12, dtype=np.float32).reshape(6, 2)
    u, s = oracle.dedup_sum(ids, g, chunk=0)
    assert u.tolist() == [3, 5, 9]
    assert s.tolist() == [[2 + 8, 3 + 9], [0 + 4 + 6, 1 + 5 + 7], [10, 11]]
    u2, s2 = oracle.dedup_sum(ids, g, chunk=2)
    assert np.array_equal(u2, u) and np.array_equal(s2, s)


def test_sparse_adagrad_matches_formula():
    t = np.zeros((4, 2), np.float32)
    a = np.full((4, 2), 0.1, np.float32)
    ids = np.array([1, 1, 3], np.int32)
    g = np.array([[1.0, 2.0], [3.0, 4.0], [5.0, 6.0]], np.float32)
    oracle.sparse_adagrad(t, a, ids, g, lr=0.05)
    gs = np.array([4.0, 6.0], np.float32)
    acc = np.float32(0.1) + gs * gs
    np.testing.assert_array_equal(a[1], acc)
    np.testing.assert_array_equal(t[1], -(np.float32(0.05) * gs) / (np.sqrt(acc) + np.float32(1e-7)))
    assert np.all(t[0] == 0) and np.all(a[0] == np.float32(0.1))


def test_inbatch_loss_gradients_finite_difference():
    rng = np.random.default_rng(1)
    B, E = 6, 4
    q = rng.standard_normal((B, E))
    c = rng.standard_normal((B, E))
    lq = np.log(rng.uniform(0.01, 0.3, B))
    r = oracle.inbatch_softmax_xent(q, c, lq)
    eps = 1e-6
    for (arr, key) in ((q, "dq"), (c, "dc")):
        num = np.zeros_like(arr)
        for idx in np.ndindex(*arr.shape):
            old = arr[idx]
            arr[idx] = old + eps
            lp = oracle.inbatch_softmax_xent(q, c, lq)["loss"]
            arr[idx] = old - eps
            lm = oracle.inbatch_softmax_xent(q, c, lq)["loss"]
            arr[idx] = old
            num[idx] = (lp - lm) / (2 * eps)
        np.testing.assert_allclose(r[key], num, rtol=1e-5, atol=1e-6)
    # CE with eye labels and SUM reduction == sum of row losses
    S = q @ c.T - lq[None, :]
    lse = np.log(np.exp(S).sum(1))
    assert np.isclose(r["loss"], np.sum(lse - np.diag(S)))


def test_gather_concat_numeric_first_and_oob_zero():
    t = np.arange(6, dtype=np.float32).reshape(3, 2)
    out = oracle.gather_concat([np.array([7.0, 8.0], np.float32)], [t], [np.array([2, 5], np.int32)])
    assert out.tolist() == [[7.0, 4.0, 5.0], [8.0, 0.0, 0.0]]


def test_topk_merge_equals_global_topk():
    rng = np.random.default_rng(3)
    q = rng.standard_normal((5, 8)).astype(np.float32)
    c = np.round(rng.standard_normal((40, 8)), 1).astype(np.float32)
    s, i, _ = oracle.bruteforce_topk(q, c, 6)
    parts = []
    for b, e in ((0, 13), (13, 27), (27, 40)):
        ps, pi, _ = oracle.bruteforce_topk(q, c[b:e], 6)
        parts.append((ps, pi + b))
    ms, mi = oracle.topk_merge(np.stack([p[0] for p in parts]), np.stack([p[1] for p in parts]), 6)
    assert np.array_equal(mi, i) and np.array_equal(ms, s)


def test_vocab_value_counts_order():
    v = oracle.vocab_from_values(["b", "a", "b", "c", "a", "b"], max_vocab_size=2)
    assert v.tolist() == ["b", "a"]
    assert oracle.string_lookup(v, ["a", "zzz", "b"]).tolist() == [2, 0, 1]


def test_bf16_round_is_round_to_nearest_even():
    """oracle.bf16_round == torch's fp32 -> bfloat16 conversion (RNE), incl.
    ties, infinities and values near the top of the range."""
    import torch

    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(10000).astype(np.float32) * 10.0 ** rng.integers(-30, 30, 10000),
                        np.array([1.0 + 2.0 ** -8, 1.0 + 3 * 2.0 ** -8, -(1.0 + 2.0 ** -8), np.inf, -np.inf, 0.0,
                                  3.0e38], np.float32)]).astype(np.float32)
    ref = torch.from_numpy(x).to(torch.bfloat16).float().numpy()
    assert np.array_equal(oracle.bf16_round(x), ref)


def test_inbatch_contract_oracle_properties():
    """The kernels' arithmetic contract restated (oracle.inbatch_softmax_xent_bf16):
    close to the fp64 loss/gradients (bf16 negatives only); row blocks with a
    positive offset give the same rows as the full batch; a one-column batch
    has loss 0 and zero gradients (P_pos = 1 exactly)."""
    rng = np.random.default_rng(3)
    B, E = 96, 32
    q = np.maximum(rng.standard_normal((B, E)) * 0.5, 0).astype(np.float32)
    c = np.maximum(rng.standard_normal((B, E)) * 0.5, 0).astype(np.float32)
    lq = np.log(rng.uniform(1e-5, 1e-2, B)).astype(np.float32)
    ref = oracle.inbatch_softmax_xent(q, c, lq)
    con = oracle.inbatch_softmax_xent_bf16(q, c, lq)
    rel = lambda a, b: np.linalg.norm(a - b) / np.linalg.norm(b)
    assert abs(con["loss"] - ref["loss"]) <= 1e-3 * abs(ref["loss"])
    assert rel(con["dq"], ref["dq"]) <= 1e-2 and rel(con["dc"], ref["dc"]) <= 1e-2
    G, b = 4, B // 4
    for r in range(G):
        sl = slice(r * b, (r + 1) * b)
        blk = oracle.inbatch_softmax_xent_bf16(q[sl], c, lq, pos_offset=r * b)
        assert np.array_equal(blk["dq"], con["dq"][sl]) and np.array_equal(blk["row_loss"], con["row_loss"][sl])
        dc = oracle.inbatch_cols_bf16(q, con["lse"], con["row_loss"], c[sl], lq[sl], pos_offset=r * b)
        np.testing.assert_allclose(dc, con["dc"][sl], rtol=1e-6, atol=1e-7)
    one = oracle.inbatch_softmax_xent_bf16(q[:1], c[:1], lq[:1])
    assert one["loss"] == 0.0 and not one["dq"].any() and not one["dc"].any()
