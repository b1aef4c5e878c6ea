"""Writes tests/golden/reference_tests.json: the inputs and expected outputs
that the reference's own unit tests hold (data only), plus integer forms
derived by the CPU restatement and checked against those expectations.

Sources (read as text; TensorFlow is absent, the tests cannot run here):
  /root/reference/tests/test_layers.py:8-39   LogQCorrection
  /root/reference/tests/test_indices.py:63-132 BruteForceIndex top-2
  /root/reference/tests/test_recall.py:8-95   IndexRecall with StaticIndex
  /root/reference/tests/test_transformations.py:6-36 date_filter
Run: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402

G = {}
G["logq"] = {
    "source": "tests/test_layers.py:8-39",
    "logits": [[1.0, -1.5, 2.5], [-1.0, -2.5, 1.5], [2.5, -1.5, -1.0]],
    "candidate_ids": ["id1", "id2", "id3"],
    "candidate_prob_lookup": {"id1": 0.3, "id2": 0.2, "id3": 0.5},
    "expected": [[2.2039728043, 0.1094379124, 3.1931471806],
                 [0.2039728043, -0.8905620876, 2.1931471806],
                 [3.7039728043, 0.1094379124, -0.3068528194]],
    "round_decimals": 5,
}
G["bruteforce"] = {
    "source": "tests/test_indices.py:63-132",
    "query_vocab": ["query_1", "query_2", "query_3"],
    "query_embeddings": [[1.0, 1.0], [0.5, -1.0], [1.0, -0.5], [-1.0, -0.5]],
    "candidate_ids": ["candidate_1", "candidate_2", "candidate_3", "candidate_4", "candidate_5"],
    "candidate_embeddings": [[2.0, -1.5], [-1.5, 3.0], [-0.5, -1.0], [1.0, -1.5], [-2.0, -1.5]],
    "queries": ["query_1", "query_2", "query_3", "query_4", "query_1"],
    "k": 2,
    "expected": [["candidate_1", "candidate_4"], ["candidate_1", "candidate_4"], ["candidate_5", "candidate_3"],
                 ["candidate_2", "candidate_1"], ["candidate_1", "candidate_4"]],
}
G["recall"] = {
    "source": "tests/test_recall.py:8-95",
    "static_candidates": [f"id{i}" for i in range(1, 11)],
    "k": 5,
    "true_candidate_ids": ["id1", "id7", "id2", "id2", "id10"],
    "batch_size": 2,
    "ks": [1, 2, 5],
    "expected": {"1": 0.2, "2": 0.6, "5": 0.6},
}
G["date_filter"] = {
    "source": "tests/test_transformations.py:6-36",
    "date_col": ["2024-01-01", "2024-02-01", "2024-03-01", "2024-04-01", "2024-05-01"],
    "ranges": [["2024-01-01", "2024-02-01"], ["2024-03-01", "2024-04-01"]],
    "expected_min_max": [["2024-01-01", "2024-02-01"], ["2024-03-01", "2024-04-01"]],
}

# Derived integer forms (checked against the string expectations above).
bf = G["bruteforce"]
rows = oracle.string_lookup(bf["query_vocab"], bf["queries"])
q = np.asarray(bf["query_embeddings"], np.float32)[rows]
c = np.asarray(bf["candidate_embeddings"], np.float32)
s, i, _ = oracle.bruteforce_topk(q, c, bf["k"])
assert [[bf["candidate_ids"][j] for j in r] for r in i] == bf["expected"]
bf["derived_query_rows"] = rows.tolist()
bf["derived_topk_indices"] = i.tolist()
bf["derived_topk_scores"] = s.tolist()
lg = G["logq"]
out = oracle.logq_correction(lg["logits"], lg["candidate_ids"], lg["candidate_prob_lookup"])
assert np.array_equal(np.round(out, 5), np.round(np.asarray(lg["expected"], np.float32), 5))

path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_tests.json")
with open(path, "w") as f:
    json.dump(G, f, indent=1)
print("wrote", path)
