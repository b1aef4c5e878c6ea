"""CPU: the input pipeline's host side and the export format (no GPU compute).

* libtt's native StringLookup (tt_vocab_*) against the
  reference semantics restated as a Python dict: vocab[i] -> i + 1, anything
  else -> 0 (input_layer.py:33-36, StringLookup num_oov_indices=1), values
  compared as str() (the reference's features are tf.string).
* epoch order / EncodedDataset batching (tfrecord_dataset.py:59-98).
* the vectorised logQ lookup vs the reference's default-1.0 semantics
  (logq_correction.py:32-42,66-71) and row_table's precondition.
* save/load round trips of towers, the two-tower model and the index files
  (weights-only .pt + .json + .npz, no pickles).
"""
import ctypes
import json

import numpy as np
import pytest
import torch

from pkg import _native, dtypes
from pkg.modelling.dataset import EncodedDataset, encode_dataframe, epoch_order
from pkg.modelling.layers.logq_correction import LogQCorrection
from pkg.schema.features import Feature, FeatureFamily
from pkg.schema.vocab import NativeVocab, string_arena


def dict_lookup(vocab, values):
    table = {str(v): i + 1 for i, v in enumerate(vocab)}
    out = []
    for v in values:
        if isinstance(v, bytes):
            v = v.decode()
        out.append(table.get(str(v), 0))
    return np.asarray(out, np.int32)


@pytest.mark.parametrize("threads", [1, 3, 0])
def test_native_vocab_matches_dict_lookup(threads):
    rng = np.random.default_rng(1)
    vocab = [f"{x:064x}" for x in rng.integers(0, 2**62, 20000)] + ["", "é", "a", "ünï", "a b", "0"]
    v = NativeVocab(vocab)
    assert v.size == len(vocab)
    picks = [vocab[i] for i in rng.integers(0, len(vocab), 200000)]
    vals = np.array(picks + ["zz", "", "é", "A", "a ", " a", "00"], dtype=object)
    np.testing.assert_array_equal(v.encode(vals, threads), dict_lookup(vocab, vals))


def test_native_vocab_value_kinds():
    vocab = ["1", "3", "True", "1.5", "-7", "x"]
    v = NativeVocab(vocab)
    for vals in ([1, 3, 5, -7], np.array([1, 3, 5], np.int64), np.array([3], np.uint8), [True, False, 1.5, 2.0],
                 [b"x", b"3", b"q"], np.array(["x", "1"]), np.array([b"x", b"1"]), ["x", 3, b"1", 1.5]):
        np.testing.assert_array_equal(v.encode(vals), dict_lookup(vocab, list(vals)))
    assert v.encode([]).shape == (0,)
    # a value listed twice maps to its last row (the dict of Feature.lookup_table)
    d = NativeVocab(["a", "b", "a"])
    np.testing.assert_array_equal(d.encode(["a", "b", "c"]), [3, 2, 0])
    # None reads as str(None) and float32 as str(np.float32(x)), the text a
    # str()-cast column holds (no widening of 0.1f to 0.10000000149011612)
    wv = ["None", "0.1", "x", "2.5", "nan"]
    w = NativeVocab(wv)
    for vals in (np.array(["x", None], dtype=object), [None, "x", 0.1],
                 np.array([0.1, 2.5, 0.3], np.float32), np.array([0.1, np.nan], np.float64),
                 np.array([np.float32(0.1), None, "x"], dtype=object)):
        np.testing.assert_array_equal(w.encode(vals), dict_lookup(wv, list(vals)))
    import pyarrow as pa
    with pytest.raises(ValueError):  # an Arrow array's nulls have no text
        v.encode(pa.array(["x", None]))


def test_native_vocab_host_validation():
    lib = _native.lib()
    h = ctypes.c_void_p()
    assert lib.tt_vocab_create(None, None, 3, ctypes.byref(h)) == _native.TT_ERR_BAD_ARG
    assert lib.tt_vocab_create(None, None, -1, ctypes.byref(h)) == _native.TT_ERR_BAD_ARG
    off = np.array([0, 2, 1], np.int64)
    data = np.frombuffer(b"abc", np.uint8)
    rc = lib.tt_vocab_create(ctypes.c_void_p(data.ctypes.data), ctypes.c_void_p(off.ctypes.data), 2, ctypes.byref(h))
    assert rc == _native.TT_ERR_BAD_ARG and "decrease" in lib.tt_last_error().decode()
    assert lib.tt_vocab_encode(None, None, None, 0, None, 0) == _native.TT_ERR_BAD_ARG
    assert lib.tt_vocab_size(None) == -1


def test_string_arena_offsets_and_slices():
    import pyarrow as pa

    arr = pa.array(["ab", "", "cde", "f"]).slice(1)
    data, off, n, _ = string_arena(arr)
    assert n == 3
    got = [bytes(data[off[i]:off[i + 1]]).decode() for i in range(n)]
    assert got == ["", "cde", "f"]


def test_feature_encode_uses_native_and_survives_pickle():
    import pickle

    f = Feature("c", dtypes.string, FeatureFamily.QUERY, embedding_size=4, vocab=["a", "b"])
    np.testing.assert_array_equal(f.encode(["b", "a", "z"]), [2, 1, 0])
    g = pickle.loads(pickle.dumps(f))
    np.testing.assert_array_equal(g.encode(["b", "zz"]), [2, 0])


def test_epoch_order_windows_and_dataset_batches():
    o = epoch_order(1000, 128, 3, 1)
    assert sorted(o.tolist()) == list(range(1000))
    for s in range(0, 1000, 128):  # a shuffle buffer never moves an element out of its window
        assert sorted(o[s:s + 128].tolist()) == list(range(s, min(s + 128, 1000)))
    assert np.array_equal(epoch_order(10, None, 0, 5), np.arange(10))
    cols = {"a": np.arange(1000, dtype=np.int32), "b": np.arange(1000, dtype=np.float32) * 0.5}
    ds = EncodedDataset(cols, 300, 128, seed=3, device=torch.device("cpu"))
    ds._epoch = 1
    batches = list(ds)
    assert [len(b["a"]) for b in batches] == [300, 300, 300, 100]
    np.testing.assert_array_equal(np.concatenate([b["a"].numpy() for b in batches]), o)


def test_logq_vectorised_lookup_matches_reference_semantics():
    lookup = {"a": 0.5, "b": 0.25, "c": 1e-6}
    corr = LogQCorrection(lookup)
    ids = ["a", "c", "zz", b"b", 7]
    ref = np.log(np.array([lookup.get(x.decode() if isinstance(x, bytes) else str(x), 1.0) for x in ids],
                          np.float32)).astype(np.float32)
    np.testing.assert_array_equal(corr.log_probs(ids), ref)
    f = Feature("article_id", dtypes.string, FeatureFamily.CANDIDATE, embedding_size=4, vocab=["a", "b"])
    with pytest.raises(ValueError, match="__logq__"):
        corr.row_table(f, torch.device("cpu"))
    import pandas as pd

    df = pd.DataFrame({"article_id": ["a", "c", "q"]})
    cols = encode_dataframe(df, [f], logq=corr, candidate_col="article_id")
    np.testing.assert_array_equal(cols["__logq__"], corr.log_probs(["a", "c", "q"]))
    np.testing.assert_array_equal(cols["article_id"], [1, 0, 0])


def _features():
    return ([Feature("customer_id", dtypes.string, FeatureFamily.QUERY, embedding_size=8,
                     vocab=[f"c{i}" for i in range(50)]),
             Feature("age", dtypes.float32, FeatureFamily.QUERY)],
            [Feature("article_id", dtypes.string, FeatureFamily.CANDIDATE, embedding_size=8,
                     vocab=[f"a{i}" for i in range(40)]),
             Feature("section", dtypes.string, FeatureFamily.CANDIDATE, embedding_size=4, vocab=["x", "y"])])


def test_two_tower_and_tower_save_load_round_trip(tmp_path):
    from pkg.modelling.models.tower import Tower
    from pkg.modelling.models.two_tower_model import TwoTowerModel

    cpu = torch.device("cpu")
    qf, cf = _features()
    probs = {f"a{i}": 1.0 / 40 for i in range(40)}
    m = TwoTowerModel(qf, cf, "article_id", 16, [24], [20], candidate_prob_lookup=probs, device=cpu, seed=5)
    m.save(str(tmp_path / "model") + "/")
    meta = json.load(open(tmp_path / "model" / "two_tower.json"))
    assert meta["candidate_id_col"] == "article_id" and meta["query_tower_units"] == [24]
    r = TwoTowerModel.load(str(tmp_path / "model") + "/", device=cpu)
    for k, v in m.state_dict().items():
        assert torch.equal(v, r.state_dict()[k]), k
    assert [f.name for f in r.query_features] == ["customer_id", "age"]
    assert list(r.candidate_features[0].vocab) == list(cf[0].vocab)
    assert r.logq_correction.lookup == m.logq_correction.lookup
    t = Tower.load(str(tmp_path / "model" / "query_tower"), device=cpu)
    assert torch.equal(t.dense.flat, m.query_tower.dense.flat)
    assert torch.equal(t.input_layer.embedding_layers["customer_id"].weight,
                       m.query_tower.input_layer.embedding_layers["customer_id"].weight)
    # weights-only files: the tensors load without unpickling code
    sd = torch.load(tmp_path / "model" / "two_tower.pt", weights_only=True)
    assert "query_tower.dense.flat" in sd
    with np.load(tmp_path / "model" / "two_tower.npz", allow_pickle=False) as z:
        assert "candidate.vocab.article_id" in z.files
