"""GPU: the device-resident input pipeline and export / serving (SURVEY §8f
rows 1 and 4).

* DeviceDataset (tt_batch_take) yields exactly EncodedDataset's batches —
  same windowed shuffle, same partial last batch (tfrecord_dataset.py:59-98);
  a take past the epoch raises through the status word.
* fit over a DeviceDataset (one hipGraph replay per batch: device take +
  train step) leaves bit-identical tables / MLP weights and the same epoch
  loss as eager fit over the host-batched EncodedDataset.
* export: a trained model saved and loaded embeds bit-identically; a saved
  index, loaded as a Retriever, answers RAW string queries with the ids the
  in-memory index gives and that the fp32 oracle top-k gives
  (brute_force.py:54-83).
"""
import numpy as np
import pytest
import torch

from oracle import oracle
from pkg import dtypes
from pkg.modelling import hip_ops
from pkg.modelling.dataset import DeviceDataset, EncodedDataset
from pkg.modelling.export import Retriever
from pkg.modelling.indices.brute_force import BruteForceIndex
from pkg.modelling.models.two_tower_model import TwoTowerModel
from pkg.modelling.optimizer_factory import OptimizerFactory
from pkg.schema.features import Feature, FeatureFamily

pytestmark = pytest.mark.gpu


def _columns(n, seed=0):
    rng = np.random.default_rng(seed)
    return {"cust": (rng.zipf(1.3, n) % 301).astype(np.int32), "post": (rng.zipf(1.3, n) % 51).astype(np.int32),
            "art": (rng.zipf(1.3, n) % 301).astype(np.int32), "ptn": rng.integers(0, 21, n).astype(np.int32),
            "age": rng.standard_normal(n).astype(np.float32)}


def _model(cuda, seed=0):
    V = [str(i) for i in range(300)]
    qf = [Feature("cust", dtypes.string, FeatureFamily.QUERY, embedding_size=16, vocab=V),
          Feature("post", dtypes.string, FeatureFamily.QUERY, embedding_size=8, vocab=V[:50]),
          Feature("age", dtypes.float32, FeatureFamily.QUERY)]
    cf = [Feature("art", dtypes.string, FeatureFamily.CANDIDATE, embedding_size=16, vocab=V),
          Feature("ptn", dtypes.string, FeatureFamily.CANDIDATE, embedding_size=8, vocab=V[:20])]
    probs = {str(i): float(p) for i, p in enumerate(np.random.default_rng(seed).dirichlet(np.ones(300)))}
    m = TwoTowerModel(qf, cf, "art", 32, [64], [48], probs, device=cuda, seed=seed)
    m.compile(optimizer=OptimizerFactory.get_optimizer("adagrad", {"learning_rate": 0.05}))
    return m


@pytest.mark.parametrize("shuffle", [None, 700])
def test_device_dataset_batches_equal_encoded_dataset(cuda, shuffle):
    cols = _columns(5000, 1)
    host = EncodedDataset(cols, 1024, shuffle, seed=4, device=cuda)
    dev = DeviceDataset(cols, 1024, shuffle, seed=4, device=cuda)
    assert dev.keys == ["art", "cust", "post", "ptn", "age"]
    for _ in range(2):  # two epochs: a fresh order each
        hb, db = list(host), list(dev)
        assert [len(b["art"]) for b in db] == [1024] * 4 + [904]
        for h, d in zip(hb, db):
            assert set(h) == set(d)
            for k in h:
                assert d[k].dtype == h[k].dtype and torch.equal(d[k], h[k]), k
    dev.check_status()
    mapped = dev.map(lambda b: (b["cust"], b["age"]))
    first = next(iter(mapped))
    assert torch.equal(first[0], next(iter(EncodedDataset(cols, 1024, shuffle, seed=4, device=cuda)))["cust"])


def test_batch_take_past_the_epoch_is_flagged(cuda):
    dev = DeviceDataset(_columns(100), 64, device=cuda)
    dev.begin_epoch()
    dev.take(64)
    w = dev.take(64)  # 36 rows left: the rest are flagged, written as zeros
    torch.cuda.synchronize()
    assert torch.all(w[:, 36:] == 0)
    with pytest.raises(RuntimeError, match="past the end"):
        dev.check_status()


def test_graphed_device_fit_equals_eager_host_fit(cuda):
    cols = _columns(2600, 2)  # 5 full batches of 512 + a partial one
    a, b = _model(cuda, 3), _model(cuda, 3)
    ha = a.fit(EncodedDataset(cols, 512, 1000, seed=7, device=cuda), epochs=2, use_graph=False)
    hb = b.fit(DeviceDataset(cols, 512, 1000, seed=7, device=cuda), epochs=2, use_graph=True)
    torch.cuda.synchronize()
    assert b._device_fit_graph is not None  # the graphed device path ran
    np.testing.assert_allclose(hb["loss"], ha["loss"], rtol=1e-12)
    for ta, tb in zip(a.towers, b.towers):
        assert torch.equal(ta.dense.flat, tb.dense.flat)
        for n in ta.input_layer.embedding_layers:
            assert torch.equal(ta.input_layer.embedding_layers[n].weight, tb.input_layer.embedding_layers[n].weight)


def test_export_round_trip_and_retriever_on_raw_queries(cuda, tmp_path):
    m = _model(cuda, 5)
    m.fit(DeviceDataset(_columns(2048, 5), 512, device=cuda), epochs=1, use_graph=True)
    m.save(str(tmp_path / "model") + "/")
    r = TwoTowerModel.load(str(tmp_path / "model") + "/", device=cuda)
    q = {k: torch.as_tensor(v, device=cuda) for k, v in _columns(300, 9).items()}
    assert torch.equal(m.query_tower(q), r.query_tower(q))
    assert torch.equal(m.candidate_tower(q), r.candidate_tower(q))

    # index over string identifiers, searched with raw string queries
    art = [str(i) for i in range(300)]
    cand = {"art": torch.arange(1, 301, dtype=torch.int32, device=cuda),
            "ptn": torch.as_tensor(np.arange(300) % 21, dtype=torch.int32, device=cuda)}
    ids = np.array([f"article-{a}" for a in art])
    index = BruteForceIndex(10, m.query_tower, [(ids, m.candidate_tower(cand))])
    index.save(str(tmp_path / "index" / "i"))
    served = Retriever.load(str(tmp_path / "index" / "i"), device=cuda)
    rng = np.random.default_rng(3)
    raw = {"cust": [str(x) for x in rng.integers(0, 320, 64)],  # includes OOV ids
           "post": [str(x) for x in rng.integers(0, 60, 64)], "age": rng.standard_normal(64).astype(np.float32)}
    enc = m.query_tower.input_layer.encode(raw)
    want = index(enc)
    got, scores = served(raw, scores=True)
    assert np.array_equal(got, want)
    emb = m.query_tower(enc).cpu().numpy()
    rs, ri, _ = oracle.bruteforce_topk(emb, index._candidates.cpu().numpy(), 10)
    assert np.array_equal(got, ids[ri]) and np.array_equal(scores.cpu().numpy(), rs)


def test_graphed_fits_back_to_back_after_a_larger_graph(cuda):
    """In one process: a GraphedTrainStep of a third model at a LARGER batch
    (its workspaces grow past what the fits need), then graphed
    DeviceDataset fits of two different models on two different datasets
    back to back (each recapturing, each with a partial last batch), each
    bit-identical to the same model trained eagerly on the host batches."""
    from pkg.modelling.models.two_tower_model import GraphedTrainStep

    big = _model(cuda, 11)
    cols_big = _columns(4096, 12)
    g = GraphedTrainStep(big, {k: torch.as_tensor(v, device=cuda) for k, v in cols_big.items()}, warmup=1)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    for seed, (n, bs, shuffle) in ((21, (3000, 768, None)), (22, (2100, 256, 500))):
        cols = _columns(n, seed)
        a, b = _model(cuda, seed), _model(cuda, seed)
        ha = a.fit(EncodedDataset(cols, bs, shuffle, seed=seed, device=cuda), epochs=2, use_graph=False)
        hb = b.fit(DeviceDataset(cols, bs, shuffle, seed=seed, device=cuda), epochs=2, use_graph=True)
        torch.cuda.synchronize()
        assert b._device_fit_graph is not None
        np.testing.assert_allclose(hb["loss"], ha["loss"], rtol=1e-12)
        for ta, tb in zip(a.towers, b.towers):
            assert torch.equal(ta.dense.flat, tb.dense.flat)
            for name in ta.input_layer.embedding_layers:
                assert torch.equal(ta.input_layer.embedding_layers[name].weight,
                                   tb.input_layer.embedding_layers[name].weight), name
    g.replay()  # the first graph still replays after the fits' captures
    torch.cuda.synchronize()
