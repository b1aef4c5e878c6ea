"""CPU: host-side logic of the reference-API mirror (no GPU compute).

Mirrors the reference's constructor validation (features.py:55-80,
two_tower_model.py:47-50, optimizer_factory.py:43-53), vocab building, the
StaticIndex/IndexRecall golden (tests/test_recall.py) through our classes,
the LogQCorrection golden (tests/test_layers.py) through our layer, and the
date_filter golden (tests/test_transformations.py).
"""
import json
import os

import numpy as np
import pandas as pd
import pytest
import torch

from pkg import dtypes
from pkg.etl.transformations import date_filter
from pkg.modelling.indices.static_index import StaticIndex
from pkg.modelling.layers.logq_correction import LogQCorrection
from pkg.modelling.metrics.index_recall import IndexRecall
from pkg.modelling.optimizer_factory import Adagrad, Adam, OptimizerFactory
from pkg.modelling.dataset import EncodedDataset, encode_dataframe
from pkg.schema.features import Feature, FeatureFamily
from pkg.schema.model_config import ModelConfig
from pkg.schema.schema import Schema
from pkg.schema.training_config import TrainingConfig
from pkg.utils.settings import Settings

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_tests.json")))


def test_feature_validation_mirrors_reference():
    with pytest.raises(TypeError):
        Feature("x", "int64", FeatureFamily.QUERY)
    with pytest.raises(ValueError):
        Feature("x", dtypes.string, "query")
    with pytest.raises(TypeError):
        Feature("x", dtypes.float32, FeatureFamily.QUERY, embedding_size=4)
    with pytest.raises(TypeError):
        Feature("x", dtypes.string, FeatureFamily.QUERY, embedding_size=4, max_vocab_size=2.5)
    f = Feature("x", "tf.string", FeatureFamily.QUERY, embedding_size=4)
    assert f.dtype == dtypes.string and not f.is_built
    n = Feature("p", dtypes.float32, FeatureFamily.QUERY, vocab=["a"])
    assert n.vocab is None and n.is_built


def test_vocab_from_dataframe_and_string_lookup():
    df = pd.DataFrame({"x": ["b", "a", "b", "c", "a", "b"]})
    f = Feature("x", dtypes.string, FeatureFamily.QUERY, embedding_size=4, max_vocab_size=2)
    f.set_vocab_from_dataframe(df)
    assert f.vocab.tolist() == ["b", "a"] and f.num_rows == 3
    assert f.encode(["a", b"b", "zz"]).tolist() == [2, 1, 0]
    with pytest.raises(ValueError):
        f.set_vocab_from_dataframe(pd.DataFrame({"y": [1]}))


def test_schema_split_build_save_load(tmp_path):
    feats = [Feature("q", dtypes.string, FeatureFamily.QUERY, embedding_size=4),
             Feature("c", dtypes.string, FeatureFamily.CANDIDATE, embedding_size=4, vocab=["u", "v"])]
    s = Schema(feats, TrainingConfig(8, 8, "adagrad", {"learning_rate": 0.1}), ModelConfig(4, [1, 2]))
    assert [f.name for f in s.query_features] == ["q"] and [f.name for f in s.candidate_features] == ["c"]
    s.build_features_from_dataframe(pd.DataFrame({"q": ["z", "z", "y"], "c": ["u", "u", "u"]}))
    assert s.query_features[0].vocab.tolist() == ["z", "y"]
    assert s.candidate_features[0].vocab.tolist() == ["u", "v"]  # given vocab kept
    s.set_candidate_prob_lookup({"u": 1.0})
    p = tmp_path / "sub" / "schema.pkl"
    s.save(str(p))
    t = Schema.load_from_filepath(str(p))
    assert t.training_config.candidate_prob_lookup == {"u": 1.0}
    assert t.query_features[0].encode(["y"]).tolist() == [2]


def test_optimizer_factory_errors_and_types():
    with pytest.raises(ValueError, match="name must be one of"):
        OptimizerFactory.get_optimizer("sgd", {"learning_rate": 0.1})
    with pytest.raises(ValueError, match="kwarg learning_rate not found"):
        OptimizerFactory.get_optimizer("adam", {})
    a = OptimizerFactory.get_optimizer("adagrad", {"learning_rate": 0.05})
    assert isinstance(a, Adagrad) and a.initial_accumulator_value == 0.1 and a.epsilon == 1e-7
    assert isinstance(OptimizerFactory.get_optimizer("adam", {"learning_rate": 1e-3}), Adam)


def test_two_tower_candidate_id_col_validation():
    from pkg.modelling.models.two_tower_model import TwoTowerModel

    q = Feature("q", dtypes.string, FeatureFamily.QUERY, embedding_size=4, vocab=["a"])
    c = Feature("c", dtypes.string, FeatureFamily.CANDIDATE, embedding_size=4, vocab=["b"])
    with pytest.raises(ValueError, match="not a candidate feature"):
        TwoTowerModel([q], [c], "q", 8, device=torch.device("cpu"))


def test_input_layer_duplicate_name_semantics():
    """main.py declares product_type_name twice (16 and 4): the dict keeps the
    last table (input_layer.py:31) and it is looked up twice (:66-67)."""
    from pkg.modelling.layers.input_layer import InputLayer

    v = ["x", "y"]
    feats = [Feature("a", dtypes.string, FeatureFamily.CANDIDATE, embedding_size=8, vocab=v),
             Feature("p", dtypes.string, FeatureFamily.CANDIDATE, embedding_size=16, vocab=v),
             Feature("p", dtypes.string, FeatureFamily.CANDIDATE, embedding_size=4, vocab=v),
             Feature("n", dtypes.float32, FeatureFamily.CANDIDATE)]
    layer = InputLayer(feats, device=torch.device("cpu"))
    assert list(layer.embedding_layers) == ["a", "p"]
    assert layer.embedding_layers["p"].dim == 4
    assert layer.output_dim == 1 + 8 + 4 + 4
    assert layer.column_offsets() == [1, 9, 13]


def test_main_schema_widths_match_survey():
    import bench

    s = bench.main_schema()
    from pkg.modelling.layers.input_layer import InputLayer

    assert InputLayer(s.query_features, device=torch.device("cpu")).output_dim == 258
    assert InputLayer(s.candidate_features, device=torch.device("cpu")).output_dim == 200


def test_static_index_recall_golden_host_path():
    g = GOLD["recall"]
    feats = [Feature("query_id", dtypes.string, FeatureFamily.QUERY, embedding_size=2)]
    idx = StaticIndex(k=g["k"], input_features=feats, candidates=np.array(g["static_candidates"]).reshape(1, -1))
    metric = IndexRecall(idx, ks=g["ks"])
    t = g["true_candidate_ids"]
    for s in range(0, len(t), g["batch_size"]):
        part = t[s:s + g["batch_size"]]
        metric({"query_id": np.array([[b"q"]] * len(part))}, np.array(part, dtype=object))
    for k, v in g["expected"].items():
        assert metric.metric[int(k)] == np.float64(v)


def test_logq_correction_golden():
    g = GOLD["logq"]
    layer = LogQCorrection(g["candidate_prob_lookup"])
    out = layer(torch.tensor(g["logits"]), g["candidate_ids"]).numpy()
    exp = np.asarray(g["expected"], np.float32)
    assert np.array_equal(np.round(out, 5), np.round(exp, 5))


def test_date_filter_golden():
    g = GOLD["date_filter"]
    df = pd.DataFrame({"date_col": g["date_col"]})
    for (lo, hi), (mn, mx) in zip(g["ranges"], g["expected_min_max"]):
        out = date_filter(df, "t", "date_col", (lo, hi))
        assert (out["date_col"].min(), out["date_col"].max()) == (mn, mx)


def test_encoded_dataset_batches_partial_last_and_shards(tmp_path):
    f = Feature("x", dtypes.string, FeatureFamily.QUERY, embedding_size=2, vocab=["a", "b"])
    n = Feature("v", dtypes.float32, FeatureFamily.QUERY)
    df = pd.DataFrame({"x": ["a", "b", "c", "a", "b"], "v": [1.0, 2.0, 3.0, 4.0, 5.0]})
    cols = encode_dataframe(df, [f, n])
    ds = EncodedDataset(cols, batch_size=2, device=torch.device("cpu"))
    bs = list(ds)
    assert [b["x"].tolist() for b in bs] == [[1, 2], [0, 1], [2]]
    ds.save(str(tmp_path), max_rows=3)
    back = EncodedDataset.load(str(tmp_path), batch_size=4, device=torch.device("cpu"))
    assert [b["v"].tolist() for b in back] == [[1.0, 2.0, 3.0, 4.0], [5.0]]
    sh = EncodedDataset(cols, batch_size=5, shuffle_size=5, seed=1, device=torch.device("cpu"))
    assert sorted(next(iter(sh))["v"].tolist()) == [1.0, 2.0, 3.0, 4.0, 5.0]


def test_settings_fields_match_reference():
    import dataclasses

    names = [f.name for f in dataclasses.fields(Settings)]
    assert names[:3] == ["raw_data_filepath", "articles_data_filepath", "customers_data_filepath"]
    assert names[-2:] == ["tensorboard_logs_dir", "max_tfrecord_rows"]
    assert len(names) == 19


def test_hip_ops_reject_cpu_tensors():
    """No CPU fallback: every op refuses host tensors."""
    from pkg.modelling import hip_ops

    q = torch.zeros(4, 8)
    with pytest.raises(ValueError, match="GPU"):
        hip_ops.inbatch_rows(q, q, None)
    with pytest.raises(ValueError, match="GPU"):
        hip_ops.gather_grouped([(torch.zeros(3, 2), torch.zeros(4, dtype=torch.int32), 0)], 4, torch.zeros(4, 2))


def test_workspace_scopes_nest_and_empty_scope_is_root():
    """A sort issued under scope(s) and the apply that reads its buffer must
    resolve the same key; scope("") is the root scope (the key prefix is "")."""
    from pkg.modelling.hip_ops import Workspace
    from pkg.modelling.losses import TOWER_C_SCOPE

    assert Workspace._scope == ""
    with Workspace.scope(""):
        assert Workspace._scope == ""
    with Workspace.scope(TOWER_C_SCOPE):
        assert Workspace._scope == TOWER_C_SCOPE + "/"
        with Workspace.scope(""):
            assert Workspace._scope == ""
        assert Workspace._scope == TOWER_C_SCOPE + "/"
    assert Workspace._scope == ""


def test_capture_topology_rules():
    """hip_ops.CaptureTopology (the capture guard's fork / join check) on
    stand-in streams: forks from the origin or from a branch and joins into
    the origin pass; a branch joining another branch raises NestedJoinError
    after joining every branch into the origin (the capture can still end)."""
    from pkg.modelling import hip_ops

    class S:
        def __init__(self, n):
            self.cuda_stream = n
            self.waited = []

        def __eq__(self, o):
            return isinstance(o, S) and o.cuda_stream == self.cuda_stream

        def __hash__(self):
            return self.cuda_stream

        def wait_stream(self, o):
            self.waited.append(o.cuda_stream)

    origin, s1, s2, s3 = S(0), S(1), S(2), S(3)
    t = hip_ops.CaptureTopology()
    t.origin = origin
    ev = {}

    def rec(name, stream, topo=None):
        ev[name] = object()
        (topo or t).source[id(ev[name])] = stream
        return ev[name]

    t.waiting(s1, rec("a", origin))      # fork from the origin
    t.waiting(s2, rec("b", s1))          # fork from a branch
    t.waiting(origin, rec("c", s2))      # the origin joins a branch
    t.waiting(s1, rec("d", origin))      # a branch waits on the origin again
    t.waiting(s3, rec("e", origin))
    with pytest.raises(hip_ops.NestedJoinError, match="origin"):
        t.waiting(s1, rec("f", s3))      # a branch joining a sibling branch
    assert sorted(origin.waited) == [1, 2, 3]  # every branch joined into the origin
    t2 = hip_ops.CaptureTopology()
    t2.origin = origin
    t2.waiting(s1, rec("g", origin, t2))
    t2.waiting(s2, rec("h", s1, t2))
    with pytest.raises(hip_ops.NestedJoinError):
        t2.waiting(s1, rec("i", s2, t2))     # tools/graph_fork_probe.py nested_join


def test_workspace_retired_buffers_follow_graph_lifetime():
    """hip_ops.Workspace: a buffer a live graph's snapshot holds is retired
    (kept) when it regrows, and freed once that graph (the snapshot's owner)
    is gone — no leak across captures (host logic, CPU tensors)."""
    import gc

    from pkg.modelling import hip_ops

    W = hip_ops.Workspace
    dev = torch.device("cpu", 0)
    with W.scope("t_lifetime"):
        a = W.get(1024, dev, "buf")

        class Graph:  # stands in for torch.cuda.CUDAGraph
            pass

        g = Graph()
        snap = W.snapshot(owner=g)
        assert W.unchanged(snap)
        b = W.get(4096, dev, "buf")  # regrowth while g may replay into `a`
        assert b.data_ptr() != a.data_ptr() and not W.unchanged(snap)
        assert any(r.data_ptr() == a.data_ptr() for r in W._retired)
        del g
        gc.collect()
        assert not any(r.data_ptr() == a.data_ptr() for r in W._retired)
        c = W.get(8192, dev, "buf")  # no live graph holds `b`: not retired
        assert not any(r.data_ptr() == b.data_ptr() for r in W._retired) and c.numel() >= 8192
    W._bufs = {k: v for k, v in W._bufs.items() if "t_lifetime" not in k[1]}
