"""Runners (mirror of /root/reference/pkg/modelling/runner.py:18-152).

modelling_runner keeps the reference's flow: load the Schema, build the
train / test / candidate datasets, create the model and optimizer, then per
epoch: embed every candidate, build a BruteForceIndex, measure Recall@ks on
the test set BEFORE the epoch's training (runner.py:99-103), fit one epoch,
save model and index; finally re-log the last recall (runner.py:107).

Datasets are this framework's encoded shards (pkg.modelling.dataset) found in
the directories of the settings' *_tfrecord_path fields.  On the GPU they are
loaded into HBM once (DeviceDataset: batches assembled on the device) and
training replays one hipGraph per batch (take + train step); use_graph=False
or device_resident=False select the eager / host-batched paths.  If a shard carries
"__raw__<candidate_col>" (integer codes of the raw candidate ids), those are
used as index identifiers and recall ground truth, so OOV candidates that
share embedding row 0 remain distinct, as raw string ids are in the
reference.
"""
from __future__ import annotations

import logging
import os

import torch

from pkg.etl.transformations import date_filter, load_dataframe
from pkg.modelling.dataset import DeviceDataset, EncodedDataset
from pkg.modelling.indices.brute_force import BruteForceIndex
from pkg.modelling.indices.static_index import StaticIndex
from pkg.modelling.losses import CategoricalCrossentropy
from pkg.modelling.metrics.index_recall import IndexRecall
from pkg.modelling.models.two_tower_model import TwoTowerModel
from pkg.modelling.optimizer_factory import OptimizerFactory
from pkg.schema.schema import Schema
from pkg.utils.settings import Settings

logger = logging.getLogger(__name__)

RAW_PREFIX = "__raw__"


def modelling_runner(settings: Settings, use_graph: bool = True, device_resident: bool = True):
    """Train a Two-Tower Model and evaluate it (runner.py:18-108)."""
    logger.info("--- Modelling Starting ---")
    schema = Schema.load_from_filepath(settings.schema_filepath)
    tc = schema.training_config
    cand_col = settings.candidate_col_name
    raw_col = RAW_PREFIX + cand_col
    resident = device_resident and torch.cuda.is_available()
    loader = DeviceDataset.load if resident else EncodedDataset.load
    train_ds = loader(os.path.dirname(settings.train_data_tfrecord_path), tc.train_batch_size, tc.shuffle_size)
    test_ds = loader(os.path.dirname(settings.test_data_tfrecord_path), tc.test_batch_size)
    test_ds = test_ds.map(lambda x: ({f.name: x[f.name] for f in schema.query_features},
                                     x[raw_col] if raw_col in x else x[cand_col]))
    candidate_ds = loader(os.path.dirname(settings.candidate_tfrecord_path), tc.candidate_batch_size)

    model = TwoTowerModel.create_from_schema(schema, cand_col)
    optimizer = OptimizerFactory.get_optimizer(tc.optimizer_name, tc.optimizer_kwargs)
    model.compile(loss=CategoricalCrossentropy(from_logits=True, reduction="sum"), optimizer=optimizer)
    metric_calc = None
    for epoch in range(tc.epochs):
        candidate_embeddings = candidate_ds.map(
            lambda x: ((x[raw_col] if raw_col in x else x[cand_col]).reshape(-1), model.candidate_tower(x)))
        index = BruteForceIndex(max(schema.model_config.ks), model.query_tower, candidate_embeddings)
        metric_calc = IndexRecall(index, schema.model_config.ks)
        for query_features, true_candidates in test_ds:
            metric_calc(query_features, true_candidates)
        metric_calc.log_metric(epoch + 1)
        model.fit(train_ds, epochs=1, use_graph=use_graph)
        model.save(settings.trained_model_path)
        index.save(settings.index_path)
    if metric_calc is not None:
        # the reference re-logs the last pre-fit recall here (runner.py:107)
        metric_calc.log_metric(tc.epochs + 1)
    logger.info("--- Modelling Finishing ---")
    return model


def baseline_modelling_runner(settings: Settings):
    """Popularity baseline evaluated with the same recall (runner.py:111-152)."""
    logger.info("--- Baseline Modelling Starting ---")
    df = load_dataframe(settings.raw_data_filepath, "raw_transactions")
    schema = Schema.load_from_filepath(settings.schema_filepath)
    candidates = date_filter(df, "raw_transactions", settings.date_col_name,
                             settings.baseline_model_date_range)[settings.candidate_col_name]
    logger.info(f"Building Static Popularity Index using {len(candidates)} candidates")
    test_df = load_dataframe(settings.test_data_filepath, "test")
    index = StaticIndex.build_popularity_index_from_series_schema(schema, candidates)
    metric_calc = IndexRecall(index, schema.model_config.ks)
    bs = schema.training_config.test_batch_size
    for s in range(0, len(test_df), bs):
        part = test_df.iloc[s:s + bs]
        metric_calc({f.name: part[f.name].values for f in schema.query_features},
                    part[settings.candidate_col_name].astype(str).values)
    metric_calc.log_metric(None, to_tensorboard=False)
    index.save(settings.baseline_index_path)
    logger.info("--- Baseline Modelling Finishing ---")
    return metric_calc
