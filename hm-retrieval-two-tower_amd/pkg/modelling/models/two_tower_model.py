"""TwoTowerModel (mirror of /root/reference/pkg/modelling/models/two_tower_model.py:12-205).

train_step (two_tower_model.py:94-130) on MI355X:
  1. query / candidate InputLayer gathers        tt_gather_multi (both towers + logq, 1 launch)
  2. tower MLPs                                   tt_mlp_rows (bf16x3 MFMA, bias + relu epilogue)
  3. scores + logQ + eye-label CE-SUM + dQ/dC     tt_inbatch_softmax_xent (rows + cols passes,
                                                  bf16 MFMA, fp32 accumulation)
  4. MLP backward                                 tt_mlp_wgrad weight + bias gradients and
                                                  tt_mlp_rows input gradients (ReluGrad fused)
  5. optimizer                                    tt_dense_adagrad + tt_sparse_adagrad (dedup in-kernel)
Every launch is stream-ordered with no host synchronisation, so the whole step
can be captured once and replayed as a hipGraph (GraphedTrainStep).
"""
from __future__ import annotations

import logging
import os
from typing import Any, Dict, Iterable, List, Optional

import numpy as np
import torch

from pkg.schema.features import Feature
from pkg.schema.schema import Schema
from pkg.modelling.device import default_device, make_generator
from pkg.modelling.layers.logq_correction import LogQCorrection
from pkg.modelling.losses import TOWER_C_SCOPE, InBatchSoftmaxCrossEntropy, towers_inbatch_softmax_xent
from pkg.modelling.models.abstract_keras_model import AbstractKerasModel, TensorSpec
from pkg.modelling import hip_ops
from pkg.modelling.layers.input_layer import InputLayer
from pkg.modelling.models import tower as _tower_mod
from pkg.modelling.models.tower import Tower

logger = logging.getLogger(__name__)

__all__ = ["TwoTowerModel", "GraphedTrainStep", "LOGQ_KEY"]

# Optional batch entry carrying per-example log p(candidate) computed from raw
# ids at encoding time (exact even for ids outside a truncated vocab).
LOGQ_KEY = "__logq__"
# where the embedding update's id sort may start: as soon as the batch's ids
# are gathered ("gather", default: 6 interleaved A/B pairs on the C3 step,
# 6.6 us/step faster than "loss" on average) or after the whole forward ("loss");
# either way it is captured after the backward, so its launch follows them
SORT_AFTER = os.environ.get("TT_SORT_AFTER", "gather")
# each tower's dense (MLP) Adagrad step issued inside the backward on that
# tower's stream the moment its weight gradient exists, instead of after the
# join (the embedding update stays one call after the backward)
DENSE_EARLY = os.environ.get("TT_DENSE_EARLY", "1") == "1"
# fused apply: the per-tower id sorts issued right after the gather
FUSED_SORT_EARLY = os.environ.get("TT_FUSED_SORT_EARLY", "1") == "1"
# with DENSE_EARLY: each layer's Adagrad step applied by its weight-gradient
# launches (tt_mlp_wgrad_adagrad: the partial-sum launch updates the layer)
# instead of one dense_adagrad launch per tower after its backward
FUSED_DENSE_WGRAD = os.environ.get("TT_FUSED_DENSE_WGRAD", "1") == "1"
# The towers' MLP weight images packed by the train step's gather launch
# (tt_gather_multi_pack) instead of one pack launch per tower at the start of
# each tower's forward (TT_PACK_WITH_GATHER=0).
PACK_WITH_GATHER = os.environ.get("TT_PACK_WITH_GATHER", "1") == "1"


class TwoTowerModel(AbstractKerasModel):
    """
    Two Tower Model class.

    Parameters
    ----------
    query_features: List[Feature]
        Features for the query tower.
    candidate_features: List[Feature]
        Features for the candidate tower.
    candidate_id_col: str
        The column containing the candidate_id.
    joint_embedding_size: int
        Joint embedding size which gets dot product.
    query_tower_units: Optional[List[int]]
        Hidden units for the query tower.
    candidate_tower_units: Optional[List[int]]
        Hidden units for the candidate tower.
    candidate_prob_lookup: Optional[Dict[str, float]]
        If provided, logQ correction is applied before the loss.
    """

    def __init__(self, query_features: List[Feature], candidate_features: List[Feature], candidate_id_col: str,
                 joint_embedding_size: int, query_tower_units: Optional[List[int]] = None,
                 candidate_tower_units: Optional[List[int]] = None,
                 candidate_prob_lookup: Optional[Dict[str, float]] = None,
                 device: Optional[torch.device] = None, seed: Optional[int] = None,
                 fused_optimizer_apply: bool = False):
        # apply each tower's Adagrad step inside the backward (see train_step)
        self.fused_optimizer_apply = bool(fused_optimizer_apply)
        self.query_features = query_features
        self.candidate_features = candidate_features
        if candidate_id_col not in [f.name for f in candidate_features]:
            raise ValueError(f"candidate_id_col {candidate_id_col} not a candidate feature")
        self.candidate_id_col = candidate_id_col
        self.device = device if device is not None else default_device()
        gen = make_generator(seed)
        self.query_tower = Tower(query_features, joint_embedding_size, query_tower_units, self.device, gen)
        self.candidate_tower = Tower(candidate_features, joint_embedding_size, candidate_tower_units, self.device, gen)
        self.logq_correction = LogQCorrection(candidate_prob_lookup) if candidate_prob_lookup else None
        self._logq_rows: Optional[torch.Tensor] = None
        self.optimizer = None
        self.loss = InBatchSoftmaxCrossEntropy()
        self.initialise_model()

    @property
    def towers(self) -> List[Tower]:
        return [self.query_tower, self.candidate_tower]

    # ------------------------------------------------------------------
    def _split(self, x: Dict[str, Any]):
        q = {f.name: x[f.name] for f in self.query_features}
        c = {f.name: x[f.name] for f in self.candidate_features}
        return q, c

    def call(self, x: Dict[str, Any], training: bool = True) -> torch.Tensor:
        """[Q, C] scores of every query against every candidate of the batch
        (two_tower_model.py:65-92); materialised.  An INSPECTION path, not
        the hot path: fit / train_step / the graphed and sharded steps never
        call it (they never form [B, B]: losses.towers_inbatch_softmax_xent,
        the fused tt_inbatch kernels).  The score matrix is libtt's
        (hip_ops.score_matrix, bf16x3 MFMA: fp32-faithful); with gradients
        enabled it is hip_ops.ScoreMatrix, whose backward GEMMs (dQ = G.C,
        dC = G^T.Q) run on the same kernel, so a caller can differentiate
        through it (the reference's tf.matmul semantics)."""
        q, c = self._split(x)
        with torch.set_grad_enabled(training and torch.is_grad_enabled()):
            qe, ce = self.query_tower.call(q), self.candidate_tower.call(c)
            if torch.is_grad_enabled():
                return hip_ops.ScoreMatrix.apply(qe, ce)
            return hip_ops.score_matrix(qe, ce)

    def candidate_logq(self, x: Dict[str, Any]) -> Optional[torch.Tensor]:
        """Per-example log p(candidate) [B] for the logQ correction, or None."""
        if self.logq_correction is None:
            return None
        if LOGQ_KEY in x:
            v = x[LOGQ_KEY]
            v = v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v, np.float32))
            return v.reshape(-1).to(device=self.device, dtype=torch.float32).contiguous()
        if self._logq_rows is None:
            feat = next(f for f in self.candidate_features if f.name == self.candidate_id_col)
            self._logq_rows = self.logq_correction.row_table(feat, self.device)
        ids = x[self.candidate_id_col]
        ids = ids if isinstance(ids, torch.Tensor) else torch.as_tensor(np.asarray(ids))
        ids = ids.reshape(-1).to(self.device, torch.int32).contiguous()
        # one libtt gather launch: the logq table is a 1-wide embedding of the
        # candidate ids (ids outside the table read 0 = the missing-id value)
        out = torch.empty(ids.numel(), 1, dtype=torch.float32, device=self.device)
        hip_ops.gather_grouped([(self._logq_rows.view(-1, 1), ids, 0)], ids.numel(), out)
        return out.view(-1)

    def _logq_call(self, x: Dict[str, Any]):
        """(segments, out) of the logQ lookup as a 1-wide gather call, or None
        when logQ comes another way (precomputed in the batch / disabled)."""
        if self.logq_correction is None or LOGQ_KEY in x:
            return None
        ids = x[self.candidate_id_col]
        if not isinstance(ids, torch.Tensor) or ids.device.type != "cuda" or ids.dtype != torch.int32:
            return None
        if self._logq_rows is None:
            feat = next(f for f in self.candidate_features if f.name == self.candidate_id_col)
            self._logq_rows = self.logq_correction.row_table(feat, self.device)
        ids = ids.reshape(-1).contiguous()
        out = torch.empty(ids.numel(), 1, dtype=torch.float32, device=self.device)
        return [(self._logq_rows.view(-1, 1), ids, 0)], out

    def compute_loss(self, x: Dict[str, Any], training: bool = True) -> torch.Tensor:
        q, c = self._split(x)
        with torch.set_grad_enabled(training):
            call = self._logq_call(x)  # rides in the towers' gather launch
            # ... and so do the towers' MLP weight images of this forward (at most 8 jobs)
            pack = []
            if training and PACK_WITH_GATHER and torch.is_grad_enabled() and self.device.type == "cuda":
                pack = [j for t in self.towers for j in t.dense.prepack_jobs(t.dense.flat.detach())]
                if len(pack) > 8:
                    for t in self.towers:
                        t.dense.__dict__["_prepacked"] = None
                    pack = []
            qi, ci = InputLayer.gather_many([self.query_tower.input_layer, self.candidate_tower.input_layer], [q, c],
                                            extra=[call] if call is not None else (), pack_jobs=pack or None)
            self._sort_issued = False
            if training and qi.is_cuda:
                # the embedding update's id sort needs only these ids
                self._ids_ready = torch.cuda.Event()
                self._ids_ready.record()
                if (SORT_AFTER == "early" and getattr(self, "_in_train_step", False)
                        and hasattr(self.optimizer, "prepare")
                        and getattr(self, "_on_tower", None) in (None, self._apply_dense_tower)):
                    # issued (and so captured) right here: a graph replays nodes
                    # in capture order, so a sort captured after the backward
                    # starts after it even when only the ids gate it
                    self.optimizer.prepare(self.towers, after=self._ids_ready)
                    self._sort_issued = True
                if (FUSED_SORT_EARLY and getattr(self, "_in_train_step", False)
                        and getattr(self, "_on_tower", None) == self._apply_tower):
                    # fused apply: the per-tower id sorts captured right after the
                    # gather (their only input), so they overlap the forward
                    # instead of landing in front of the backward
                    self.optimizer.prepare_towers(self.towers, ["", TOWER_C_SCOPE])
                    self._sort_issued = True
            logq = call[1].view(-1) if call is not None else self.candidate_logq(x)
            return self.tower_loss(qi, ci, logq)

    def tower_loss(self, qi: torch.Tensor, ci: torch.Tensor, logq: Optional[torch.Tensor]) -> torch.Tensor:
        """Loss from the gathered tower inputs: with gradients, both MLPs and the
        in-batch loss run as one autograd node (losses.towers_inbatch_softmax_xent)."""
        if torch.is_grad_enabled():
            return towers_inbatch_softmax_xent(qi, ci, self.query_tower.dense, self.candidate_tower.dense, logq,
                                               self.loss.reduction, getattr(self, "_on_tower", None),
                                               getattr(self, "_on_dx", None))
        return self.loss(self.query_tower.dense(qi), self.candidate_tower.dense(ci), logq)

    def compile(self, loss=None, optimizer=None, **kwargs) -> None:
        """Keras-style compile: the loss must be the in-batch softmax CE
        (CategoricalCrossentropy(from_logits=True, reduction=SUM) in the
        reference, runner.py:78-83)."""
        if loss is not None:
            if not isinstance(loss, InBatchSoftmaxCrossEntropy):
                raise TypeError("loss must be pkg.modelling.losses.CategoricalCrossentropy(from_logits=True, ...)")
            self.loss = loss
        if optimizer is not None:
            self.optimizer = optimizer
            # a cached fit graph holds the old optimizer's slot addresses
            self._device_fit_graph = None

    def check_optimizer_status(self) -> None:
        """Raise if a sparse apply since the last check refused stale or
        foreign keys (tt_sparse_status; one stream sync)."""
        check = getattr(self.optimizer, "check_status", None)
        if check is not None and self.device.type == "cuda":
            check(self.device)

    def train_step(self, data: Dict[str, Any]) -> Dict[str, torch.Tensor]:
        """One optimisation step on a batch of positive pairs; returns the
        (device) loss without synchronising.  With fused_optimizer_apply (opt-in,
        Adagrad on the GPU) each tower's dense and sparse updates are applied
        inside the backward, the moment that tower's gradients exist (the
        candidate tower's beside the query tower's backward); the updates are
        the same as applying them afterwards (each table and MLP buffer is
        touched by one tower only; tests/test_model_gpu.py checks bit-identity)."""
        from pkg.modelling.optimizer_factory import Adagrad

        if self.optimizer is None:
            raise RuntimeError("call compile(optimizer=...) before training")
        fused = self.fused_optimizer_apply and isinstance(self.optimizer, Adagrad) and self.device.type == "cuda"
        dense_early = (not fused and DENSE_EARLY and isinstance(self.optimizer, Adagrad)
                       and self.device.type == "cuda")
        self._dense_done = set()
        self._sparse_done = set()
        for t in self.towers:
            t.dense.fused_applied = set()
            t.dense.fused_adagrad = None
            if dense_early and FUSED_DENSE_WGRAD:
                opt = self.optimizer
                (acc,) = opt._slot(t.dense.flat, 1, opt.initial_accumulator_value)
                t.dense.fused_adagrad = (acc, opt.learning_rate, opt.epsilon)
        self._on_tower = self._apply_tower if fused else (self._apply_dense_tower if dense_early else None)
        # fused: each tower's embedding update the moment its input gradient
        # exists (the weight gradients follow it on that tower's stream)
        self._on_dx = self._apply_tower_sparse if (fused and _tower_mod.IGRAD_FIRST) else None
        self._in_train_step = True
        try:
            loss = self.compute_loss(data, training=True)
        finally:
            self._on_tower = None
            self._on_dx = None
            self._in_train_step = False
        fwd_done = None
        if fused and not getattr(self, "_sort_issued", False):
            # one id sort per tower on a side stream, before the backward needs it
            self.optimizer.prepare_towers(self.towers, ["", TOWER_C_SCOPE])
        elif hasattr(self.optimizer, "prepare") and loss.is_cuda and not getattr(self, "_sort_issued", False):
            if SORT_AFTER == "gather" and getattr(self, "_ids_ready", None) is not None:
                fwd_done = self._ids_ready
            else:
                fwd_done = torch.cuda.Event()
                fwd_done.record()
        if fwd_done is not None and SORT_AFTER == "mid":
            # captured between the forward and the backward: launched before the
            # backward's nodes, ordered after the forward only
            self.optimizer.prepare(self.towers, after=fwd_done)
            fwd_done = None
        for t in self.towers:
            t.dense.flat.grad = None
        if getattr(self, "_one", None) is None or self._one.device != loss.device:
            self._one = torch.ones((), dtype=loss.dtype, device=loss.device)
        try:
            loss.backward(self._one)  # a persistent seed: no ones-fill launch per step
        finally:
            for t in self.towers:
                t.dense.fused_adagrad = None
        if fused:
            self.optimizer.iterations += 1
            # the update is applied: a later apply_gradients must not apply it again
            for t in self.towers:
                t.dense.flat.grad = None
                t.input_layer.last_grad = None
        else:
            for i in self._dense_done:  # applied inside the backward: not again
                self.towers[i].dense.flat.grad = None
            self._dense_done = set()
            if fwd_done is not None:
                # the embedding update's id sort needs only the forward's ids; issued
                # after the backward (so the backward's chains are launched first)
                # but ordered only after the forward, it overlaps the backward
                self.optimizer.prepare(self.towers, after=fwd_done)
            self.optimizer.apply_gradients(self.towers)
        return {"loss": loss.detach()}

    def _apply_tower(self, i: int, input_grad: Optional[torch.Tensor], flat_grad: torch.Tensor) -> None:
        if i in self._sparse_done:  # its embedding update ran at the input gradient
            self.optimizer.apply_dense(self.towers[i], flat_grad)
            return
        self.optimizer.apply_tower(self.towers[i], input_grad, flat_grad)

    def _apply_tower_sparse(self, i: int, input_grad: Optional[torch.Tensor]) -> None:
        self.optimizer.apply_tower_sparse(self.towers[i], input_grad)
        self._sparse_done.add(i)

    def _apply_dense_tower(self, i: int, input_grad: Optional[torch.Tensor], flat_grad: torch.Tensor) -> None:
        st = self.towers[i].dense
        if st.fused_applied:  # the weight-gradient launches applied those layers' step
            for li, (w_off, fi, fo, _) in enumerate(st.layout):
                if li not in st.fused_applied:  # a layer outside tt_mlp_wgrad's contract
                    n = (fi + 1) * fo
                    (acc,) = self.optimizer._slot(st.flat, 1, self.optimizer.initial_accumulator_value)
                    hip_ops.dense_adagrad(st.flat.data[w_off:w_off + n], acc[w_off:w_off + n],
                                          flat_grad[w_off:w_off + n], self.optimizer.learning_rate,
                                          self.optimizer.epsilon)
        else:
            self.optimizer.apply_dense(self.towers[i], flat_grad)
        self._dense_done.add(i)

    def fit(self, dataset: Iterable[Dict[str, Any]], epochs: int = 1, callbacks=None,
            use_graph: bool = False) -> Dict[str, List[float]]:
        """Train for `epochs` passes; returns {"loss": [mean batch loss per epoch]}
        (Keras' loss metric is the running mean over the epoch's batches)."""
        from pkg.modelling.dataset import DeviceDataset

        if use_graph and isinstance(dataset, DeviceDataset) and dataset.fn is None and dataset.batch_size:
            return self._fit_device(dataset, epochs, callbacks)
        history: Dict[str, List[float]] = {"loss": []}
        graphed: Optional[GraphedTrainStep] = None
        for epoch in range(epochs):
            total = torch.zeros((), dtype=torch.float64, device=self.device)
            n = 0
            for batch in dataset:
                bs = next(iter(batch.values())).shape[0]
                if use_graph and graphed is None:
                    # the single warm-up step IS this batch's optimisation step
                    graphed = GraphedTrainStep(self, batch, warmup=1)
                    out = graphed.warmup_out
                elif use_graph and bs == graphed.batch_size:
                    out = graphed(batch)
                else:  # eager (also the partial last batch of a graphed epoch)
                    out = self.train_step(batch)
                total += out["loss"].double()
                n += 1
            self.check_optimizer_status()
            mean = float(total.item()) / max(n, 1)
            history["loss"].append(mean)
            logger.info(f"epoch {epoch + 1}/{epochs}: loss {mean:.6f} over {n} batches")
            for cb in callbacks or []:
                if callable(cb):
                    cb(epoch, {"loss": mean})
        return history

    def _fit_device(self, ds, epochs: int, callbacks) -> Dict[str, List[float]]:
        """fit over an HBM-resident DeviceDataset: each full batch is one replay
        of a graph that takes the batch on the device and trains on it; the
        partial last batch runs eagerly.  One host sync per epoch (the loss)."""
        history: Dict[str, List[float]] = {"loss": []}
        B, nfull = int(ds.batch_size), ds.full_batches
        rem = ds.num_rows - nfull * B
        graphed = None
        for epoch in range(epochs):
            ds.begin_epoch()
            todo = nfull
            # before every epoch's replays (the eager partial batch of the last
            # one, or other work since, may have regrown a workspace)
            graphed = getattr(self, "_device_fit_graph", None)
            if graphed is not None and not graphed.reusable(self, ds):
                graphed = self._device_fit_graph = None
            if todo and graphed is None:
                graphed = GraphedTrainStep(self, None, warmup=1, source=ds)  # warm-up = this epoch's batch 0
                self._device_fit_graph = graphed
                todo -= 1
            elif graphed is not None:
                graphed.loss_total.zero_()
            for _ in range(todo):
                graphed.graph.replay()
            total = graphed.loss_total.clone() if graphed is not None else torch.zeros(
                (), dtype=torch.float64, device=self.device)
            if rem:
                total += self.train_step(ds.view(ds.take(rem)))["loss"].double()
            ds.check_status()
            self.check_optimizer_status()
            n = nfull + (1 if rem else 0)
            mean = float(total.item()) / max(n, 1)
            history["loss"].append(mean)
            logger.info(f"epoch {epoch + 1}/{epochs}: loss {mean:.6f} over {n} batches (device-resident, graphed)")
            for cb in callbacks or []:
                if callable(cb):
                    cb(epoch, {"loss": mean})
        return history

    @classmethod
    def create_from_schema(cls, schema: Schema, candidate_id_col: str, **kwargs) -> "TwoTowerModel":
        """Instance from a Schema (two_tower_model.py:132-158)."""
        return TwoTowerModel(
            query_features=schema.query_features,
            candidate_features=schema.candidate_features,
            candidate_id_col=candidate_id_col,
            joint_embedding_size=schema.model_config.joint_embedding_size,
            query_tower_units=schema.model_config.query_tower_units,
            candidate_tower_units=schema.model_config.candidate_tower_units,
            candidate_prob_lookup=schema.training_config.candidate_prob_lookup,
            **kwargs,
        )

    def get_input_signature(self) -> Dict[str, TensorSpec]:
        return {f.name: TensorSpec((None, 1), f.dtype, f.name) for f in self.candidate_features + self.query_features}

    def state_dict(self) -> Dict[str, torch.Tensor]:
        sd = {f"query_tower.{k}": v for k, v in self.query_tower.state_dict().items()}
        sd.update({f"candidate_tower.{k}": v for k, v in self.candidate_tower.state_dict().items()})
        return sd

    def save(self, model_path: str) -> None:
        """Save the two-tower model and each tower separately in the
        two_tower / query_tower / candidate_tower entries of the model
        directory (two_tower_model.py:176-205): weights (.pt, weights-only),
        architecture (.json) and vocabularies (.npz) — pkg.modelling.export."""
        from pkg.modelling import export

        base = os.path.dirname(model_path)
        os.makedirs(base or ".", exist_ok=True)
        logging.info(f"Saving two_tower, query_tower, candidate_tower under {base or '.'}")
        export.save_two_tower(self, os.path.join(base, "two_tower"))
        export.save_tower(self.query_tower, os.path.join(base, "query_tower"))
        export.save_tower(self.candidate_tower, os.path.join(base, "candidate_tower"))

    @classmethod
    def load(cls, model_path: str, device: Optional[torch.device] = None) -> "TwoTowerModel":
        """The model saved by save(model_path) (compile() it again to train)."""
        from pkg.modelling import export

        return export.load_two_tower(os.path.join(os.path.dirname(model_path), "two_tower"), device)


class GraphedTrainStep:
    """Capture TwoTowerModel.train_step once as a hipGraph and replay it.

    The batch lives in two static device buffers (int32 ids [K, B], float32
    values [F, B]); a replay is one D2D copy per buffer (or none, for
    `replay()`), then the whole step — gathers, MLP GEMMs, the fused
    loss kernels and the optimizer kernels — with no Python or launch
    overhead.  Warm-up steps (run eagerly on a side stream before capture)
    are real optimisation steps on the example batch.  Requires an optimizer
    whose kernels do not depend on the host step count (Adagrad)."""

    def __init__(self, model: TwoTowerModel, example_batch: Optional[Dict[str, Any]], warmup: int = 2,
                 source=None):
        """source: a pkg.modelling.dataset.DeviceDataset whose next batch is
        taken on the device inside the graph (tt_batch_take, cursor in device
        memory) — every replay then trains on the dataset's next batch and
        adds its loss to `loss_total` (fp64, device) with no host work."""
        from pkg.modelling.optimizer_factory import Adagrad

        if not isinstance(model.optimizer, Adagrad):
            raise ValueError("graph capture needs the Adagrad optimizer (Adam's coefficients depend on the step)")
        self.model = model
        self.source = source
        if source is not None:
            if not source.batch_size:
                raise ValueError("a graphed DeviceDataset source needs a batch_size")
            self.int_keys, self.float_keys = list(source.int_keys), list(source.float_keys)
            self.batch_size = int(source.batch_size)
            ex = None
        else:
            ex = {k: self._to_dev(v, model.device).reshape(-1) for k, v in example_batch.items()}
            self.int_keys = sorted(k for k, v in ex.items() if v.dtype != torch.float32)
            self.float_keys = sorted(k for k, v in ex.items() if v.dtype == torch.float32)
            self.batch_size = next(iter(ex.values())).shape[0]
        B = self.batch_size
        K, F = len(self.int_keys), len(self.float_keys)
        # one [K + F, B] buffer of 32-bit words: int rows first, then float rows
        # (the DeviceDataset layout, so one take launch fills the whole batch)
        self._wbuf = torch.empty(max(K + F, 1), B, dtype=torch.int32, device=model.device)
        self._ibuf = self._wbuf[:K] if K else torch.empty(1, B, dtype=torch.int32, device=model.device)
        self._fbuf = (self._wbuf[K:K + F].view(torch.float32) if F
                      else torch.empty(1, B, dtype=torch.float32, device=model.device))
        self.static = {k: self._ibuf[i] for i, k in enumerate(self.int_keys)}
        self.static.update({k: self._fbuf[i] for i, k in enumerate(self.float_keys)})
        self.loss_total = torch.zeros((), dtype=torch.float64, device=model.device)
        if ex is not None:
            self.load(ex)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(warmup, 1)):
                out = self._step()
            self.warmup_out = {k: v.clone() for k, v in out.items()}
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        # thread_local: other host threads (a process group's watchdog, the
        # dataset's order prefetch) may query events while this thread captures
        self._graph_events: list = []  # events created during the capture live as long as the graph
        with hip_ops.capture_guard(self._graph_events), torch.cuda.graph(self.graph,
                                                                          capture_error_mode="thread_local"):
            self.out = self._step()
        # what the captured pointers refer to (see reusable)
        self.optimizer = model.optimizer
        self.ws_snapshot = hip_ops.Workspace.snapshot(owner=self.graph)

    def reusable(self, model: "TwoTowerModel", source=None) -> bool:
        """True while a replay still trains `model` from `source` through the
        buffers it was captured with: same optimizer object (its slots), no
        libtt workspace regrown or cleared since the capture."""
        return (self.model is model and self.source is source and self.optimizer is model.optimizer
                and (source is None or int(source.batch_size) == self.batch_size)
                and hip_ops.Workspace.unchanged(self.ws_snapshot))

    def _step(self) -> Dict[str, torch.Tensor]:
        if self.source is not None:
            self.source.take(self.batch_size, out=self._wbuf)
        out = self.model.train_step(self.static)
        if self.source is not None:
            self.loss_total += out["loss"].double()
        return out

    @staticmethod
    def _to_dev(v, device):
        t = v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))
        return t.to(device)

    def pack(self, batch: Dict[str, Any]):
        """Device buffers laid out like the static batch (copy with one D2D each)."""
        ib = torch.stack([self._to_dev(batch[k], self.model.device).reshape(-1).to(torch.int32)
                          for k in self.int_keys]) if self.int_keys else self._ibuf.clone()
        fb = torch.stack([self._to_dev(batch[k], self.model.device).reshape(-1).to(torch.float32)
                          for k in self.float_keys]) if self.float_keys else self._fbuf.clone()
        return ib.contiguous(), fb.contiguous()

    def load(self, batch: Dict[str, Any]) -> None:
        for k, v in batch.items():
            self.static[k].copy_(self._to_dev(v, self.model.device).reshape(-1), non_blocking=True)

    def replay(self) -> Dict[str, torch.Tensor]:
        self.graph.replay()
        return self.out

    def __call__(self, batch: Optional[Dict[str, Any]] = None, packed=None) -> Dict[str, torch.Tensor]:
        if packed is not None:
            self._ibuf.copy_(packed[0], non_blocking=True)
            if self.float_keys:
                self._fbuf.copy_(packed[1], non_blocking=True)
        elif batch is not None:
            self.load(batch)
        return self.replay()
