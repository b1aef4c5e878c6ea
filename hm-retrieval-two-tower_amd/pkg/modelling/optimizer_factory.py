"""Optimizers with tf.keras.optimizers.legacy semantics, applied by libtt.

Mirror of /root/reference/pkg/modelling/optimizer_factory.py:8-57 (same names,
same required kwargs and error messages).  The update rules are the legacy
Keras / TF kernels the reference reaches:
  Adagrad (initial_accumulator_value=0.1, epsilon=1e-7):
    dense  ResourceApplyAdagradV2        -> tt_dense_adagrad (one launch per tower)
    sparse dedup + ResourceSparseApplyAdagradV2 -> tt_sparse_adagrad
  Adam (beta_1=0.9, beta_2=0.999, epsilon=1e-7):
    dense  ResourceApplyAdam             -> tt_dense_adam
    sparse legacy _resource_apply_sparse (decays the WHOLE m/v slots, then a
           dense var update)              -> tt_sparse_adam
Slots are created on first use, as Keras creates them on the first
apply_gradients.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional
import logging

import torch

from pkg.modelling import hip_ops

logger = logging.getLogger(__name__)

__all__ = ["OptimizerFactory", "Adagrad", "Adam"]


class _Optimizer:
    def __init__(self, learning_rate: float = 0.001, name: str = "", **kwargs):
        self.learning_rate = float(learning_rate)
        self.name = name
        self.iterations = 0
        self._slots: Dict[int, List[torch.Tensor]] = {}
        if kwargs:
            unknown = set(kwargs) - {"clipnorm", "clipvalue", "global_clipnorm", "decay"}
            if unknown:
                raise TypeError(f"Unexpected keyword argument(s) passed to optimizer: {sorted(unknown)}")
            if any(kwargs.get(k) for k in ("clipnorm", "clipvalue", "global_clipnorm", "decay")):
                raise NotImplementedError("gradient clipping / decay are not supported")

    def _slot(self, param: torch.Tensor, n: int, init: float) -> List[torch.Tensor]:
        key = id(param)
        s = self._slots.get(key)
        if s is None or s[0].shape != param.shape:
            s = [torch.full_like(param, init, requires_grad=False) for _ in range(n)]
            self._slots[key] = s
        return s

    def apply_gradients(self, towers) -> None:
        """Dense step on each tower's flat MLP buffer, sparse step on its tables."""
        self._apply(towers)
        self.iterations += 1

    minimize = apply_gradients


class Adagrad(_Optimizer):
    def __init__(self, learning_rate: float = 0.001, initial_accumulator_value: float = 0.1, epsilon: float = 1e-7,
                 name: str = "Adagrad", **kwargs):
        super().__init__(learning_rate, name, **kwargs)
        if initial_accumulator_value < 0.0:
            raise ValueError(f"initial_accumulator_value must be non-negative: {initial_accumulator_value}")
        self.initial_accumulator_value = float(initial_accumulator_value)
        self.epsilon = float(epsilon)
        self._prepared = None
        self._side_streams = {}

    def _sparse_specs(self, towers, with_grad: bool, grad: Optional[torch.Tensor] = None):
        init = self.initial_accumulator_value
        specs, batch = [], None
        for tower in towers:
            layer = tower.input_layer
            if not layer.embedding_layers:
                continue
            g = grad if grad is not None else layer.last_grad
            if with_grad and g is None:
                continue
            for src in layer.sparse_sources():
                t = src["table"]
                (acc,) = self._slot(t.weight, 1, init)
                batch = src["ids"][0].numel()
                specs.append(dict(table=t.weight, slot0=acc, ids=src["ids"], grad_col_offset=src["grad_col_offset"],
                                  grad=g if with_grad else None))
        return specs, batch

    # -- per-tower application from inside the backward (TwoTowerModel.train_step)
    def prepare_towers(self, towers, scopes: List[str]) -> None:
        """One id sort per tower (tower i's workspace scope scopes[i]) on the
        side stream, before the backward, so each tower's update can be applied
        by apply_tower the moment that tower's gradients exist."""
        self._tower_prep = {}
        if not torch.cuda.is_available():
            return
        cur = torch.cuda.current_stream()
        side = self._side_streams.get(cur.device)
        if side is None:
            side = self._side_streams[cur.device] = torch.cuda.Stream(device=cur.device)
        side.wait_stream(cur)
        for tower, scope in zip(towers, scopes):
            with torch.cuda.stream(side), hip_ops.Workspace.scope(scope):
                specs, batch = self._sparse_specs([tower], with_grad=False)  # new accumulators filled on `side`
                if not specs or len(specs) > 16 or not batch:
                    # not presorted: apply_tower sorts on the current stream,
                    # which must first see the accumulators filled on `side`
                    if specs:
                        cur.wait_stream(side)
                    continue
                hip_ops.sparse_sort(specs, batch)
                key = hip_ops.Workspace._scope  # the apply must find its sorted keys in this scope's buffer
            done = torch.cuda.Event()
            done.record(side)
            self._tower_prep[id(tower)] = ([id(s["table"]) for s in specs], batch, done, key)

    def apply_dense(self, tower, flat_grad: torch.Tensor) -> None:
        """Tower's dense Adagrad step alone, on the current stream (the same
        update _apply makes from flat.grad)."""
        flat = tower.dense.flat
        (acc,) = self._slot(flat, 1, self.initial_accumulator_value)
        hip_ops.dense_adagrad(flat.data, acc, flat_grad, self.learning_rate, self.epsilon)

    def apply_tower(self, tower, input_grad: Optional[torch.Tensor], flat_grad: torch.Tensor) -> None:
        """Tower's dense Adagrad step and its tables' sparse step, on the current
        stream and workspace scope (the ones prepare_towers used for it)."""
        self.apply_dense(tower, flat_grad)
        self.apply_tower_sparse(tower, input_grad)

    def apply_tower_sparse(self, tower, input_grad: Optional[torch.Tensor]) -> None:
        """Tower's tables' sparse Adagrad step alone (apply_tower's second
        half), on the current stream and workspace scope."""
        lr, eps = self.learning_rate, self.epsilon
        prep = getattr(self, "_tower_prep", {}).pop(id(tower), None)
        if input_grad is None:
            return
        specs, batch = self._sparse_specs([tower], with_grad=True, grad=input_grad)
        if not specs:
            return
        if prep is None:  # prepare_towers skipped this tower: sort here
            hip_ops.sparse_adagrad(specs, batch, None, lr, eps)
            return
        torch.cuda.current_stream().wait_event(prep[2])
        if (prep[0] != [id(s["table"]) for s in specs] or prep[1] != batch
                or prep[3] != hip_ops.Workspace._scope):
            raise RuntimeError(f"apply_tower: presorted state {prep[0]}/{prep[1]}/{prep[3]!r} does not match "
                               f"this apply ({[id(s['table']) for s in specs]}/{batch}/{hip_ops.Workspace._scope!r})")
        hip_ops.sparse_adagrad(specs, batch, None, lr, eps, presorted=True)

    def prepare(self, towers, after: Optional[torch.cuda.Event] = None) -> None:
        """Start the embedding update's id sort early, on a side stream (it reads
        only the lookup ids of the last gather), so it overlaps the backward
        pass; apply_gradients then joins it.  `after`: an event of the current
        stream the sort must follow (default: everything queued so far).
        Optional: without it the sort runs inside apply_gradients."""
        self._prepared = None
        if not torch.cuda.is_available():
            return
        cur = torch.cuda.current_stream()
        side = self._side_streams.get(cur.device)
        if side is None:
            side = self._side_streams[cur.device] = torch.cuda.Stream(device=cur.device)
        if after is not None:
            side.wait_event(after)  # ordered after that point of this stream only
        else:
            side.wait_stream(cur)
        with torch.cuda.stream(side):
            # accumulators created here are filled on this stream, ahead of
            # anything ordered after the sort
            specs, batch = self._sparse_specs(towers, with_grad=False)
            if not specs or len(specs) > 16 or not batch:
                if specs:  # the apply sorts on `cur`: order it after the accumulator fills
                    cur.wait_stream(side)
                return
            hip_ops.sparse_sort(specs, batch)
        done = torch.cuda.Event()
        done.record(side)
        self._prepared = ([id(s["table"]) for s in specs], batch, done)

    def _apply(self, towers) -> None:
        lr, eps, init = self.learning_rate, self.epsilon, self.initial_accumulator_value
        for tower in towers:
            flat = tower.dense.flat
            if flat.grad is not None:
                (acc,) = self._slot(flat, 1, init)
                hip_ops.dense_adagrad(flat.data, acc, flat.grad, lr, eps)
        specs, batch = self._sparse_specs(towers, with_grad=True)
        prepared, self._prepared = self._prepared, None
        if prepared is not None:  # join the side stream before anything touches the workspace
            torch.cuda.current_stream().wait_event(prepared[2])
        if specs:
            # every tower's tables in ONE call: one sort, one block pass (each
            # table reads its own tower's input gradient)
            if prepared is None:
                hip_ops.sparse_adagrad(specs, batch, None, lr, eps)
            elif prepared[0] == [id(s["table"]) for s in specs] and prepared[1] == batch:
                hip_ops.sparse_adagrad(specs, batch, None, lr, eps, presorted=True)
            else:
                raise RuntimeError(f"apply_gradients: presorted state {prepared[0]}/{prepared[1]} does not match "
                                   f"this apply ({[id(s['table']) for s in specs]}/{batch})")

    def check_status(self, device: Optional[torch.device] = None) -> None:
        """Raise if any sparse apply since the last check found keys that were
        not its call's (libtt records it on the device instead of applying;
        tt_sparse_status).  Synchronises the current stream."""
        from pkg.modelling.losses import TOWER_C_SCOPE

        if not torch.cuda.is_available():
            return
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        for scope in ("", TOWER_C_SCOPE):
            hip_ops.sparse_status(dev, "sparse", scope)


class Adam(_Optimizer):
    def __init__(self, learning_rate: float = 0.001, beta_1: float = 0.9, beta_2: float = 0.999,
                 epsilon: float = 1e-7, amsgrad: bool = False, name: str = "Adam", **kwargs):
        super().__init__(learning_rate, name, **kwargs)
        if amsgrad:
            raise NotImplementedError("amsgrad is not supported")
        self.beta_1, self.beta_2, self.epsilon = float(beta_1), float(beta_2), float(epsilon)

    def _apply(self, towers) -> None:
        step = self.iterations + 1
        lr, b1, b2, eps = self.learning_rate, self.beta_1, self.beta_2, self.epsilon
        for tower in towers:
            flat = tower.dense.flat
            if flat.grad is not None:
                m, v = self._slot(flat, 2, 0.0)
                hip_ops.dense_adam(flat.data, m, v, flat.grad, lr, b1, b2, eps, step)
            layer = tower.input_layer
            if layer.last_grad is None or not layer.embedding_layers:
                continue
            specs = []
            for src in layer.sparse_sources():
                t = src["table"]
                m, v = self._slot(t.weight, 2, 0.0)
                specs.append(dict(table=t.weight, slot0=m, slot1=v, ids=src["ids"],
                                  grad_col_offset=src["grad_col_offset"]))
            hip_ops.sparse_adam(specs, layer.last_grad.shape[0], layer.last_grad, lr, b1, b2, eps, step)


class OptimizerFactory:
    """
    Fetch a supported optimizer instance using config.
    Some kwargs are required.
    """

    _supported_optimizers = {
        "adam": Adam,
        "adagrad": Adagrad,
    }

    _required_kwargs = ["learning_rate"]

    @classmethod
    def get_optimizer(cls, optimizer_name: str, optimizer_kwargs: Dict[str, Any]) -> _Optimizer:
        if optimizer_name not in cls._supported_optimizers:
            raise ValueError(
                "name must be one of "
                f"{list(cls._supported_optimizers.keys())}, "
                f"got {optimizer_name}"
            )
        for kwarg in cls._required_kwargs:
            if kwarg not in optimizer_kwargs:
                raise ValueError(f"kwarg {kwarg} not found in kwargs: {optimizer_kwargs}")
        logger.info(f"Creating {optimizer_name} obj with kwargs: {optimizer_kwargs}")
        return cls._supported_optimizers[optimizer_name](**optimizer_kwargs)
