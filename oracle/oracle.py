"""CPU restatement of the reference hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / reported CPU baseline.  The
product (hm-retrieval-two-tower_amd/pkg) never imports it.

Every function restates SelvinSelbaraju/hm-retrieval-two-tower (cited as
/root/reference/<file>:<line>) on numpy / plain C.  The reference itself
cannot run here (TensorFlow is not installed), so parity is
pinned by the golden values of the reference's own tests
(tests/golden/reference_tests.json, checked by tests/test_oracle.py) and,
for the paths no reference test covers (gather, dedup + Adagrad, in-batch
loss and gradients, top-k tie breaking), by this restatement alone
("parity unpinned by the reference").
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_float, c_int, c_int32, c_int64, c_void_p
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libtt_oracle.so")
_lib = None

# Keras legacy Adagrad defaults (tf.keras.optimizers.legacy.Adagrad).
ADAGRAD_INITIAL_ACCUMULATOR = 0.1
ADAGRAD_EPSILON = 1e-7
# GPU summation block (csrc/tt_sparse.hip kBlock).
GPU_DEDUP_CHUNK = 32


def build() -> str:
    """Compile the C restatement (make -C oracle) if needed; returns the .so path."""
    if not os.path.exists(_SO):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_SO)
        L.oracle_bruteforce_topk.restype = c_int
        L.oracle_bruteforce_topk.argtypes = [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64, c_int, c_int,
                                             c_void_p, c_void_p, c_int]
        L.oracle_scores.restype = None
        L.oracle_scores.argtypes = [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64, c_int, c_void_p]
        L.oracle_dedup_sum.restype = c_int
        L.oracle_dedup_sum.argtypes = [c_void_p, c_int64, c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p]
        L.oracle_sparse_adagrad_apply.restype = None
        L.oracle_sparse_adagrad_apply.argtypes = [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_float,
                                                  c_float]
        _lib = L
    return _lib


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


def _i32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.int32)


# ---------------------------------------------------------------------------
# a1: vocab / StringLookup (features.py:106-127, input_layer.py:33-36)
def vocab_from_values(values: Sequence, max_vocab_size: Optional[int] = None) -> np.ndarray:
    """value_counts() order (count desc, first-seen on ties), head(max), str()."""
    import pandas as pd

    vc = pd.Series(list(values)).value_counts()
    idx = list(vc.head(max_vocab_size).index) if max_vocab_size else list(vc.index)
    return np.array([str(x) for x in idx])


def string_lookup(vocab: Sequence[str], values: Sequence) -> np.ndarray:
    """StringLookup(num_oov_indices=1): vocab[i] -> i+1, anything else -> 0."""
    table = {v: i + 1 for i, v in enumerate(vocab)}
    return np.array([table.get(str(v) if not isinstance(v, bytes) else v.decode(), 0) for v in values],
                    dtype=np.int32)


# ---------------------------------------------------------------------------
# a2: InputLayer.call (input_layer.py:45-69)
def gather_concat(numeric: Sequence[np.ndarray], tables: Sequence[np.ndarray], ids: Sequence[np.ndarray]) -> np.ndarray:
    """Numeric columns first, then table[ids] per categorical feature, concat."""
    cols: List[np.ndarray] = [np.asarray(v, np.float32).reshape(-1, 1) for v in numeric]
    for t, i in zip(tables, ids):
        i = np.asarray(i, np.int64).reshape(-1)
        valid = (i >= 0) & (i < t.shape[0])
        g = np.zeros((i.size, t.shape[1]), np.float32)
        g[valid] = t[i[valid]]
        cols.append(g)
    return np.concatenate(cols, axis=1) if cols else np.zeros((0, 0), np.float32)


# ---------------------------------------------------------------------------
# a7: LogQCorrection (logq_correction.py:32-42, 66-71); prob table etl/runner.py:75-78
def logq_from_lookup(candidate_ids: Sequence, lookup: Dict[str, float]) -> np.ndarray:
    """log(p[id]) in fp32 with the StaticHashTable default 1.0 (-> 0)."""
    p = np.array([lookup.get(str(x) if not isinstance(x, bytes) else x.decode(), 1.0) for x in candidate_ids],
                 dtype=np.float32)
    return np.log(p).astype(np.float32)


def logq_correction(logits: np.ndarray, candidate_ids: Sequence, lookup: Dict[str, float]) -> np.ndarray:
    """logits [B,B] - log p[candidate_ids]^T broadcast over rows."""
    return (np.asarray(logits, np.float32) - logq_from_lookup(candidate_ids, lookup)[None, :]).astype(np.float32)


def prob_lookup_from_values(values: Sequence) -> Dict[str, float]:
    """etl/runner.py:75-78: p = value_counts / len(train), keys str(id)."""
    import pandas as pd

    s = pd.Series(list(values))
    probs = s.value_counts() / len(s)
    return {str(probs.index[i]): float(probs.iloc[i]) for i in range(len(probs))}


# ---------------------------------------------------------------------------
# a5: Tower.call (tower.py:41-49, 51-75): Dense(relu)* then Dense(E, relu)
def tower_forward(x: np.ndarray, layers: Sequence[Tuple[np.ndarray, np.ndarray]], dtype=np.float64) -> np.ndarray:
    h = np.asarray(x, dtype)
    for w, b in layers:
        h = np.maximum(h @ np.asarray(w, dtype) + np.asarray(b, dtype), 0)
    return h


# ---------------------------------------------------------------------------
# a6-a8: scores, logQ, CE(from_logits, SUM) with eye labels and its gradient
# (two_tower_model.py:92, 113-124; runner.py:78-83)
def inbatch_softmax_xent(q: np.ndarray, c: np.ndarray, logq: Optional[np.ndarray] = None, pos_offset: int = 0,
                         dtype=np.float64):
    """Returns dict(loss, row_loss, lse, dq, dc) for local rows q [R,E] against
    columns c [C,E]; the positive of row i is column i + pos_offset.  dc is
    the column gradient of THIS row block (sum over blocks = full dc)."""
    q = np.asarray(q, dtype)
    c = np.asarray(c, dtype)
    R = q.shape[0]
    S = q @ c.T
    if logq is not None:
        S = S - np.asarray(logq, dtype)[None, :]
    m = S.max(axis=1)
    e = np.exp(S - m[:, None])
    lse = m + np.log(e.sum(axis=1))
    rows = np.arange(R)
    pos = rows + pos_offset
    row_loss = lse - S[rows, pos]
    P = e / e.sum(axis=1, keepdims=True)
    P[rows, pos] -= 1.0
    return {
        "loss": row_loss.sum(),
        "row_loss": row_loss,
        "lse": lse,
        "dq": P @ c,
        "dc": P.T @ q,
    }


def bf16_round(x: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 -> fp32, round to nearest even (v_cvt_pk_bf16_f32; the
    in-batch prep and P packing of csrc/tt_inbatch.hip)."""
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


# log2(e) as the kernels hold it (an fp32 constant)
LOG2E_F32 = float(np.float32(1.4426950408889634))


def _exp2_arg(s32: np.ndarray, m: np.ndarray) -> np.ndarray:
    """fp32 fmaf(s, LOG2E_F32, -m) for fp32 s and integer-valued m: the fp64
    product of two fp32 values is exact and so is subtracting the integer,
    so one rounding to fp32 gives exactly the fused result."""
    return (np.asarray(s32, np.float32).astype(np.float64) * LOG2E_F32 - m).astype(np.float32)


def _softplus(x: np.ndarray) -> np.ndarray:
    return np.where(x > 0, x + np.log1p(np.exp(-np.abs(x))), np.log1p(np.exp(np.minimum(x, 0.0))))


def inbatch_softmax_xent_bf16(q: np.ndarray, c: np.ndarray, logq: Optional[np.ndarray] = None, pos_offset: int = 0,
                              rows_q: Optional[np.ndarray] = None, block: int = 2048) -> Dict[str, np.ndarray]:
    """The arithmetic contract of tt_inbatch_* (include/tt.h), restated: the
    same loss and gradients as inbatch_softmax_xent (two_tower_model.py:92,
    113-124; logq_correction.py:66-71), computed the way the kernels compute
    them, so the GPU can be held to it tightly:
      * negative pairs: S = bf16(q) . bf16(c) (RNE, exact products, rounded to
        fp32) - logq; p = fp32(2^(S log2e - M)) with M an integer (the kernel's
        running max is an integer in log2 units, so any integer gives the same
        bf16(p) up to rare last-bit ties of the fp32 exponent argument); the
        P.C product uses bf16(p) and bf16(c); the row sum L uses the fp32 p;
      * the positive pair is scored in fp32: a = lse over the negatives,
        row_loss = softplus(a - pos), dq = sigmoid(a - pos) (O / L - c_pos);
      * columns (every row i of q against c, with the rows' lse and loss):
        p = bf16(fp32(exp(bf16(q_i).bf16(c_j) - lse_i))) for the negatives,
        dc_j = exp(-logq_j) sum_i p bf16(q_i) - (-expm1(-row_loss_pos)) q_pos.
    Rows q [R,E] against columns c [C,E]; the positive of row i is column
    i + pos_offset.  `rows_q` ([C + ...] rows for the column pass; default q
    with R == C) is every row of the batch when q holds one rank's block.
    Returns dict(loss, row_loss, lse, dq) and, when the rows cover every
    column's positive (rows_q None and R == C, pos_offset 0), dc."""
    q32, c32 = np.asarray(q, np.float32), np.asarray(c, np.float32)
    R, E = q32.shape
    C = c32.shape[0]
    qb = bf16_round(q32).astype(np.float64)
    cb = bf16_round(c32).astype(np.float64)
    lq = np.zeros(C) if logq is None else np.asarray(logq, np.float32).astype(np.float64)
    pos = np.arange(R) + pos_offset
    # fp32 positive logits (q_i . c_pos in fp64, rounded; the GPU's fp32 fma
    # chain agrees to a few ulp)
    pos_logit = (np.einsum("ij,ij->i", q32.astype(np.float64), c32[pos].astype(np.float64)) - lq[pos])
    pos_logit = pos_logit.astype(np.float32).astype(np.float64)
    row_loss = np.empty(R)
    lse = np.empty(R)
    dq = np.empty((R, E))
    for r0 in range(0, R, block):
        r1 = min(R, r0 + block)
        S = ((qb[r0:r1] @ cb.T) - lq[None, :]).astype(np.float32).astype(np.float64)
        rr = np.arange(r1 - r0)
        S[rr, pos[r0:r1]] = -np.inf
        mx = (S.max(axis=1) * LOG2E_F32)
        M = np.where(np.isfinite(mx), np.ceil(mx), 0.0)
        p = np.exp2(_exp2_arg(S, M[:, None]).astype(np.float64)).astype(np.float32)
        L = p.astype(np.float64).sum(axis=1)
        O = bf16_round(p).astype(np.float64) @ cb
        none = ~(L > 0)
        with np.errstate(divide="ignore", invalid="ignore"):
            a = np.where(none, -np.inf, M * np.log(2.0) + np.log(np.where(none, 1.0, L)))
            d = a - pos_logit[r0:r1]
            loss = np.where(none, 0.0, _softplus(np.where(none, 0.0, d)))
            g = np.where(none, 0.0, 1.0 / (1.0 + np.exp(-np.where(none, 0.0, d))))
            mean = np.where(none[:, None], 0.0, O / np.where(none, 1.0, L)[:, None])
        dq[r0:r1] = g[:, None] * (mean - c32[pos[r0:r1]].astype(np.float64))
        row_loss[r0:r1] = loss
        lse[r0:r1] = pos_logit[r0:r1] + loss
    row_loss32 = row_loss.astype(np.float32)
    lse32 = (pos_logit.astype(np.float32) + row_loss32).astype(np.float32)
    out = {"loss": float(row_loss32.astype(np.float64).sum()), "row_loss": row_loss32, "lse": lse32,
           "dq": dq.astype(np.float32)}
    if rows_q is None and R == C and pos_offset == 0:
        out["dc"] = inbatch_cols_bf16(q32, lse32, row_loss32, c32, logq, 0, block)
    return out


def inbatch_cols_bf16(q_all: np.ndarray, lse: np.ndarray, row_loss: np.ndarray, c: np.ndarray,
                      logq: Optional[np.ndarray] = None, pos_offset: int = 0, block: int = 2048) -> np.ndarray:
    """Column pass of the contract (inbatch_softmax_xent_bf16): dc [C,E] of the
    columns c against every row q_all [R,E] with its lse and row_loss; the
    positive of column j is row j + pos_offset."""
    q32, c32 = np.asarray(q_all, np.float32), np.asarray(c, np.float32)
    R, E = q32.shape
    C = c32.shape[0]
    qb = bf16_round(q32).astype(np.float64)
    cb = bf16_round(c32).astype(np.float64)
    lse64 = np.asarray(lse, np.float32).astype(np.float64)
    O = np.zeros((C, E))
    cols = np.arange(C)
    for r0 in range(0, R, block):
        r1 = min(R, r0 + block)
        s = ((qb[r0:r1] @ cb.T) - lse64[r0:r1, None]).astype(np.float32).astype(np.float64)
        hit = (cols + pos_offset >= r0) & (cols + pos_offset < r1)
        s[cols[hit] + pos_offset - r0, cols[hit]] = -np.inf
        p = np.exp2(_exp2_arg(s, 0.0).astype(np.float64)).astype(np.float32)
        O += bf16_round(p).astype(np.float64).T @ qb[r0:r1]
    scale = np.ones(C) if logq is None else np.exp(-np.asarray(logq, np.float32).astype(np.float64))
    omp = -np.expm1(-np.asarray(row_loss, np.float32).astype(np.float64)[cols + pos_offset])
    return (O * scale[:, None] - omp[:, None] * q32[cols + pos_offset].astype(np.float64)).astype(np.float32)


# bf16 operands (8 significant bits, round to nearest): unit roundoff 2^-8 per
# operand, so a product of two rounded operands is within 2^-7 + 2^-16 of the
# exact one; fp32 accumulation of <= 128 exact bf16 products adds < 2^-17.
BF16_DOT_EPS = 2.0 ** -7 + 2.0 ** -15


def inbatch_error_bound(q: np.ndarray, c: np.ndarray, pos_offset: int = 0) -> Dict[str, np.ndarray]:
    """Certified bound of the fused bf16-MFMA loss against the exact one.

    Each score S'_ij is computed from bf16(q_i) . bf16(c_j):
      |S~_ij - S_ij| <= d_ij = BF16_DOT_EPS * sum_k |q_ik| |c_jk|.
    lse is a softmax-weighted mean of the perturbations, so
      |lse~_i - lse_i| <= max_j d_ij  (+ fp32 softmax arithmetic, ~1e-5 |lse|),
    and the positive logit is an fp32 dot product, so the row loss has the
    same bound and the batch loss at most the sum of the rows'.
    Returns dict(lse=[R], loss=float)."""
    A = np.abs(np.asarray(q, np.float64)) @ np.abs(np.asarray(c, np.float64)).T
    row = BF16_DOT_EPS * A.max(axis=1)
    return {"lse": row, "loss": float(row.sum())}


# ---------------------------------------------------------------------------
# a3/a4: dedup + sparse Adagrad (legacy Keras optimizer; see tt_oracle.c)
def dedup_sum(ids: np.ndarray, grad: np.ndarray, chunk: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    ids = _i32(ids).reshape(-1)
    grad = _f32(grad)
    n, dim = grad.shape
    uniq = np.empty(max(n, 1), np.int32)
    sums = np.empty((max(n, 1), dim), np.float32)
    u = lib().oracle_dedup_sum(ids.ctypes.data, n, grad.ctypes.data, grad.strides[0] // 4, dim, chunk,
                               uniq.ctypes.data, sums.ctypes.data)
    return uniq[:u].copy(), sums[:u].copy()


def sparse_adagrad(table: np.ndarray, accum: np.ndarray, ids: np.ndarray, grad: np.ndarray, lr: float,
                   eps: float = ADAGRAD_EPSILON, chunk: int = GPU_DEDUP_CHUNK) -> None:
    """In place: dedup (ids out of [0, rows) skipped) then Adagrad per distinct row."""
    ids = _i32(ids).reshape(-1)
    valid = (ids >= 0) & (ids < table.shape[0])
    uniq, sums = dedup_sum(ids[valid], _f32(grad)[valid], chunk)
    assert table.dtype == np.float32 and accum.dtype == np.float32 and table.flags.c_contiguous
    lib().oracle_sparse_adagrad_apply(table.ctypes.data, accum.ctypes.data, table.shape[1], uniq.ctypes.data,
                                      sums.ctypes.data, len(uniq), lr, eps)


def dense_adagrad(param: np.ndarray, accum: np.ndarray, grad: np.ndarray, lr: float,
                  eps: float = ADAGRAD_EPSILON) -> None:
    """ResourceApplyAdagradV2: accum += g^2; var -= g*lr / (sqrt(accum) + eps) (fp32, in place)."""
    g = _f32(grad)
    lr = np.float32(lr)
    eps = np.float32(eps)
    accum += g * g
    param -= (g * lr) / (np.sqrt(accum) + eps)


def dense_adam(param, m, v, grad, lr, beta1, beta2, eps, step) -> None:
    """ResourceApplyAdam (fp32, in place)."""
    f = np.float32
    g = _f32(grad)
    b1p = f(np.power(f(beta1), f(step)))
    b2p = f(np.power(f(beta2), f(step)))
    alpha = f((f(lr) * np.sqrt(f(1) - b2p)) / (f(1) - b1p))
    m += (g - m) * (f(1) - f(beta1))
    v += (g * g - v) * (f(1) - f(beta2))
    param -= (m * alpha) / (np.sqrt(v) + f(eps))


def sparse_adam(table, m, v, ids, grad, lr, beta1, beta2, eps, step, chunk: int = GPU_DEDUP_CHUNK) -> None:
    """Legacy Adam._resource_apply_sparse after dedup (fp32, in place)."""
    f = np.float32
    ids = _i32(ids).reshape(-1)
    valid = (ids >= 0) & (ids < table.shape[0])
    uniq, sums = dedup_sum(ids[valid], _f32(grad)[valid], chunk)
    b1p = f(np.power(f(beta1), f(step)))
    b2p = f(np.power(f(beta2), f(step)))
    lr_t = f(f(lr) * (np.sqrt(f(1) - b2p) / (f(1) - b1p)))
    m *= f(beta1)
    v *= f(beta2)
    m[uniq] += sums * (f(1) - f(beta1))
    v[uniq] += (sums * sums) * (f(1) - f(beta2))
    table -= (lr_t * m) / (np.sqrt(v) + f(eps))


# ---------------------------------------------------------------------------
# a10: BruteForceIndex.call (brute_force.py:75-83)
def bruteforce_topk(q: np.ndarray, c: np.ndarray, k: int, threads: int = 0) -> Tuple[np.ndarray, np.ndarray, int]:
    """Exact fp32 fmaf-chain scores, top-k (score desc, index asc).  Returns
    (scores [Q,k], indices [Q,k] int32, threads used)."""
    q = _f32(q)
    c = _f32(c)
    nq, d = q.shape
    n = c.shape[0]
    if k > n:
        raise ValueError(f"k={k} > number of candidates {n}")
    out_s = np.empty((nq, k), np.float32)
    out_i = np.empty((nq, k), np.int32)
    used = lib().oracle_bruteforce_topk(q.ctypes.data, d, nq, c.ctypes.data, d, n, d, k, out_s.ctypes.data,
                                        out_i.ctypes.data, threads)
    return out_s, out_i, used


def fmaf_scores(q: np.ndarray, c: np.ndarray) -> np.ndarray:
    q = _f32(q)
    c = _f32(c)
    out = np.empty((q.shape[0], c.shape[0]), np.float32)
    lib().oracle_scores(q.ctypes.data, q.shape[1], q.shape[0], c.ctypes.data, c.shape[1], c.shape[0], q.shape[1],
                        out.ctypes.data)
    return out


def topk_merge(scores: np.ndarray, idx: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """[L,Q,k_in] sorted lists -> global top-k with the top_k order."""
    L, Q, kin = scores.shape
    s = np.transpose(scores, (1, 0, 2)).reshape(Q, L * kin)
    i = np.transpose(idx, (1, 0, 2)).reshape(Q, L * kin)
    order = np.lexsort((i, -s.astype(np.float64)), axis=1)[:, :k]
    return np.take_along_axis(s, order, 1), np.take_along_axis(i, order, 1)


# ---------------------------------------------------------------------------
# StaticIndex.call (static_index.py:37-55) and IndexRecall (index_recall.py:22-59)
def static_index(candidates: Sequence, k: int, batch: int) -> np.ndarray:
    row = np.asarray(list(candidates)[:k])
    return np.tile(row[None, :], (batch, 1))


class RecallAccumulator:
    """hits[k] += sum(equal(true, cands[:, :k])) (int32); metric = hits/seen (float64)."""

    def __init__(self, ks: Sequence[int]):
        self.ks = list(ks)
        self.hits = {k: 0 for k in self.ks}
        self.seen = 0
        self.metric: Dict[int, float] = {}

    def update(self, true_ids: Sequence, candidates: np.ndarray) -> Dict[int, float]:
        t = np.asarray(list(true_ids)).reshape(-1, 1)
        self.seen += t.shape[0]
        for k in self.ks:
            self.hits[k] += int(np.sum(t == candidates[:, :k]))
            self.metric[k] = np.float64(self.hits[k]) / np.float64(self.seen)
        return self.metric


# ---------------------------------------------------------------------------
# CPU baseline: one full train step (TwoTowerModel.train_step,
# two_tower_model.py:94-130, with legacy Adagrad) in numpy fp32.
def glorot_uniform(rng: np.random.Generator, fan_in: int, fan_out: int) -> np.ndarray:
    lim = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=(fan_in, fan_out)).astype(np.float32)


class CpuTwoTower:
    """fp32 numpy train step: gather -> towers -> scores/logQ/CE-SUM -> grads ->
    dense Adagrad (MLP) + dedup + sparse Adagrad (tables)."""

    def __init__(self, q_tables: List[np.ndarray], c_tables: List[np.ndarray], q_layers, c_layers, lr: float,
                 inbatch: str = "fp32"):
        """inbatch: "fp32" — the in-batch scores, softmax and gradients in
        fp32 (the reference's arithmetic); "bf16" — the gradients dQ, dC by
        the kernels' arithmetic contract (inbatch_softmax_xent_bf16), the
        returned loss still the fp32 one (self.last_contract_loss holds the
        contract's)."""
        if inbatch not in ("fp32", "bf16"):
            raise ValueError(f"inbatch must be 'fp32' or 'bf16', got {inbatch!r}")
        self.inbatch = inbatch
        self.last_contract_loss = None
        self.q_tables, self.c_tables = q_tables, c_tables
        self.q_layers = [[w.copy(), b.copy()] for w, b in q_layers]
        self.c_layers = [[w.copy(), b.copy()] for w, b in c_layers]
        self.lr = lr
        acc = ADAGRAD_INITIAL_ACCUMULATOR
        self.q_acc = [np.full_like(t, acc) for t in q_tables]
        self.c_acc = [np.full_like(t, acc) for t in c_tables]
        self.ql_acc = [[np.full_like(w, acc), np.full_like(b, acc)] for w, b in self.q_layers]
        self.cl_acc = [[np.full_like(w, acc), np.full_like(b, acc)] for w, b in self.c_layers]

    @staticmethod
    def _tower(x, layers):
        acts = [x]
        for w, b in layers:
            acts.append(np.maximum(acts[-1] @ w + b, 0).astype(np.float32))
        return acts

    @staticmethod
    def _tower_bwd(acts, layers, g):
        grads = []
        for li in range(len(layers) - 1, -1, -1):
            w, _ = layers[li]
            g = g * (acts[li + 1] > 0)
            grads.append((acts[li].T @ g, g.sum(0)))
            g = g @ w.T
        return grads[::-1], g

    def forward(self, q_ids: List[np.ndarray], c_ids: List[np.ndarray]):
        """Both towers' activations [x, h_1, ..., h_L] (fp32)."""
        xq = gather_concat([], self.q_tables, q_ids)
        xc = gather_concat([], self.c_tables, c_ids)
        return self._tower(xq, self.q_layers), self._tower(xc, self.c_layers)

    @staticmethod
    def _scores_loss(Q, C, logq):
        """fp32 scores - logQ, softmax terms and the CE-SUM loss
        (two_tower_model.py:92,113-122, logq_correction.py:66-71)."""
        S = Q @ C.T
        if logq is not None:
            S -= logq[None, :]
        m = S.max(1, keepdims=True)
        e = np.exp(S - m)
        z = e.sum(1, keepdims=True)
        B = S.shape[0]
        loss = float(np.sum(np.log(z[:, 0]) + m[:, 0] - S[np.arange(B), np.arange(B)]))
        return S, m, e, z, loss

    def loss_only(self, q_ids: List[np.ndarray], c_ids: List[np.ndarray], logq: Optional[np.ndarray]) -> float:
        """The fp32 loss of a batch from this restatement's own forward (no update)."""
        qa, ca = self.forward(q_ids, c_ids)
        return self._scores_loss(qa[-1], ca[-1], logq)[-1]

    def step(self, q_ids: List[np.ndarray], c_ids: List[np.ndarray], logq: Optional[np.ndarray],
             acts=None) -> float:
        """One train step.  acts: optional (query, candidate) activation lists
        to use instead of this restatement's own forward (a caller holding
        another implementation's forward — equal to this one within fp32
        rounding — checks the rest of the step against the same ReLU masks: a
        unit whose pre-activation rounds to the other side of 0 would otherwise
        switch a whole row's gradient path)."""
        if acts is None:
            qa, ca = self.forward(q_ids, c_ids)
        else:
            qa, ca = [np.asarray(a, np.float32) for a in acts[0]], [np.asarray(a, np.float32) for a in acts[1]]
        Q, C = qa[-1], ca[-1]
        S, m, e, z, loss = self._scores_loss(Q, C, logq)
        B = S.shape[0]
        if self.inbatch == "bf16":
            del S, e
            r = inbatch_softmax_xent_bf16(Q, C, logq)
            self.last_contract_loss = r["loss"]
            dQ, dC = r["dq"], r["dc"]
        else:
            P = e / z
            P[np.arange(B), np.arange(B)] -= 1.0
            dQ = P @ C
            dC = P.T @ Q
        gq, dxq = self._tower_bwd(qa, self.q_layers, dQ)
        gc, dxc = self._tower_bwd(ca, self.c_layers, dC)
        for layers, accs, grads in ((self.q_layers, self.ql_acc, gq), (self.c_layers, self.cl_acc, gc)):
            for (w, b), (aw, ab), (dw, db) in zip(layers, accs, grads):
                dense_adagrad(w, aw, dw, self.lr)
                dense_adagrad(b, ab, db, self.lr)
        # A table looked up by several features gets ONE update from the
        # concatenation of its lookups (TF aggregates the IndexedSlices of a
        # variable used twice before the sparse apply).
        for tables, accs, ids, dx in ((self.q_tables, self.q_acc, q_ids, dxq), (self.c_tables, self.c_acc, c_ids, dxc)):
            groups = {}
            off = 0
            for t, a, i in zip(tables, accs, ids):
                g = groups.setdefault(id(t), [t, a, [], []])
                g[2].append(np.asarray(i, np.int32).reshape(-1))
                g[3].append(dx[:, off:off + t.shape[1]])
                off += t.shape[1]
            for t, a, il, gl in groups.values():
                sparse_adagrad(t, a, np.concatenate(il), np.concatenate(gl), self.lr)
        return loss
