#!/usr/bin/env python3
"""Benchmark: positive pairs/s of the two-tower train step (+ index QPS).

Workload at N=1 (BASELINE.json configs[2], "C3"): the reference's main.py
schema (customer_id 128, fashion_news_frequency 2, postal_code 128 /
article_id 128, product_type_name 16+4 (declared twice, table of 4 used
twice), colour 8, department 32, index 4, section 16, garment 4) with H&M
vocabulary sizes, towers [256] -> 128, logQ-corrected in-batch softmax,
legacy Adagrad lr 0.05, batch 16384.  Synthetic ids: articles Zipf(1.1)
over a random permutation, customers Zipf(0.6), per-entity attributes fixed;
random-init weights (no dataset/checkpoint download).  A step is one full
train_step (gather, towers, fused in-batch CE fwd+bwd, MLP backward, dense
+ sparse Adagrad), replayed as a hipGraph; inputs are resident in HBM.

N>1 (torchrun, one process per GPU, RCCL), default --negatives global: the
C3 step itself (global batch 16384, the reference's loss over the WHOLE
batch, two_tower_model.py:113-122) split over the ranks — 16384/N rows per
rank, candidate embeddings + logq all-gathered, each rank's rows scored
against all 16384 candidates, query embeddings + lse all-gathered for the
dC of each rank's candidates (ShardedTrainStep
global_negatives): strong scaling, value = 16384 x steps / max-over-ranks
time.  --negatives replica: weak scaling, each rank its own batch of 16384
with per-replica negatives (a labelled variant).  The large tables
(customer, postal, article) are row-sharded over the ranks (all_to_all of
requested rows forward, of per-row gradient sums backward, Adagrad on the
owner); small tables, MLP gradients and the loss share one all_reduce
bucket (ShardedTrainStep).  value = total pairs / max-over-ranks time.  The
index line at N>1 is configs[3] candidate-sharded (ShardedBruteForceIndex,
all_to_all of per-shard top-k lists to each query block's owner + merge).

The JSON line also carries the roofline of the dominant kernel (the fused
in-batch rows pass, bf16 MFMA), the index QPS of BASELINE configs[3] at a
bounded query count on this GPU, and the CPU baseline (oracle/ numpy fp32
restatement of the same step on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

# H&M cardinalities (public dataset).
HM_VOCAB = {
    "customer_id": 1371980,
    "fashion_news_frequency": 4,
    "postal_code": 352899,
    "article_id": 105542,
    "product_type_name": 131,
    "colour_group_name": 50,
    "department_name": 250,
    "index_name": 10,
    "section_name": 56,
    "garment_group_name": 21,
}
MI355X_HBM_PEAK_GBS = 8000.0      # spec, MI355X_MICROARCH.md
MI355X_BF16_DENSE_TFLOPS = 2500.0  # spec dense (no sparsity)


def main_schema(emb_big: int = 128, joint: int = 128, hidden=(256,)):
    """The reference main.py schema (main.py:32-111) with synthetic H&M vocabs."""
    from pkg import dtypes
    from pkg.schema.features import Feature, FeatureFamily
    from pkg.schema.model_config import ModelConfig
    from pkg.schema.schema import Schema
    from pkg.schema.training_config import TrainingConfig

    Q, C = FeatureFamily.QUERY, FeatureFamily.CANDIDATE
    spec = [
        ("customer_id", Q, emb_big), ("fashion_news_frequency", Q, 2), ("postal_code", Q, emb_big),
        ("article_id", C, emb_big), ("product_type_name", C, 16), ("product_type_name", C, 4),
        ("colour_group_name", C, 8), ("department_name", C, 32), ("index_name", C, 4),
        ("section_name", C, 16), ("garment_group_name", C, 4),
    ]
    feats = []
    for name, fam, d in spec:
        f = Feature(name, dtypes.string, fam, embedding_size=d)
        f.vocab = np.arange(HM_VOCAB[name]).astype(str)  # rows 1..V, 0 = OOV
        f.is_built = True
        feats.append(f)
    tc = TrainingConfig(train_batch_size=16384, test_batch_size=2048, optimizer_name="adagrad",
                        optimizer_kwargs={"learning_rate": 0.05})
    mc = ModelConfig(joint_embedding_size=joint, ks=[10, 100, 1000], query_tower_units=list(hidden),
                     candidate_tower_units=list(hidden))
    return Schema(feats, tc, mc)


def zipf_probs(n: int, a: float) -> np.ndarray:
    p = np.arange(1, n + 1, dtype=np.float64) ** (-a)
    return p / p.sum()


class SyntheticHM:
    """Device-resident synthetic batches with H&M shapes (seeded)."""

    def __init__(self, device, seed: int = 0, stream: int = 0):
        """seed fixes the catalogue (popularity, attributes, logQ); stream picks
        the sample sequence (one per data-parallel rank)."""
        rng = np.random.default_rng(seed)
        self.device = device
        V = HM_VOCAB
        self.art_perm = rng.permutation(V["article_id"]) + 1
        self.cust_perm = rng.permutation(V["customer_id"]) + 1
        self.art_p = zipf_probs(V["article_id"], 1.1)
        self.cust_cdf = torch.as_tensor(np.cumsum(zipf_probs(V["customer_id"], 0.6)), device=device)
        self.art_cdf = torch.as_tensor(np.cumsum(self.art_p), device=device)
        self.cust_attr = {k: torch.as_tensor(rng.integers(1, V[k] + 1, V["customer_id"] + 1), device=device,
                                             dtype=torch.int32)
                          for k in ("fashion_news_frequency", "postal_code")}
        self.art_attr = {k: torch.as_tensor(rng.integers(1, V[k] + 1, V["article_id"] + 1), device=device,
                                            dtype=torch.int32)
                         for k in ("product_type_name", "colour_group_name", "department_name", "index_name",
                                   "section_name", "garment_group_name")}
        self.art_perm_t = torch.as_tensor(self.art_perm, device=device, dtype=torch.int32)
        self.cust_perm_t = torch.as_tensor(self.cust_perm, device=device, dtype=torch.int32)
        self.gen = torch.Generator(device=device)
        self.gen.manual_seed(seed + 1 + 7919 * stream)

    def prob_lookup(self):
        """candidate_prob_lookup: article row -> p (str keys, as the ETL writes)."""
        return {str(int(r) - 1): float(p) for r, p in zip(self.art_perm, self.art_p)}

    def batch(self, B: int):
        u = torch.rand(B, generator=self.gen, device=self.device, dtype=torch.float64)
        ar = torch.searchsorted(self.art_cdf, u).clamp_(max=self.art_cdf.numel() - 1)
        art = self.art_perm_t[ar]
        u = torch.rand(B, generator=self.gen, device=self.device, dtype=torch.float64)
        cr = torch.searchsorted(self.cust_cdf, u).clamp_(max=self.cust_cdf.numel() - 1)
        cust = self.cust_perm_t[cr]
        out = {"customer_id": cust, "article_id": art}
        for k, t in self.cust_attr.items():
            out[k] = t[cust.long()]
        for k, t in self.art_attr.items():
            out[k] = t[art.long()]
        return {k: v.to(torch.int32).contiguous() for k, v in out.items()}


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def max_over_ranks(x: float, device) -> float:
    """The maximum of x over the ranks (the slowest rank's time); over gloo
    (TT_BENCH_REHEARSE) through a host tensor."""
    import torch.distributed as tdist

    on = "cpu" if tdist.get_backend() == "gloo" else device
    t = torch.tensor([x], device=on, dtype=torch.float64)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return float(t.item())


def build_model(device, rank, fused_apply: bool = False):
    from pkg.modelling.models.two_tower_model import TwoTowerModel
    from pkg.modelling.optimizer_factory import OptimizerFactory

    schema = main_schema()
    data = SyntheticHM(device, seed=1234, stream=rank)
    schema.set_candidate_prob_lookup(data.prob_lookup())
    model = TwoTowerModel.create_from_schema(schema, "article_id", device=device, seed=0,
                                             fused_optimizer_apply=fused_apply)
    model.compile(optimizer=OptimizerFactory.get_optimizer("adagrad", {"learning_rate": 0.05}))
    return model, data


def time_train(args, model, data, device, ws):
    """Times args.steps train steps (after args.warmup) bracketed by barrier +
    synchronize; returns (max-over-ranks seconds, final loss).  At N>1 (or
    --train-mode sharded) the large tables of `model` move into the
    row-sharded step, so kernel-level timings must run before this."""
    from pkg.modelling.models.two_tower_model import GraphedTrainStep
    from pkg.modelling.distributed import ShardedTrainStep

    B = local_batch(args, ws)
    pool = [data.batch(B) for _ in range(4)]
    torch.cuda.synchronize()
    if ws > 1 or args.train_mode == "sharded":
        # large tables (customer, postal, article) row-sharded over the ranks
        step = ShardedTrainStep(model, shard_min_rows=100_000, global_negatives=args.negatives == "global")
        # routing (ids only) runs two batches ahead on a side stream
        run = lambda i: step(pool[i % len(pool)], ahead=[pool[(i + 1) % len(pool)], pool[(i + 2) % len(pool)]])
    else:
        step = GraphedTrainStep(model, pool[0], warmup=2)
        packed = [step.pack(b) for b in pool]  # one D2D copy per step
        run = lambda i: step(packed=packed[i % len(packed)])
    for i in range(args.warmup):
        run(i)
    if getattr(step, "host_times", None) is not None:
        step.host_times.clear()
    torch.cuda.synchronize()
    if ws > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = None
    for i in range(args.steps):
        out = run(i)
    torch.cuda.synchronize()
    if ws > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if ws > 1:
        dt = max_over_ranks(dt, device)
    loss = float(out["loss"].item())
    # after the timed region: no sparse apply recorded refused keys
    if hasattr(step, "check_status"):
        step.check_status()  # the shards' owner applies and per-request sums
    else:
        model.optimizer.check_status(device)
    if getattr(step, "host_times", None):
        print("host ms/step by phase:", {k: round(v / args.steps * 1e3, 3)
                                         for k, v in step.host_times.items()}, file=sys.stderr)  # timed steps only
    return dt, loss


def local_batch(args, ws: int) -> int:
    """Rows per rank: the global batch split over the ranks (global
    negatives), or a full batch per rank (per-replica negatives)."""
    if ws > 1 and args.negatives == "global":
        if args.batch % ws:
            raise SystemExit(f"--batch {args.batch} must split evenly over {ws} ranks")
        return args.batch // ws
    return args.batch


def time_inbatch_kernel(model, data, device, B: int, reps: int = 20):
    """Dominant kernels of the step: the two passes of the fused in-batch
    softmax CE (tt_inbatch_softmax_xent, the entry the train step calls) on
    the step's own embeddings.  Each pass kernel alone is bracketed by HIP
    events recorded on its launch stream (tt_probe_arm), per launch, over
    `reps` calls; the whole entry (prep + rows pass + combine + cols pass +
    combine) is timed beside it."""
    from pkg.modelling import hip_ops

    batch = data.batch(B)
    with torch.no_grad():
        q = model.query_tower.call({f.name: batch[f.name] for f in model.query_features})
        c = model.candidate_tower.call({f.name: batch[f.name] for f in model.candidate_features})
        logq = model.candidate_logq(batch)
    E = q.shape[1]
    for _ in range(3):
        hip_ops.inbatch_fused(q, c, logq)
    stream = torch.cuda.current_stream()
    ev = lambda: torch.cuda.Event(enable_timing=True)
    rows, cols = [], []
    e0, e1 = ev(), ev()
    e0.record(stream)
    for _ in range(reps):
        r, k = (ev(), ev()), (ev(), ev())
        hip_ops.probe_arm(hip_ops.PROBE_INBATCH_ROWS, *r)
        hip_ops.probe_arm(hip_ops.PROBE_INBATCH_COLS, *k)
        hip_ops.inbatch_fused(q, c, logq)
        rows.append(r)
        cols.append(k)
    e1.record(stream)
    e1.synchronize()
    ms_entry = e0.elapsed_time(e1) / reps
    ms_rows = sum(a.elapsed_time(b) for a, b in rows) / reps
    ms_cols = sum(a.elapsed_time(b) for a, b in cols) / reps
    # back-to-back launches of one pass between ONE event pair (tt_probe_arm_repeat):
    # no event record between launches, the launch-to-launch rate the step sees
    burst, calls = 10, 4
    rb, cb = [], []
    for _ in range(calls):
        r, k = (ev(), ev()), (ev(), ev())
        hip_ops.probe_arm_repeat(hip_ops.PROBE_INBATCH_ROWS, *r, burst)
        hip_ops.inbatch_fused(q, c, logq)
        hip_ops.probe_arm_repeat(hip_ops.PROBE_INBATCH_COLS, *k, burst)
        hip_ops.inbatch_fused(q, c, logq)
        rb.append(r)
        cb.append(k)
    torch.cuda.synchronize()
    ms_rows_b = sum(a.elapsed_time(b) for a, b in rb) / (calls * burst)
    ms_cols_b = sum(a.elapsed_time(b) for a, b in cb) / (calls * burst)
    flops = 4.0 * B * B * E  # S (2 B^2 E) + P.C (2 B^2 E) per pass
    # the opt-in fp32-faithful entry (bf16x3 scores, TT_INBATCH_X3=1): its cost
    for _ in range(3):
        hip_ops.inbatch_fused(q, c, logq, x3=True)
    e0, e1 = ev(), ev()
    e0.record(stream)
    for _ in range(reps):
        hip_ops.inbatch_fused(q, c, logq, x3=True)
    e1.record(stream)
    e1.synchronize()
    ms_x3 = e0.elapsed_time(e1) / reps
    return flops, (ms_rows_b, ms_rows), (ms_cols_b, ms_cols), ms_entry, ms_x3


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    summary (profiles/*_pmc_traffic.json: separate FETCH_SIZE / WRITE_SIZE
    passes, gfx950 FETCH_SIZE doubled); None if no summary is present."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    for name in _name_variants(kernel):
        for k, v in d.items():
            if name in k and isinstance(v, dict):
                return {"bytes_per_launch": v["hbm_bytes_per_launch"], "source": os.path.relpath(files[-1], ROOT)}
    return None


def _name_variants(kernel: str):
    """The in-batch pass's rocprof name with the round-6 X3 template flag
    (`<128, 0, false>`), then as older profiles hold it (`<128, 0>`)."""
    if kernel.startswith("inbatch_pass_kernel<") and kernel.endswith(">") and kernel.count(",") == 1:
        return [kernel[:-1] + ", false>", kernel]
    return [kernel]


def _graph_time(fn, reps: int) -> float:
    """ms per call of fn, `reps` calls replayed from one hipGraph between HIP
    events on the current stream (no host overhead between launches)."""
    from pkg.modelling import hip_ops

    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with hip_ops.capture_guard(), torch.cuda.graph(graph, stream=side):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(side)
    graph.replay()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    graph.replay()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def time_gather_uniform(model, device, B: int, reps: int = 50, c5_rows: int = 100_000_000, c5_batch: int = 65536):
    """The gather with no cache help: (1) the C3 step's both-tower launch with
    UNIFORM ids over every table (the 1.37M-row customer table alone is 702 MB,
    far beyond the 256 MB Infinity Cache); (2) BASELINE configs[4]'s 100M x 128
    fp32 table (51.2 GB) gathered at batch 65,536 with uniform ids."""
    from pkg.modelling import hip_ops

    g = torch.Generator(device=device)
    g.manual_seed(7)
    launches, nbytes = [], 0
    for tower in (model.query_tower, model.candidate_tower):
        layer = tower.input_layer
        segs = []
        for f in layer.numerical_features:
            segs.append((torch.zeros(B, device=device), None, len(segs)))
            nbytes += B * 8
        for f, off in zip(layer.categorical_features, layer.column_offsets()):
            w = layer.embedding_layers[f.name].weight
            ids = torch.randint(0, w.shape[0], (B,), generator=g, device=device, dtype=torch.int32)
            segs.append((w, ids, off))
            nbytes += B * (4 + 8 * w.shape[1])
        launches.append((segs, torch.empty(B, layer.output_dim, device=device)))
    with torch.no_grad():
        ms = _graph_time(lambda: hip_ops.gather_multi(launches, B), reps)
    gbs = nbytes / (ms * 1e-3) / 1e9
    out = {"kernel": "gather_grouped_kernel, C3 step shapes, uniform ids", "bound": "hbm", "achieved": gbs,
           "peak": MI355X_HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / MI355X_HBM_PEAK_GBS,
           "algorithmic_bytes_per_launch": nbytes, "ms_per_launch": ms,
           "copy_floor": copy_floor(device, nbytes, ms, reps)}
    if c5_rows:
        table = torch.empty(c5_rows, 128, device=device)  # 51.2 GB; contents irrelevant to the rate
        ids = torch.randint(0, c5_rows, (c5_batch,), generator=g, device=device, dtype=torch.int32)
        o = torch.empty(c5_batch, 128, device=device)
        with torch.no_grad():
            ms5 = _graph_time(lambda: hip_ops.gather_grouped([(table, ids, 0)], c5_batch, o), reps)
        nb5 = c5_batch * (4 + 8 * 128)
        out["c5_100m_table"] = {"rows": c5_rows, "dim": 128, "batch": c5_batch, "ms_per_launch": ms5,
                                "achieved": nb5 / (ms5 * 1e-3) / 1e9, "unit": "GB/s",
                                "frac": nb5 / (ms5 * 1e-3) / 1e9 / MI355X_HBM_PEAK_GBS,
                                "algorithmic_bytes_per_launch": nb5}
        del table
        torch.cuda.empty_cache()
    return out


def copy_floor(device, nbytes: int, gather_ms: float, reps: int = 50) -> dict:
    """The launch-size floor of an HBM-bound kernel moving `nbytes`: a plain
    device copy of nbytes / 2 read + nbytes / 2 written (torch's vectorised
    copy kernel; no index loads, fully coalesced, HBM-resident source of
    nbytes / 2 > L2), timed like the gather (one hipGraph of `reps` launches).
    What the gather's launch of the same bytes can at best approach:
    frac_of_copy = copy ms / gather ms."""
    n = nbytes // 8
    src = torch.rand(n, device=device)
    dst = torch.empty_like(src)
    # twelve rotating sources (30 MB each, 365 MB with dst > the 256 MB Infinity Cache): HBM reads
    srcs = [src] + [torch.rand(n, device=device) for _ in range(11)]
    it = iter(range(1 << 30))
    ms = _graph_time(lambda: dst.copy_(srcs[next(it) % 12]), reps)
    return {"kernel": "torch device copy (the same bytes, half read, half written)", "ms_per_launch": ms,
            "achieved": nbytes / (ms * 1e-3) / 1e9, "unit": "GB/s", "frac_of_copy": ms / gather_ms}


def rocprof_avg_ms(kernel: str):
    """Average duration (ms) of `kernel` in the newest committed rocprofv3
    --stats summary (profiles/*_bench_kernel_stats.csv), or None."""
    import csv
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_bench_kernel_stats.csv")))
    if not files:
        return None
    with open(files[-1]) as f:
        rows = list(csv.DictReader(f))
    for name in _name_variants(kernel):
        for r in rows:
            if name in r["Name"]:
                return {"ms": float(r["AverageNs"]) * 1e-6, "calls": int(r["Calls"]),
                        "source": os.path.relpath(files[-1], ROOT)}
    return None


def time_gather(model, data, device, B: int, reps: int = 50):
    """K2+K3 gather of both towers' inputs for one step's batch in one
    tt_gather_multi launch (as the train step issues it), HIP events on the
    launching stream.  Algorithmic bytes per launch:
    per categorical lookup 4 B id + D_f*4 B row read + D_f*4 B output write;
    per numeric column 4 B read + 4 B write."""
    from pkg.modelling import hip_ops

    batch = data.batch(B)
    launches = []
    nbytes = 0
    for tower in (model.query_tower, model.candidate_tower):
        layer = tower.input_layer
        segs = []
        for f in layer.numerical_features:
            v = batch[f.name].reshape(-1).to(torch.float32).contiguous()
            segs.append((v, None, len(segs)))
            nbytes += B * 8
        for f, off in zip(layer.categorical_features, layer.column_offsets()):
            w = layer.embedding_layers[f.name].weight
            segs.append((w, batch[f.name].reshape(-1).to(torch.int32).contiguous(), off))
            nbytes += B * (4 + 8 * w.shape[1])
        out = torch.empty(B, layer.output_dim, device=device)
        launches.append((segs, out))
    with torch.no_grad():
        for _ in range(3):
            hip_ops.gather_multi(launches, B)
        torch.cuda.synchronize()
        # reps launches captured in a hipGraph: the replay has no host overhead
        # between launches, so the events see the kernel, not the Python call.
        graph = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            with hip_ops.capture_guard(), torch.cuda.graph(graph, stream=side):
                for _ in range(reps):
                    hip_ops.gather_multi(launches, B)
        torch.cuda.current_stream().wait_stream(side)
        graph.replay()
        torch.cuda.synchronize()
        stream = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        graph.replay()
        e1.record(stream)
        e1.synchronize()
    ms = e0.elapsed_time(e1) / reps  # one launch: both towers
    gbs = nbytes / (ms * 1e-3) / 1e9
    return {"kernel": "gather_grouped_kernel (tt_gather_multi: query + candidate tower inputs, one launch)",
            "bound": "hbm",
            "achieved": gbs, "peak": MI355X_HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / MI355X_HBM_PEAK_GBS,
            "algorithmic_bytes_per_launch": nbytes, "ms_per_launch": ms,
            "traffic": (pmc_traffic("gather_grouped_kernel") or {}).get("bytes_per_launch"),
            "traffic_source": (pmc_traffic("gather_grouped_kernel") or {}).get("source"),
            "note": "Zipf ids: popular rows hit L2/Infinity Cache, so the algorithmic rate can exceed HBM"}


def time_index(device, n_queries: int, n_cand: int, k: int, E: int = 128, check: int = 512):
    """BASELINE configs[3] shape: relu(N(0,1)) candidates [105542,128], queries
    relu(N(0,1)) with 1% all-zero rows, top-100, one GPU (bounded query count)."""
    from pkg.modelling import hip_ops

    g = torch.Generator(device=device)
    g.manual_seed(1)
    C = torch.relu(torch.randn(n_cand, E, generator=g, device=device))
    g.manual_seed(2)
    Q = torch.relu(torch.randn(n_queries, E, generator=g, device=device))
    Q[::100] = 0.0
    image = hip_ops.bruteforce_build(C)
    hip_ops.bruteforce_search(image, C, Q, k)  # warm: code + the full-size workspace, outside the timed region
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s, i = hip_ops.bruteforce_search(image, C, Q, k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tf = 2.0 * n_queries * n_cand * E / dt / 1e12
    res = {"queries": n_queries, "candidates": n_cand, "k": k, "dim": E, "seconds": dt,
           "qps": n_queries / dt, "tflops_scoring": tf,
           "roofline": {"bound": "mfma", "achieved": tf, "peak": MI355X_BF16_DENSE_TFLOPS, "unit": "TFLOP/s",
                        "frac": tf / MI355X_BF16_DENSE_TFLOPS,
                        "note": "2*Q*N*E scoring flops over the whole search (screen + exact finalize)"}}
    if check:
        try:
            from oracle import oracle

            sel = np.linspace(0, n_queries - 1, check).astype(np.int64)
            qs, cs = Q[sel].cpu().numpy(), C.cpu().numpy()
            t0 = time.perf_counter()
            _, ri, used = oracle.bruteforce_topk(qs, cs, k)
            t_cpu = time.perf_counter() - t0
            gi = i[sel].cpu().numpy()
            res["exact_match_rows"] = int((gi == ri).all(axis=1).sum())
            res["checked_rows"] = int(check)
            res["recall_at_100_vs_exact"] = float(np.mean([len(set(a) & set(b)) / k for a, b in zip(gi, ri)]))
            # the same exact search on the host: the C restatement (fp32 fmaf chain + top-k)
            res["cpu_baseline"] = {"value": check / t_cpu, "unit": "queries/s", "cores": int(used), "kind": "port",
                                   "sample": f"{check} of the queries x {n_cand} candidates, top-{k}, "
                                             f"oracle/tt_oracle.c (fp32 fmaf chain), {t_cpu:.1f}s"}
        except Exception as e:  # the check is informative only
            res["check_error"] = repr(e)
    res["runner_point"] = time_index_runner_point(image, C, Q)
    return res


def time_index_runner_point(image, C: torch.Tensor, Q: torch.Tensor, batch: int = 2048, k: int = 1000,
                            batches: int = 32, check: int = 256):
    """The reference runner's own index operating point: IndexRecall over the
    test set in batches of test_batch_size = 2048 (/root/reference/main.py:99)
    at k = max(ks) = 1000 (main.py:107; brute_force.py:54-83 per batch).
    `batches` consecutive search calls of 2048 queries each, back to back on
    the stream (one call per test batch, as the runner issues them)."""
    from pkg.modelling import hip_ops

    nq = min(batch * batches, Q.shape[0])
    chunks = [Q[b:b + batch] for b in range(0, nq, batch)]
    hip_ops.bruteforce_search(image, C, chunks[0], k)  # warm: code + workspace
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = [hip_ops.bruteforce_search(image, C, q, k) for q in chunks]
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res = {"queries": nq, "batch": batch, "k": k, "calls": len(chunks), "seconds": dt, "qps": nq / dt,
           "ms_per_batch": dt / len(chunks) * 1e3,
           "tflops_scoring": 2.0 * nq * C.shape[0] * C.shape[1] / dt / 1e12}
    if check:
        try:
            from oracle import oracle

            # `check` rows spread over every batch of the run, each vs the C restatement
            sel = np.linspace(0, nq - 1, check).astype(np.int64)
            qs = Q[:nq][sel].cpu().numpy()
            rs, ri, _ = oracle.bruteforce_topk(qs, C.cpu().numpy(), k)
            gi = np.stack([outs[j // batch][1][j % batch].cpu().numpy() for j in sel])
            gs = np.stack([outs[j // batch][0][j % batch].cpu().numpy() for j in sel])
            res["exact_match_rows"] = int(((gi == ri) & (gs == rs)).all(axis=1).sum())
            res["checked_rows"] = int(check)
        except Exception as e:  # informative only
            res["check_error"] = repr(e)
    return res


def time_runner_recall(model, data, device, batch: int = 2048, batches: int = 32, ks=(10, 100, 1000)):
    """The reference runner's evaluation end to end on the trained model:
    IndexRecall (index_recall.py:52-58) over `batches` test batches of
    test_batch_size = 2048 (main.py:99) with ks = [10, 100, 1000] (main.py:107):
    per batch the query tower on the batch's query features (gather + MLP),
    BruteForceIndex.call at k = max(ks) over every article's candidate-tower
    embedding (brute_force.py:54-83: search + identifier lookup) and the
    on-device recall counts (tt_recall_hits).  Timed from the first call to
    the last batch's counts."""
    from pkg.modelling.indices.brute_force import BruteForceIndex
    from pkg.modelling.metrics.index_recall import IndexRecall

    V = HM_VOCAB["article_id"]
    ids = torch.arange(1, V + 1, device=device, dtype=torch.int32)
    feats = {"article_id": ids, **{n: t[ids.long()].contiguous() for n, t in data.art_attr.items()}}
    cemb = model.candidate_tower(feats)
    index = BruteForceIndex(max(ks), model.query_tower, [(ids, cemb)], device=device)
    qnames = [f.name for f in model.query_features]
    tests = [data.batch(batch) for _ in range(batches + 1)]
    qx = [{n: b[n] for n in qnames} for b in tests]
    IndexRecall(index, list(ks))(qx[0], tests[0]["article_id"])  # warm: code + workspaces
    rec = IndexRecall(index, list(ks))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for x, b in zip(qx[1:], tests[1:]):
        rec(x, b["article_id"])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    hits = rec.hits  # read after the timed region
    return {"queries": batch * batches, "batch": batch, "k": max(ks), "ks": list(ks), "calls": batches,
            "seconds": dt, "qps": batch * batches / dt, "ms_per_batch": dt / batches * 1e3,
            "recall": {str(k): float(hits[k]) / (batch * batches) for k in ks},
            "note": "IndexRecall per test batch: query tower (tt_gather_multi + tt_mlp_rows) -> "
                    "tt_bruteforce_search over 105,542 candidate-tower embeddings -> identifier lookup -> "
                    "tt_recall_hits; the trained C3 model of the train leg, synthetic H&M catalogue"}


def time_index_sharded(device, n_queries: int, n_cand: int, k: int, ws: int, rank: int, E: int = 128,
                       check: int = 256):
    """configs[3] candidate-sharded over the ranks (ShardedBruteForceIndex):
    rank r holds only candidate rows shard_range(N, G, r) and computes their
    exact top-k for every query (tt_bruteforce_search, global indices); one
    all_to_all hands each query block's per-shard lists to its owner, which
    merges them (tt_topk_merge).  Strong scaling: Q and N fixed.  QPS =
    Q / max-over-ranks wall time of search_owned, barrier + sync both sides.
    Beside it, `query_sharded`: the same queries split over the ranks against
    replicated candidates (QueryShardedBruteForceIndex, no exchange)."""
    from pkg.modelling.distributed import ShardedBruteForceIndex, shard_range

    g = torch.Generator(device=device)
    g.manual_seed(1)
    C = torch.relu(torch.randn(n_cand, E, generator=g, device=device))
    g.manual_seed(2)
    Q = torch.relu(torch.randn(n_queries, E, generator=g, device=device))
    Q[::100] = 0.0
    idx = ShardedBruteForceIndex.from_full(k, None, C)  # a copy of this rank's rows only
    idx.search_owned(Q)  # warm: code + full-size workspaces, outside the timed region
    torch.cuda.synchronize()
    torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    (qb, qe), s, i = idx.search_owned(Q)
    torch.cuda.synchronize()
    torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dt = max_over_ranks(dt, device)
    tf = 2.0 * n_queries * n_cand * E / dt / 1e12
    res = {"queries": n_queries, "candidates": n_cand, "k": k, "dim": E, "shards": ws, "seconds": dt,
           "qps": n_queries / dt, "scaling": "strong (candidates row-sharded over the ranks, all queries)",
           "roofline": {"bound": "mfma", "achieved": tf, "peak": MI355X_BF16_DENSE_TFLOPS * ws, "unit": "TFLOP/s",
                        "frac": tf / (MI355X_BF16_DENSE_TFLOPS * ws),
                        "note": "2*Q*N*E scoring flops / wall time incl. all_to_all + merge, vs G x dense bf16 peak"}}
    # the same queries query-sharded over replicated candidates (no exchange)
    from pkg.modelling.distributed import QueryShardedBruteForceIndex

    qidx = QueryShardedBruteForceIndex(k, None, C)
    qidx.search_owned(Q)  # warm
    torch.cuda.synchronize()
    torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    qidx.search_owned(Q)
    torch.cuda.synchronize()
    torch.distributed.barrier()
    torch.cuda.synchronize()
    dq = time.perf_counter() - t0
    dq = max_over_ranks(dq, device)
    res["query_sharded"] = {"seconds": dq, "qps": n_queries / dq,
                            "scaling": "strong (queries split over the ranks, candidates replicated)",
                            "roofline_frac": 2.0 * n_queries * n_cand * E / dq / 1e12 / (MI355X_BF16_DENSE_TFLOPS * ws)}
    if rank == 0 and check:
        try:
            from oracle import oracle

            sel = np.linspace(qb, qe - 1, check).astype(np.int64)
            _, ri, _ = oracle.bruteforce_topk(Q[sel].cpu().numpy(), C.cpu().numpy(), k)
            gi = i[sel - qb].cpu().numpy()
            res["exact_match_rows"] = int((gi == ri).all(axis=1).sum())
            res["checked_rows"] = int(check)
        except Exception as ex:  # informative only
            res["check_error"] = repr(ex)
    return res


def time_c5_sharded(device, ws: int, rank: int, steps: int = 20, rows: int = 100_000_000,
                    global_batch: int = 65536, D: int = 128):
    """BASELINE configs[4]: a 100M x 128 fp32 table row-sharded over the ranks
    (ShardedTables; global row r on rank r % G, each rank holding only its
    rows and their Adagrad accumulator) and a GLOBAL batch of 65,536 uniform
    ids split over the ranks (65,536 / G per rank: the configuration as
    stated).  A step, replayed as one hipGraph (fixed-capacity routing: no
    host sync): routing (tt_route_fixed: dedup + owner buckets + fixed
    per-owner slots; all_to_all of the requests), fetch (tt_gather_tagged on
    the owners + all_to_all of the rows), apply (per-request sums on the
    route's own sort, tt_sparse_routed + all_to_all of the sums +
    tt_sparse_adagrad on the owners).  At one rank there is nothing to
    exchange or route: the one owner reads the rows by id and applies the
    update keyed by the ids (ShardedTables.fetch_local / apply_local: one
    gather, the single-device dedup + Adagrad).  Algorithmic HBM bytes per rank and
    step: lookups x (4 B id + 2 x 4D row read/write + 4D gradient read) +
    owner rows x 16D (param and accumulator read + write).  The all_to_all
    share is the three data all_to_alls of the same sizes timed alone.  At
    G > 1 `weak_per_rank` adds the weak-scaled variant (65,536 ids per rank)
    as a labelled extra."""
    import torch.distributed as tdist

    from pkg.modelling import hip_ops
    from pkg.modelling.distributed import ShardedTables, _a2a

    own = not tdist.is_initialized()
    if own:  # N = 1: a one-rank RCCL group
        import socket

        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        tdist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                 device_id=device)
    try:
        g = torch.Generator(device=device)
        g.manual_seed(17 + rank)
        n_local = len(range(rank, rows, ws))
        shard = torch.empty(n_local, D, device=device)
        for s0 in range(0, n_local, 1 << 24):
            shard[s0:s0 + (1 << 24)].uniform_(-0.05, 0.05, generator=g)
        st = ShardedTables({"big": shard, "__rows__": {"big": rows}}, full_tables=False)
        del shard
        graphed = tdist.get_backend() == "nccl"

        def leg(b: int) -> dict:
            ids = [torch.randint(0, rows, (b,), generator=g, device=device, dtype=torch.int32) for _ in range(2)]
            grad = torch.randn(b, D, generator=g, device=device)
            sid = ids[0].clone()  # the static batch the graph reads
            cap = st.route_capacity(1, b)
            g_req = torch.zeros(ws * cap, D, device=device)

            rows_out = torch.empty(b, D, device=device)
            side = torch.cuda.Stream(device=device)
            # world 1 ("local", default): the one owner fetches and applies by
            # id (ShardedTables.fetch_local / apply_local: 0.111 vs 0.125 ms for
            # the routed form on one stream, "serial"; 0.141 with the route
            # forked beside the fetch, "fork", 0.152 with the fetch captured
            # first, "first" — profiles/r05_c5_ab.txt)
            c5_order = os.environ.get("TT_C5_ORDER", "local")

            def body():
                if ws == 1:
                    # one rank: the shard IS the owner's answer — the fetch is a
                    # read by id (tt_gather_grouped); the route then only feeds
                    # the apply
                    # (C5_ORDER "fork": the route on a side stream beside the
                    # fetch; "first": the same with the fetch captured first)
                    main = torch.cuda.current_stream()
                    if c5_order == "local":  # the one owner: fetch and apply by id, no route
                        st.fetch_local([("big", sid)], rows_out.view(1, b, D))
                        st.apply_local([("big", sid)], [(grad, 0)], 0.05, 1e-7)
                        return
                    if c5_order == "serial":
                        rt = st.route_fixed([("big", sid)], cap)
                        hip_ops.gather_grouped([(st.shard["big"], sid, 0)], b, rows_out)
                    else:
                        fork = torch.cuda.Event()
                        fork.record(main)
                        if c5_order == "first":
                            hip_ops.gather_grouped([(st.shard["big"], sid, 0)], b, rows_out)
                        side.wait_event(fork)
                        with torch.cuda.stream(side):
                            rt = st.route_fixed([("big", sid)], cap)
                        if c5_order != "first":
                            hip_ops.gather_grouped([(st.shard["big"], sid, 0)], b, rows_out)
                        main.wait_stream(side)
                        for t in (rt.tags, rt.rows, rt.counts, rt.idx_all, *rt.table_ids, *(rt.order or ())):
                            t.record_stream(main)
                else:
                    rt = st.route_fixed([("big", sid)], cap)
                    st.fetch_routed(rt)
                st.apply_lookups(rt, [(grad, 0)], 0.05, 1e-7, g_req=g_req if ws > 1 else None)

            body()  # eager: code, workspaces
            graph = None
            if graphed:
                graph = torch.cuda.CUDAGraph()
                with hip_ops.capture_guard(), torch.cuda.graph(graph, capture_error_mode="thread_local"):
                    body()

            def step(i):
                sid.copy_(ids[i % 2])
                graph.replay() if graph is not None else body()

            def timed(fn, n):
                for i in range(2):
                    fn(i)
                torch.cuda.synchronize()
                tdist.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(n):
                    fn(i)
                torch.cuda.synchronize()
                tdist.barrier()
                torch.cuda.synchronize()
                return max_over_ranks(time.perf_counter() - t0, device) / n

            sec = timed(step, steps)
            if graph is not None:
                graph.reset()
            rt = st.route([("big", ids[0])])  # compact route: the real request / owner-row counts
            rt_sizes = (rt.R, rt.n_recv)
            slots = ws * cap
            req = torch.zeros(slots, 2, dtype=torch.int32, device=device)
            req_in = torch.empty(slots, 2, dtype=torch.int32, device=device)
            rows_out = torch.empty(slots, D, device=device)
            rows_in = torch.empty(slots, D, device=device)
            grads_in = torch.empty(slots, D, device=device)
            split = [cap] * ws

            def a2a(_):
                _a2a(req_in, req, split, split, st.group)
                _a2a(rows_in, rows_out, split, split, st.group)
                _a2a(grads_in, rows_in, split, split, st.group)

            a2a_sec = timed(a2a, steps)
            nbytes = b * (4 + 12 * D) + rt_sizes[1] * 16 * D
            gbs = ws * nbytes / sec / 1e9
            return {"batch_per_rank": b, "requests_per_rank": rt_sizes[0], "owner_rows_per_rank": rt_sizes[1],
                    "slots_per_owner": cap, "ms_per_step": sec * 1e3, "lookups_per_s": ws * b / sec,
                    "roofline": {"bound": "hbm", "achieved": gbs, "peak": MI355X_HBM_PEAK_GBS * ws, "unit": "GB/s",
                                 "frac": gbs / (MI355X_HBM_PEAK_GBS * ws), "algorithmic_bytes_per_rank_step": nbytes},
                    "all_to_all_ms": a2a_sec * 1e3, "all_to_all_share": a2a_sec / sec}

        res = {"rows": rows, "dim": D, "ranks": ws, "rows_per_rank": n_local, "global_batch": global_batch,
               "scaling": "strong (the global batch of 65,536 ids split over the ranks)",
               "graphed": graphed, **leg(global_batch // ws),
               "note": "route + fetch + apply per step as one hipGraph replay (fixed-capacity routing, no host "
                       "sync; at one rank fetch + apply by id, nothing to route); uniform ids over the whole table"}
        if ws > 1:
            res["weak_per_rank"] = {"scaling": "weak (65,536 ids per rank; labelled extra)", **leg(global_batch)}
        del st
        torch.cuda.empty_cache()
        return res
    finally:
        if own:
            from pkg.modelling.distributed import destroy_process_group

            destroy_process_group()


def time_pipeline(model, data, device, rows: int, B: int, encode_n: int = 2_000_000):
    """modelling_runner's training input path at scale: `rows` synthetic
    H&M-shaped examples encoded into an HBM-resident DeviceDataset, one epoch
    of TwoTowerModel.fit (one hipGraph replay per batch: device batch take +
    train step; the partial last batch eager), timed after a first epoch
    that captures the graph.  Plus the host StringLookup rate of libtt's
    native vocabulary on 64-hex-char customer ids (H&M's id format)."""
    from pkg.modelling.dataset import DeviceDataset
    from pkg.schema.vocab import NativeVocab

    cols = {}
    for s in range(0, rows, 1 << 20):
        b = data.batch(min(1 << 20, rows - s))
        for k, v in b.items():
            cols.setdefault(k, []).append(v.cpu().numpy())
    cols = {k: np.concatenate(v) for k, v in cols.items()}
    ds = DeviceDataset(cols, B, shuffle_size=100_000, seed=0, device=device)
    model.fit(ds, epochs=1, use_graph=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    model.fit(ds, epochs=1, use_graph=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    del ds
    rng = np.random.default_rng(0)
    vocab = np.array([f"{x:016x}{x ^ 0x5bd1e995:016x}" * 2
                      for x in rng.integers(0, 2**62, HM_VOCAB["customer_id"]).tolist()])
    nv = NativeVocab(vocab)
    import pyarrow as pa

    vals = pa.array(vocab[rng.integers(0, len(vocab), encode_n)])
    nv.encode(vals[:1000])
    t = time.perf_counter()
    nv.encode(vals)
    enc_dt = time.perf_counter() - t
    return {"rows": rows, "batch": B, "shuffle_size": 100_000, "epoch_seconds": dt, "rows_per_s": rows / dt,
            "note": "fit over an HBM-resident DeviceDataset: tt_batch_take + train step replayed as one hipGraph "
                    "per batch, partial last batch eager, one host sync per epoch",
            "encode": {"values": encode_n, "vocab": len(vocab), "seconds": enc_dt, "values_per_s": encode_n / enc_dt,
                       "threads": os.cpu_count() if os.cpu_count() and os.cpu_count() < 64 else 64,
                       "note": "libtt tt_vocab_encode (host hash StringLookup) of 64-char hex ids, Arrow input"}}


def cpu_baseline(seconds_budget: float = 20.0):
    """oracle.CpuTwoTower (numpy fp32 restatement of the same train step) on
    host cores, same schema and batch, timed over whole steps until ~budget."""
    from oracle import oracle

    try:
        from threadpoolctl import threadpool_info

        threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        threads = 1
    schema = main_schema()
    rng = np.random.default_rng(0)
    V = HM_VOCAB

    def tables(feats):
        seen, out = {}, []
        for f in feats:
            if f.name not in seen:
                seen[f.name] = rng.uniform(-0.05, 0.05, (V[f.name] + 1, f.embedding_size)).astype(np.float32)
        # duplicated name: the last declaration's table, looked up per declaration
        last = {f.name: f for f in feats}
        for f in feats:
            if seen[f.name].shape[1] != last[f.name].embedding_size:
                seen[f.name] = rng.uniform(-0.05, 0.05, (V[f.name] + 1, last[f.name].embedding_size)).astype(
                    np.float32)
            out.append(seen[f.name])
        return out

    qt, ct = tables(schema.query_features), tables(schema.candidate_features)

    def layers(din):
        return [(oracle.glorot_uniform(rng, din, 256), np.zeros(256, np.float32)),
                (oracle.glorot_uniform(rng, 256, 128), np.zeros(128, np.float32))]

    wq = sum(t.shape[1] for t in qt)
    wc = sum(t.shape[1] for t in ct)
    # identical tables for repeated names -> share objects
    m = oracle.CpuTwoTower(qt, ct, layers(wq), layers(wc), 0.05)
    B = 16384
    p = zipf_probs(V["article_id"], 1.1)
    logq_rows = np.log(p).astype(np.float32)

    def batch():
        art = rng.choice(V["article_id"], size=B, p=p).astype(np.int32)
        cust = (rng.zipf(1.6, size=B) % V["customer_id"]).astype(np.int32)
        q_ids = [cust + 1, rng.integers(1, 5, B).astype(np.int32), rng.integers(1, V["postal_code"], B).astype(np.int32)]
        c_ids = [art + 1] + [rng.integers(1, V[f.name] + 1, B).astype(np.int32) for f in schema.candidate_features[1:]]
        return q_ids, c_ids, logq_rows[art]

    steps, t_total = 0, 0.0
    while t_total < seconds_budget and steps < 50:
        q_ids, c_ids, lq = batch()
        t0 = time.perf_counter()
        m.step(q_ids, c_ids, lq)
        t_total += time.perf_counter() - t0
        steps += 1
    return {"value": steps * B / t_total, "unit": "positive pairs/s", "cores": int(threads), "kind": "port",
            "sample": f"{steps} full C3 train steps (B=16384, main.py schema, H&M vocab) of the numpy fp32 "
                      f"restatement oracle/oracle.py:CpuTwoTower, {t_total:.1f}s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--index-queries", type=int, default=1_000_000)
    ap.add_argument("--no-index", action="store_true")
    ap.add_argument("--fused-apply", action="store_true",
                    help="apply each tower's Adagrad inside the backward (TwoTowerModel fused_optimizer_apply)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-uniform-gather", action="store_true",
                    help="skip the uniform-id gather legs (C3 shapes and the 100M-row C5 table)")
    ap.add_argument("--pipeline-rows", type=int, default=10_000_000,
                    help="rows of the device-resident input-pipeline leg (0 skips it; N=1 only)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-c5", action="store_true", help="skip the row-sharded 100M-row table leg (configs[4])")
    ap.add_argument("--c5-only", action="store_true", help="run only the configs[4] leg (profiling)")
    ap.add_argument("--train-mode", choices=("auto", "sharded"), default="auto",
                    help="sharded: run the N>1 row-sharded step (ShardedTrainStep) even on one rank")
    ap.add_argument("--negatives", choices=("global", "replica"), default="global",
                    help="N>1: global = the C3 batch split over the ranks with negatives from the whole batch "
                         "(strong scaling); replica = a batch per rank with per-replica negatives (weak scaling)")
    ap.add_argument("--index-mode", choices=("auto", "sharded"), default="auto",
                    help="sharded: run the N>1 candidate-sharded index (search_owned) even on one rank")
    args = ap.parse_args()

    # stdout carries exactly one JSON line: everything else written to fd 1
    # (RCCL's version banner, library chatter) goes to stderr
    sys.stdout.flush()
    real_stdout = os.dup(1)
    os.dup2(2, 1)

    ws, rank, local = dist_env()
    # TT_BENCH_REHEARSE=1: a dry run of the N > 1 path on a box with fewer
    # GPUs than ranks (ranks share the GPUs, collectives over gloo through the
    # host); its line says so and is not a measurement
    rehearse = os.environ.get("TT_BENCH_REHEARSE") == "1"
    if ws > 1 or args.train_mode == "sharded" or args.index_mode == "sharded":
        dev_index = local % torch.cuda.device_count() if rehearse else local
        torch.cuda.set_device(dev_index)
        if ws == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if rehearse:
            torch.distributed.init_process_group("gloo")
        else:
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", torch.cuda.current_device())
    if args.c5_only:
        res = time_c5_sharded(device, ws, rank, steps=args.steps)
        if rank == 0:
            os.write(real_stdout, (json.dumps({"c5_sharded_table": res}) + "\n").encode())
        if torch.distributed.is_initialized():
            from pkg.modelling.distributed import destroy_process_group

            destroy_process_group()
        return

    model, data = build_model(device, rank, args.fused_apply)
    B = args.batch
    # kernel-level timings on the unsharded model, before the train step takes its tables
    flops, ms_rows, ms_cols, ms_entry, ms_x3 = time_inbatch_kernel(model, data, device, B)
    gather = time_gather(model, data, device, B)
    if ws == 1 and not args.no_uniform_gather:
        gather["uniform_ids"] = time_gather_uniform(model, device, B)
    dt, loss = time_train(args, model, data, device, ws)
    global_neg = ws > 1 and args.negatives == "global"
    pairs = (B if global_neg else ws * B) * args.steps
    value = pairs / dt
    ms_per_step = dt / args.steps * 1e3

    (ms_rows, ms_rows_1), (ms_cols, ms_cols_1) = ms_rows, ms_cols
    achieved = flops / (ms_rows * 1e-3) / 1e12
    result = {
        "metric": "positive pairs/sec (train) + index QPS @ Recall@100, 1/2/4/8 MI355X",
        "value": value,
        "unit": "positive pairs/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        # the default (--negatives global) fixes the global batch at every N
        "scaling": "weak" if args.negatives == "replica" else "strong",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (H&M-shaped ids, Zipf; random-init weights)",
        "config": {
            "workload": "C3: main.py schema @ emb 128, towers [256]->128, logQ in-batch softmax, Adagrad, batch 16384"
                        + ((f" split over {ws} ranks ({B // ws} rows each), in-batch negatives from the whole batch "
                            "(all_gather of C, logq, Q, lse)" if global_neg else
                            " per replica, per-replica in-batch negatives (labelled variant)")
                           + "; customer/postal/article tables row-sharded over the ranks (all_to_all), small tables "
                             "and MLP replicated (all_reduce)" if ws > 1 else ""),
            "global_batch": B if global_neg else ws * B,
            "parallelism": f"dp{ws}",
        },
        "final_loss": loss,
        "roofline": {
            "kernel": "inbatch_pass_kernel<128,0> (rows pass of tt_inbatch_softmax_xent: S=QC^T-logq, online "
                      "softmax, P.C), HIP events on its launch stream around 10 back-to-back launches "
                      "(tt_probe_arm_repeat), 4 samples",
            "bound": "mfma",
            "achieved": achieved,
            "peak": MI355X_BF16_DENSE_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved / MI355X_BF16_DENSE_TFLOPS,
            "traffic": (pmc_traffic("inbatch_pass_kernel<128, 0>") or {}).get("bytes_per_launch"),
            "traffic_source": (pmc_traffic("inbatch_pass_kernel<128, 0>") or {}).get("source"),
            "ms_per_launch": ms_rows,
            "ms_per_launch_one_event_pair_each": ms_rows_1,
            "cols_pass": {"kernel": "inbatch_pass_kernel<128,1>", "ms_per_launch": ms_cols,
                          "ms_per_launch_one_event_pair_each": ms_cols_1,
                          "achieved": flops / (ms_cols * 1e-3) / 1e12},
            "ms_fused_entry": ms_entry,
            "ms_fused_entry_x3": ms_x3,
            "algorithmic_flops_per_launch": flops,
        },
        "gather_roofline": gather,
    }
    if rehearse:
        result["rehearsal"] = "TT_BENCH_REHEARSE: ranks share GPUs over gloo; not a measurement"

    rp = rocprof_avg_ms("inbatch_pass_kernel<128, 0>")
    if rp is not None:
        # the profiler's dispatch timestamps (no event overhead around each launch)
        a_rp = flops / (rp["ms"] * 1e-3) / 1e12
        result["roofline"]["rocprof"] = {"ms_per_launch": rp["ms"], "calls": rp["calls"], "achieved": a_rp,
                                         "frac": a_rp / MI355X_BF16_DENSE_TFLOPS, "source": rp["source"]}
    if ws == 1 and args.index_mode == "auto" and not args.no_index:
        result["index"] = time_index(device, args.index_queries, HM_VOCAB["article_id"], 100)
        result["index"]["runner_recall_e2e"] = time_runner_recall(model, data, device)
    elif not args.no_index:
        result["index"] = time_index_sharded(device, args.index_queries, HM_VOCAB["article_id"], 100, ws, rank)
    if not args.no_c5:
        result["c5_sharded_table"] = time_c5_sharded(device, ws, rank)
    if ws == 1 and args.pipeline_rows > 0:
        result["pipeline"] = time_pipeline(model, data, device, args.pipeline_rows, B)
        result["pipeline"]["vs_train_step_rate"] = result["pipeline"]["rows_per_s"] / value
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    if rank == 0:
        sys.stdout.flush()
        os.write(real_stdout, (json.dumps(result) + "\n").encode())
    if torch.distributed.is_initialized():
        from pkg.modelling.distributed import destroy_process_group

        destroy_process_group()  # captured step graphs (RCCL collectives) released first


if __name__ == "__main__":
    main()
