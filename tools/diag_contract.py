"""Where does a train step's in-batch gradient differ from the arithmetic-
contract restatement (oracle.inbatch_softmax_xent_bf16)?  Per step of the
C2 / C3 train-step test: the GPU pass on the GPU's own tower outputs vs the
contract on those same outputs (kernel vs restatement), and vs the contract on
the oracle's fp32 tower outputs (sensitivity to the towers' rounding).

usage: python tools/diag_contract.py [B] [emb]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from oracle import oracle  # noqa: E402
from pkg.modelling import hip_ops  # noqa: E402
from pkg.modelling.models.two_tower_model import TwoTowerModel  # noqa: E402
from pkg.modelling.optimizer_factory import OptimizerFactory  # noqa: E402
from test_configs_gpu import _mirror  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
emb = int(sys.argv[2]) if len(sys.argv) > 2 else 64
cuda = torch.device("cuda:0")
schema = bench.main_schema(emb_big=emb, joint=emb, hidden=(256,))
data = bench.SyntheticHM(cuda, seed=7)
schema.set_candidate_prob_lookup(data.prob_lookup())
m = TwoTowerModel.create_from_schema(schema, "article_id", device=cuda, seed=0)
m.compile(optimizer=OptimizerFactory.get_optimizer("adagrad", {"learning_rate": 0.05}))
qf = m.query_tower.input_layer.categorical_features
cf = m.candidate_tower.input_layer.categorical_features
rel = lambda a, b: float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
for step in range(3):
    ref = _mirror(m, "bf16")
    b = data.batch(B)
    lq = m.candidate_logq(b).cpu().numpy()
    with torch.no_grad():
        q = m.query_tower.call({f.name: b[f.name] for f in m.query_features})
        c = m.candidate_tower.call({f.name: b[f.name] for f in m.candidate_features})
    lse, rl, dq, dc = hip_ops.inbatch_fused(q.contiguous(), c.contiguous(), torch.as_tensor(lq, device=cuda))
    qn, cn = q.cpu().numpy(), c.cpu().numpy()
    dq, dc, rl = dq.cpu().numpy(), dc.cpu().numpy(), rl.cpu().numpy()
    con = oracle.inbatch_softmax_xent_bf16(qn, cn, lq)
    xq = oracle.gather_concat([], ref.q_tables, [b[f.name].cpu().numpy() for f in qf])
    xc = oracle.gather_concat([], ref.c_tables, [b[f.name].cpu().numpy() for f in cf])
    Qo, Co = ref._tower(xq, ref.q_layers)[-1], ref._tower(xc, ref.c_layers)[-1]
    con2 = oracle.inbatch_softmax_xent_bf16(Qo, Co, lq)
    flips_q = float(np.mean(oracle.bf16_round(Qo) != oracle.bf16_round(qn)))
    flips_c = float(np.mean(oracle.bf16_round(Co) != oracle.bf16_round(cn)))
    S = qn.astype(np.float64) @ cn.T.astype(np.float64) - lq[None, :]
    print(f"step {step}: |s| mean {np.abs(S).mean():.3g} max {np.abs(S).max():.3g}; loss gpu {rl.sum():.6g} "
          f"contract {con['loss']:.6g}")
    print(f"  kernel vs contract(same q,c): dq {rel(dq, con['dq']):.2e} dc {rel(dc, con['dc']):.2e} "
          f"row_loss {rel(rl, con['row_loss']):.2e}")
    print(f"  towers: Q rel {rel(qn, Qo):.2e} C rel {rel(cn, Co):.2e}; bf16 flips q {flips_q:.2e} c {flips_c:.2e}")
    print(f"  kernel vs contract(oracle towers): dq {rel(dq, con2['dq']):.2e} dc {rel(dc, con2['dc']):.2e}")
    e = np.linalg.norm(dq - con["dq"], axis=1)
    top = np.argsort(-e)[:5]
    art = b["article_id"].cpu().numpy()
    for i in top:
        dup = int((art == art[i]).sum()) - 1
        print(f"    row {i}: err {e[i]:.3g} |dq| {np.linalg.norm(con['dq'][i]):.3g} loss {con['row_loss'][i]:.3g} "
              f"dup_positives {dup}")
    m.train_step(b)
