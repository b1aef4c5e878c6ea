"""Diagnostic: where does the GPU train step deviate from the CPU restatement?"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
from oracle import oracle
from pkg.modelling import hip_ops
import test_model_gpu as T

cuda = torch.device("cuda:0")
m = T._small_model(cuda)
rng = np.random.default_rng(5)
b = T._batch(cuda, rng, 512)
q = m.query_tower.call({"cust": b["cust"], "post": b["post"]}).detach()
c = m.candidate_tower.call({"art": b["art"], "ptn": b["ptn"]}).detach()
lq = m.candidate_logq(b)
print("q stats", float(q.abs().mean()), float(q.max()), "c", float(c.abs().mean()), float(c.max()), "logq", float(lq.min()), float(lq.max()))
ref = oracle.inbatch_softmax_xent(q.cpu().numpy(), c.cpu().numpy(), lq.cpu().numpy())
lse, rl, dq = hip_ops.inbatch_rows(q, c, lq)
dc = hip_ops.inbatch_cols(q, lse, c, lq)
def rel(a, b): return float(np.linalg.norm(a - b) / np.linalg.norm(b))
print("loss", float(rl.sum()), ref["loss"], "dq rel", rel(dq.cpu().numpy(), ref["dq"]), "dc rel", rel(dc.cpu().numpy(), ref["dc"]))
e = np.abs(dc.cpu().numpy() - ref["dc"]).max(1); print("dc worst rows", np.argsort(-e)[:5], e[np.argsort(-e)[:5]], "ref norms", np.linalg.norm(ref["dc"], axis=1)[np.argsort(-e)[:5]])
print("art ids of worst", b["art"].cpu().numpy()[np.argsort(-e)[:5]], "logq", lq.cpu().numpy()[np.argsort(-e)[:5]])
