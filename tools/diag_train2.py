import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import test_model_gpu as T
cuda = torch.device("cuda:0")
for zipf in (False, True):
    m = T._small_model(cuda); ref = T._cpu_mirror(m); rng = np.random.default_rng(5)
    t0 = m.candidate_tower.input_layer.embedding_layers["art"].weight.cpu().numpy().copy()
    q0 = m.query_tower.input_layer.embedding_layers["cust"].weight.cpu().numpy().copy()
    f0 = m.candidate_tower.dense.flat.detach().cpu().numpy().copy()
    for step in range(3):
        b = T._batch(cuda, rng, 512, zipf)
        lq = m.candidate_logq(b).cpu().numpy()
        rl = ref.step([b["cust"].cpu().numpy(), b["post"].cpu().numpy()], [b["art"].cpu().numpy(), b["ptn"].cpu().numpy(), b["ptn"].cpu().numpy()], lq)
        gl = float(m.train_step(b)["loss"].item())
        t1 = m.candidate_tower.input_layer.embedding_layers["art"].weight.cpu().numpy()
        q1 = m.query_tower.input_layer.embedding_layers["cust"].weight.cpu().numpy()
        f1 = m.candidate_tower.dense.flat.detach().cpu().numpy()
        rf = np.concatenate([np.concatenate([w.reshape(-1), bb]) for w, bb in ref.c_layers])
        r = lambda a, b0, c: float(np.linalg.norm((a - b0) - (c - b0)) / np.linalg.norm(c - b0))
        print(f"zipf={zipf} step {step}: loss {gl:.4f} vs {rl:.4f}; art upd rel {r(t1, t0, ref.c_tables[0]):.2e}; cust upd rel {r(q1, q0, ref.q_tables[0]):.2e}; cand mlp rel {r(f1, f0, rf):.2e}")
