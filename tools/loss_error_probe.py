"""Measure the fused in-batch loss error against the fp64 restatement.

Prints, per configuration, the relative loss error, max |lse - ref|, and the
norm-relative dq / dc errors; then the model-level loss error over 3 train
steps (small model of tests/test_model_gpu.py).  Used to set the precision
contract of DESIGN.md §6.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle  # noqa: E402
from pkg.modelling import hip_ops  # noqa: E402


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def kernel_cases():
    dev = torch.device("cuda:0")
    cases = [(64, 16, False, 1.0), (300, 64, True, 0.5), (1024, 128, True, 0.3), (2048, 128, True, 1.0),
             (129, 100, False, 0.2), (8192, 128, True, 0.3), (4100, 64, True, 0.7), (2500, 32, False, 0.6),
             (1100, 128, True, 0.5), (60, 8, True, 1.0), (4096, 64, True, 0.3), (512, 32, True, 2.0),
             (37, 32, True, 1.0), (2, 32, True, 1.0)]
    for B, E, use_logq, scale in cases:
        rng = np.random.default_rng(B * 7 + E)
        q = np.maximum(rng.standard_normal((B, E)) * scale, 0).astype(np.float32)
        c = np.maximum(rng.standard_normal((B, E)) * scale, 0).astype(np.float32)
        logq = np.log(rng.uniform(1e-6, 1e-2, B)).astype(np.float32) if use_logq else None
        ref = oracle.inbatch_softmax_xent(q, c, logq)
        t = lambda x: torch.as_tensor(x, device=dev)
        lse, row_loss, dq, dc = hip_ops.inbatch_fused(t(q), t(c), t(logq) if use_logq else None)
        loss = float(row_loss.double().sum())
        print(f"kernel B={B:5d} E={E:3d} logq={int(use_logq)} scale={scale:4.2f}: loss {ref['loss']:.5g} "
              f"rel {abs(loss - ref['loss']) / abs(ref['loss']):.2e}  lse maxabs "
              f"{np.abs(lse.cpu().numpy() - ref['lse']).max():.2e}  dq {rel(dq.cpu().numpy(), ref['dq']):.2e}  "
              f"dc {rel(dc.cpu().numpy(), ref['dc']):.2e}", flush=True)


def model_cases():
    import test_model_gpu as tm

    dev = torch.device("cuda:0")
    for zipf in (True, False):
        m = tm._small_model(dev)
        ref = tm._cpu_mirror(m)
        rng = np.random.default_rng(5)
        for step in range(3):
            b = tm._batch(dev, rng, 512, zipf)
            lq = m.candidate_logq(b).cpu().numpy()
            rl = ref.step([b["cust"].cpu().numpy(), b["post"].cpu().numpy()],
                          [b["art"].cpu().numpy(), b["ptn"].cpu().numpy(), b["ptn"].cpu().numpy()], lq)
            gl = float(m.train_step(b)["loss"].item())
            print(f"model zipf={int(zipf)} step {step}: loss {rl:.6g} rel {abs(gl - rl) / abs(rl):.2e}", flush=True)
    for B in (1, 2, 37, 1000):
        m = tm._small_model(dev, seed=B)
        ref = tm._cpu_mirror(m)
        rng = np.random.default_rng(B)
        b = tm._batch(dev, rng, B, True)
        lq = m.candidate_logq(b).cpu().numpy()
        rl = ref.step([b["cust"].cpu().numpy(), b["post"].cpu().numpy()],
                      [b["art"].cpu().numpy(), b["ptn"].cpu().numpy(), b["ptn"].cpu().numpy()], lq)
        gl = float(m.train_step(b)["loss"].item())
        print(f"model ragged B={B}: loss {rl:.6g} abs {abs(gl - rl):.2e} rel {abs(gl - rl) / max(abs(rl), 1e-30):.2e}",
              flush=True)


if __name__ == "__main__":
    kernel_cases()
    model_cases()
