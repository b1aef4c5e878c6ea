"""Times libtt's tower GEMMs (tt_gemm) at the C3 shapes against the torch
fp32 GEMMs they replace.  usage (GPU box): python tools/bench_tt_gemm.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd")]

import torch  # noqa: E402

from pkg.modelling import hip_ops  # noqa: E402
from pkg.modelling.models.tower import _weight_grad_splits  # noqa: E402

dev = torch.device("cuda:0")


def t(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


B = int(os.environ.get("B", 16384))
splits_env = os.environ.get("SPLITS")
for fin, fout in ((258, 256), (200, 256), (256, 128)):
    X = torch.randn(B, fin + 2, device=dev)[:, :fin] * 0.05
    G = torch.randn(B, fout, device=dev)
    H = torch.relu(torch.randn(B, fout, device=dev))
    W = torch.randn(fin, fout, device=dev) * 0.1
    b = torch.randn(fout, device=dev)
    s = torch.ones(1, device=dev)
    flops = 2 * B * fin * fout
    r = {}
    for name, prec in (("x3", hip_ops.GEMM_BF16X3), ("bf16", hip_ops.GEMM_BF16)):
        y = torch.empty(B, fout, device=dev)
        r[f"fwd_{name}"] = t(lambda: hip_ops.gemm(X, W, y, bias=b, relu=True, precision=prec))
        gx = torch.empty(B, fin, device=dev)
        r[f"dx_{name}"] = t(lambda: hip_ops.gemm(G, W, gx, b_t=True, mask=H, mask_on="a", scale=s, precision=prec))
        S = int(splits_env) if splits_env else _weight_grad_splits(B, fin, fout)
        part = torch.empty(S, fin + 1, fout, device=dev)
        dwb = torch.empty(fin + 1, fout, device=dev)

        def wg():
            hip_ops.gemm(X, G, part, a_t=True, mask=H, mask_on="b", ones_row=True, splits=S, precision=prec)
            hip_ops.sum_slices(part, dwb)
        r[f"dw_{name}(S={S})"] = t(wg)
        r[f"dw_gemm_only_{name}"] = t(lambda: hip_ops.gemm(X, G, part, a_t=True, mask=H, mask_on="b", ones_row=True,
                                                           splits=S, precision=prec))
    Xc = X.contiguous()
    r["torch_fwd_fp32"] = t(lambda: torch._addmm_activation(b, Xc, W))
    r["torch_dx_fp32"] = t(lambda: torch.mm(G, W.t()))
    print(fin, fout, {k: f"{v:.1f}us({flops / v / 1e6:.0f}TF)" for k, v in r.items()}, flush=True)
