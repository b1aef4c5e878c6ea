"""Runs one tower GEMM shape repeatedly (for rocprofv3 PMC passes).
usage: python tools/gemm_probe.py {fwd,dx,dw} [x3|bf16]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd")]
import torch  # noqa: E402

from pkg.modelling import hip_ops  # noqa: E402

dev = torch.device("cuda:0")
kinds = sys.argv[1].split(",")
precs = [hip_ops.GEMM_BF16X3 if p == "x3" else hip_ops.GEMM_BF16 for p in (sys.argv[2] if len(sys.argv) > 2 else "x3").split(",")]
B, fin, fout = 16384, int(os.environ.get("FIN", 258)), int(os.environ.get("FOUT", 256))
X = torch.randn(B, fin + int(os.environ.get("PAD", 2)), device=dev)[:, :fin] * 0.05
G = torch.randn(B, fout, device=dev)
H = torch.relu(torch.randn(B, fout, device=dev))
W = torch.randn(fin, fout, device=dev) * 0.1
b = torch.randn(fout, device=dev)
y = torch.empty(B, fout, device=dev)
gx = torch.empty(B, fin, device=dev)
part = torch.empty(64, fin + 1, fout, device=dev)
import ctypes  # noqa: E402
from pkg import _native  # noqa: E402

probe = int(os.environ.get("GEMM_PROBE", "0"))
ctypes.CDLL(_native.LIB_PATH).tt_gemm_set_probe(probe)
for kind, prec in [(k, p) for k in kinds for p in precs] * 10:
    if kind == "fwd":
        hip_ops.gemm(X, W, y, bias=b, relu=True, precision=prec)
    elif kind == "dx":
        hip_ops.gemm(G, W, gx, b_t=True, mask=H, mask_on="a", precision=prec)
    else:
        hip_ops.gemm(X, G, part, a_t=True, mask=H, mask_on="b", ones_row=True, splits=64, precision=prec)
torch.cuda.synchronize()
