"""hipBLASLt fp32 vs its fast-fp32 (allow_tf32) path for every tower GEMM at
C3: time and error vs fp64.  usage (GPU box): python tools/tf32_probe.py"""
import torch

dev = torch.device("cuda:0")
B = 16384


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


for fin, fout in ((258, 256), (200, 256), (256, 128)):
    X = torch.randn(B, fin, device=dev) * 0.05
    W = torch.randn(fin, fout, device=dev) * 0.1
    G = torch.randn(B, fout, device=dev)
    b = torch.randn(fout, device=dev)
    for flag in (False, True):
        torch.backends.cuda.matmul.allow_tf32 = flag
        y = X @ W
        err = ((y.double() - X.double() @ W.double()).norm() / (X.double() @ W.double()).norm()).item()
        r = {"fwd": t(lambda: torch._addmm_activation(b, X, W)), "dx": t(lambda: torch.mm(G, W.t())),
             "dw_mm": t(lambda: torch.mm(X.t(), G)),
             **{f"dw_bmm{S}": t(lambda S=S: torch.bmm(X.view(S, B // S, fin).transpose(1, 2),
                                                      G.view(S, B // S, fout))) for S in (8, 16, 32, 64)}}
        print(fin, fout, "fast" if flag else "fp32", f"rel err {err:.1e}", {k: round(v, 1) for k, v in r.items()},
              flush=True)
