import torch, time
dev = torch.device("cuda:0")
B = 16384
def t(fn, reps=50):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3
X = torch.randn(B, 258, device=dev) * 0.05
W = torch.randn(258, 256, device=dev) * 0.1
G = torch.randn(B, 256, device=dev)
b = torch.randn(256, device=dev)
ref = (X.double() @ W.double())
for flag in (False, True):
    torch.backends.cuda.matmul.allow_tf32 = flag
    y = X @ W
    err = ((y.double() - ref).norm() / ref.norm()).item()
    r = {"fwd": t(lambda: torch._addmm_activation(b, X, W)), "dx": t(lambda: torch.mm(G, W.t())),
         "dw_bmm16": t(lambda: torch.bmm(X.view(16, B // 16, 258).transpose(1, 2), G.view(16, B // 16, 256)))}
    print("allow_tf32", flag, "rel err", err, {k: round(v, 1) for k, v in r.items()}, flush=True)
