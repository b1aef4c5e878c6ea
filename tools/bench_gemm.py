import torch, time
dev = torch.device("cuda:0")
def t(fn, reps=50):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3
B = 16384
for fin, fout in ((258, 256), (200, 256), (256, 128)):
    A = torch.randn(B, fin, device=dev); G = torch.randn(B, fout, device=dev)
    out = torch.empty(fin, fout, device=dev)
    r = {"mm": t(lambda: torch.mm(A.t(), G, out=out))}
    for S in (4, 8, 16, 32, 64):
        def f(S=S):
            p = torch.bmm(A.view(S, B // S, fin).transpose(1, 2), G.view(S, B // S, fout))
            torch.sum(p, 0, out=out)
        r[f"splitk{S}"] = t(f)
    ones = torch.ones(B, device=dev); db = torch.empty(fout, device=dev)
    r["db_sum"] = t(lambda: torch.sum(G, 0, out=db))
    r["db_mv"] = t(lambda: torch.mv(G.t(), ones, out=db))
    W = torch.randn(fin, fout, device=dev); b = torch.randn(fout, device=dev)
    r["fwd_addmm"] = t(lambda: torch.addmm(b, A, W))
    r["dx_mm"] = t(lambda: torch.mm(G, W.t()))
    H = torch.relu(torch.randn(B, fout, device=dev))
    r["thr_bwd"] = t(lambda: torch.ops.aten.threshold_backward(G, H, 0))
    flops = 2 * B * fin * fout
    print(fin, fout, {k: f"{v:.1f}us({flops / v / 1e6:.0f}TF)" for k, v in r.items()})
