"""tt_mlp_rows at the C3 tower shapes: error vs a torch fp64 reference and
time vs torch fp32 (hipBLASLt), both replayed from hipGraphs between HIP events.

usage: python tools/time_mlp.py [M]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hm-retrieval-two-tower_amd")]
import torch  # noqa: E402

from pkg.modelling import hip_ops  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
g.manual_seed(0)


def gtime(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side), torch.cuda.graph(graph, stream=side):
        for _ in range(reps):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    graph.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def rel(a, b):
    return float((a.double() - b).norm() / b.norm().clamp_min(1e-300))


for K1 in (258, 200):
    ld = (K1 + 3) // 4 * 4
    X = torch.zeros(M, ld, device=dev)
    X[:, :K1] = torch.randn(M, K1, generator=g, device=dev) * 0.05
    W1 = torch.randn(K1, 256, generator=g, device=dev) * (6.0 / (K1 + 256)) ** 0.5
    b1 = torch.randn(256, generator=g, device=dev) * 0.01
    W2 = torch.randn(256, 128, generator=g, device=dev) * (6.0 / 384) ** 0.5
    b2 = torch.randn(128, generator=g, device=dev) * 0.01
    Xv = X[:, :K1]
    img1, img2 = hip_ops.mlp_pack(W1), hip_ops.mlp_pack(W2)
    img2t, img1t = hip_ops.mlp_pack(W2, trans=True), hip_ops.mlp_pack(W1, trans=True)
    H1 = torch.empty(M, 256, device=dev)
    E = torch.empty(M, 128, device=dev)
    G1 = torch.empty(M, 256, device=dev)
    DX = torch.empty(M, K1, device=dev)
    G2 = torch.randn(M, 128, generator=g, device=dev)
    s = torch.full((), 0.5, device=dev)

    f1 = lambda: hip_ops.mlp_rows(Xv, img1, K1, 256, H1, bias=b1, relu=True)
    f2 = lambda: hip_ops.mlp_rows(H1, img2, 256, 128, E, bias=b2, relu=True)
    f3 = lambda: hip_ops.mlp_rows(G2, img2t, 128, 256, G1, amask=E, scale=s, cmask=H1)
    f4 = lambda: hip_ops.mlp_rows(G1, img1t, 256, K1, DX)
    f1(); f2(); f3(); f4()
    torch.cuda.synchronize()
    Xd, W1d, W2d = Xv.double(), W1.double(), W2.double()
    H1r = torch.relu(Xd @ W1d + b1.double())
    print(f"K1={K1} fwd1 rel {rel(H1, H1r):.2e}")
    Er = torch.relu(H1.double() @ W2d + b2.double())
    print(f"K1={K1} fwd2 rel {rel(E, Er):.2e}")
    G1r = ((G2.double() * (E > 0).double() * 0.5) @ W2d.t()) * (H1 > 0).double()
    print(f"K1={K1} dx2 rel {rel(G1, G1r):.2e}")
    DXr = G1.double() @ W1d.t()
    print(f"K1={K1} dx1 rel {rel(DX, DXr):.2e}")
    t = [gtime(f) for f in (f1, f2, f3, f4)]
    tp = [gtime(lambda: torch._addmm_activation(b1, Xv, W1)), gtime(lambda: torch._addmm_activation(b2, H1, W2)),
          gtime(lambda: torch.mm(G2, W2.t())), gtime(lambda: torch.mm(G1, W1.t()))]
    tpk = gtime(lambda: (hip_ops.mlp_pack(W1, out=img1), hip_ops.mlp_pack(W2, out=img2)))
    dwb1 = torch.empty(K1 + 1, 256, device=dev)
    dwb2 = torch.empty(257, 128, device=dev)
    hip_ops.mlp_wgrad(Xv, G1, dwb1)
    hip_ops.mlp_wgrad(H1, G2, dwb2, gmask=E, scale=s)
    torch.cuda.synchronize()
    r1 = torch.cat([Xd, torch.ones(M, 1, dtype=torch.float64, device=dev)], 1).t() @ G1.double()
    r2 = torch.cat([H1.double(), torch.ones(M, 1, dtype=torch.float64, device=dev)], 1).t() @ (
        G2.double() * (E > 0).double() * 0.5)
    print(f"K1={K1} wgrad1 rel {rel(dwb1, r1):.2e} wgrad2 rel {rel(dwb2, r2):.2e}")
    tw1 = gtime(lambda: hip_ops.mlp_wgrad(Xv, G1, dwb1))
    tw2 = gtime(lambda: hip_ops.mlp_wgrad(H1, G2, dwb2, gmask=E, scale=s))
    tb1 = gtime(lambda: torch.mm(Xv.t(), G1, out=dwb1[:K1]))
    tb2 = gtime(lambda: torch.mm(H1.t(), G2, out=dwb2[:256]))
    print(f"K1={K1} us wgrad tt: dW1 {tw1:.1f} dW2(+mask) {tw2:.1f} | torch mm (hipBLASLt): {tb1:.1f} {tb2:.1f}")
    print(f"K1={K1} us tt: fwd1 {t[0]:.1f} fwd2 {t[1]:.1f} dx2 {t[2]:.1f} dx1 {t[3]:.1f} | "
          f"torch: {tp[0]:.1f} {tp[1]:.1f} {tp[2]:.1f} {tp[3]:.1f} | pack x2 {tpk:.1f}")
