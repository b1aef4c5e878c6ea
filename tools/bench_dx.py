"""dx of the query tower's first layer at C3 ([16384,256] x [256,258]^T):
hipBLASLt tile choice at N = 258 vs a split into N = 256 + N = 2."""
import torch

dev = torch.device("cuda:0")
B = 16384
g = torch.randn(B, 256, device=dev)
W = torch.randn(258, 256, device=dev)
gx = torch.empty(B, 260, device=dev)


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


def split():
    torch.mm(g, W[:256].t(), out=gx[:, :256])
    torch.mm(g, W[256:].t(), out=gx[:, 256:258])


ref = torch.mm(g, W.t())
split()
torch.cuda.synchronize()
print("max diff", (gx[:, :258] - ref).abs().max().item())
print({"mm_258": t(lambda: torch.mm(g, W.t())), "split_256_2": t(split),
       "mm_256": t(lambda: torch.mm(g, W[:256].t())), "mm_2": t(lambda: torch.mm(g, W[256:].t()))})
