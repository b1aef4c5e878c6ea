"""Per-layer errors of DenseStack's backward against torch fp64 for odd and
aligned layer widths (diagnostic for test_dense_stack_odd_widths_vs_torch_fp64)."""
import sys

import torch

sys.path[:0] = [".", "hm-retrieval-two-tower_amd"]
from pkg.modelling.models.tower import DenseStack  # noqa: E402

cuda = torch.device("cuda", 0)
for in_dim, units, top in [(37, [66, 130], True), (37, [64, 128], True), (40, [68, 132], True),
                           (37, [66, 128], True), (37, [64, 130], True), (42, [6, 3], False)]:
    gen = torch.Generator()
    gen.manual_seed(in_dim + sum(units))
    st = DenseStack(in_dim, units, cuda, gen)
    M = 3000
    x = torch.randn(M, (in_dim + 3) // 4 * 4, device=cuda)[:, :in_dim]
    flat = st.flat.detach()
    acts = st.forward_acts(x, flat)
    gout = torch.randn(M, units[-1], device=cuda)
    s = torch.full((1,), 0.5, device=cuda) if top else None
    dx, gflat = st.backward_acts(acts, flat, gout.contiguous(), s, True)
    fd = flat.double().clone().requires_grad_(True)
    xd = x.double().clone().requires_grad_(True)
    h = xd
    for w_off, fi, fo, b_off in st.layout:
        h = torch.relu(h @ fd[w_off:w_off + fi * fo].view(fi, fo) + fd[b_off:b_off + fo])
    (h * gout.double() * (0.5 if top else 1.0)).sum().backward()
    errs = []
    for li, (w_off, fi, fo, b_off) in enumerate(st.layout):
        for nm, a, b in (("W", w_off, w_off + fi * fo), ("b", b_off, b_off + fo)):
            e = float((gflat[a:b].double() - fd.grad[a:b]).norm() / fd.grad[a:b].norm())
            errs.append(f"{nm}{li}={e:.2e}")
    e = float((dx.double() - xd.grad).norm() / xd.grad.norm())
    print(in_dim, units, " ".join(errs), f"dx={e:.2e}", flush=True)
