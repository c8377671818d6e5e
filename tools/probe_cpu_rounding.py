"""Probe how THIS host's CPU torch rounds the ops PyG's GINEConv uses (run on any box).
Prints: CPU model, whether F.linear(K=1) == fma / == mul-then-add, whether scatter_add_ and
index_add_ accumulate sequentially in edge order."""
import platform, subprocess, sys
import numpy as np
import torch
import torch.nn.functional as F

def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
        return [l for l in out.splitlines() if "Model name" in l or "Flags" in l and False][0]
    except Exception:
        return platform.processor()

print("cpu:", cpu_model(), "threads", torch.get_num_threads())
print(torch.__config__.show().splitlines()[0:12])
g = torch.Generator().manual_seed(5)
a = torch.randn(20000, 1, generator=g) * 3
w = torch.randn(64, 1, generator=g)
b = torch.randn(64, generator=g)
lin = F.linear(a, w, b)
fma = (a.double() * w.double().T + b.double()).float()
muladd = (a * w.T) + b
print("F.linear == fma:", torch.equal(lin, fma), "mismatch", (lin != fma).float().mean().item())
print("F.linear == mul+add:", torch.equal(lin, muladd), "mismatch", (lin != muladd).float().mean().item())
addmm = torch.addmm(b, a, w.T)
print("addmm == F.linear:", torch.equal(addmm, lin))
for n_edges in (20000, 200):
    aa = a[:n_edges]
    l2 = F.linear(aa, w, b)
    print(f"E={n_edges}: == fma {torch.equal(l2, fma[:n_edges])}, == mul+add {torch.equal(l2, muladd[:n_edges])}")
# scatter order
rng = np.random.default_rng(0)
E, N, D = 4000, 40, 16
dst = torch.from_numpy(rng.integers(0, N, E))
m = torch.randn(E, D) * torch.logspace(-3, 3, D)
agg = torch.zeros(N, D).scatter_add_(0, dst.view(-1, 1).expand_as(m), m)
ref = np.zeros((N, D), np.float32)
mn = m.numpy()
for e in range(E):
    ref[dst[e]] = (ref[dst[e]] + mn[e]).astype(np.float32)
print("scatter_add_ sequential:", np.array_equal(agg.numpy(), ref))
ia = torch.zeros(N, D).index_add_(0, dst, m)
print("index_add_ sequential:", np.array_equal(ia.numpy(), ref))
