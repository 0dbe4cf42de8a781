"""Bisect the device chung_lu path step by step against numpy (C5 scale) -- diagnostic."""
import numpy as np, torch, time
V=10_000_000; mean_degree=20.0; gamma=2.5
dev=torch.device("cuda",0)
rng = np.random.default_rng(4)
w = (np.arange(V, dtype=np.float64) + 1.0) ** (-1.0 / (gamma - 1.0))
w *= mean_degree * V / w.sum()
cw = np.cumsum(w); cw /= cw[-1]
m = int(V * mean_degree / 2)
r1 = rng.random(m); r2 = rng.random(m); perm = rng.permutation(V)
uh = np.searchsorted(cw, r1, side="right"); vh = np.searchsorted(cw, r2, side="right")
eh = np.stack([perm[np.minimum(uh, V-1)], perm[np.minimum(vh, V-1)]], 1)
cwt = torch.as_tensor(cw, device=dev)
u = torch.searchsorted(cwt, torch.as_tensor(r1, device=dev), right=True)
v = torch.searchsorted(cwt, torch.as_tensor(r2, device=dev), right=True)
pt = torch.as_tensor(perm, device=dev)
e = torch.stack([pt[torch.clamp(u, max=V - 1)], pt[torch.clamp(v, max=V - 1)]], 1)
print("stack/gather equal", np.array_equal(e.cpu().numpy(), eh), flush=True)
ec = e.cpu().numpy()
e2 = torch.as_tensor(np.asarray(ec, np.int64).reshape(-1, 2), device=dev)
print("roundtrip equal", np.array_equal(e2.cpu().numpy(), eh), flush=True)
mask = e2[:, 0] != e2[:, 1]
mh = eh[:, 0] != eh[:, 1]
print("mask equal", np.array_equal(mask.cpu().numpy(), mh), int(mask.sum()), int(mh.sum()), flush=True)
e3 = e2[mask]
eh3 = eh[mh]
print("masked rows", e3.shape, eh3.shape, "equal", e3.shape == eh3.shape and np.array_equal(e3.cpu().numpy(), eh3), flush=True)
nz = torch.nonzero(mask).view(-1)
print("nonzero count", nz.numel(), flush=True)
e4 = e2.index_select(0, nz)
print("index_select equal", np.array_equal(e4.cpu().numpy(), eh3), flush=True)
