"""Which torch gathers are wrong on this ROCm build at scale -- diagnostic for the device
chung_lu path.  Measured (round 3, r04): index_select / boolean-mask row selection of a [n, 2]
int64 tensor is correct up to n = 2^26 rows (2^25 selected), returns WRONG rows silently at
n = 1e8 (5e7 selected... up to all rows), and fails to launch ("invalid configuration argument")
at n = 2^27; 1-D gathers of up to 1e8 indices are correct.  This run: 1-D gathers at 2e8 and the
row gather tierc_inputs.compact_loss does from a 10M x 256 fp32 table (2.56e9 elements)."""
import numpy as np, torch
dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
n = 200_000_000
src = torch.arange(n, device=dev, dtype=torch.int64) * 3
idx = torch.as_tensor(rng.integers(0, n, n), device=dev)
got = src[idx]
print("1-D gather, 2e8 indices:", bool(torch.equal(got, idx * 3)), flush=True)
del src, idx, got
V, d = 10_000_000, 256
tab = torch.empty((V, d), device=dev, dtype=torch.float32)
tab[:, 0] = torch.arange(V, device=dev, dtype=torch.float32)       # exact below 2^24
tab[:, 1] = torch.arange(V, device=dev, dtype=torch.float32) / 1e7
tab[:, 2:] = 0.5
rows = torch.as_tensor(rng.integers(0, V, 2_200_000), device=dev)
g = tab[rows]
ok = bool(torch.equal(g[:, 1], rows.to(torch.float32) / 1e7)) and bool((g[:, 2:] == 0.5).all())
print("10M x 256 row gather of 2.2M rows:", ok, flush=True)
g2 = tab.index_select(0, rows)
print("index_select same:", bool(torch.equal(g, g2)), flush=True)
