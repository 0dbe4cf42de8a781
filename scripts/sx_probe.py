import torch, numpy as np, time
dev = torch.device("cuda", 0)
V, K, d = 1_000_000, 50, 128
X = torch.randn(V, d, device=dev)
resp = torch.rand(V, K, device=dev)
def t(fn, n=10):
    fn(); torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n): out = fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / n, out
def splitk(C=256):
    n = V // C * C
    part = torch.bmm(resp[:n].view(C, n // C, K).transpose(1, 2), X[:n].view(C, n // C, d)).sum(0)
    if n < V:
        part = part + resp[n:].t() @ X[n:]
    return part
def splitk64(C=256):
    n = V // C * C
    part = torch.bmm(resp[:n].view(C, n // C, K).transpose(1, 2), X[:n].view(C, n // C, d)).double().sum(0)
    if n < V:
        part = part + (resp[n:].t() @ X[n:]).double()
    return part
ms, ref = t(lambda: resp.t() @ X)
print("resp.t()@X", round(ms, 3))
print("nk sum f64", round(t(lambda: resp.sum(0, dtype=torch.float64))[0], 3))
print("nk sum f32", round(t(lambda: resp.sum(0))[0], 3))
for C in (64, 256, 1000, 4000):
    ms, o = t(lambda: splitk(C))
    print("splitk", C, round(ms, 3), float((o - ref).abs().max() / ref.abs().max()))
ms, o = t(lambda: splitk64(1000))
print("splitk64 1000", round(ms, 3))
r64 = resp.double(); X64 = X.double()
# k-means centre sums: index_add_ of V rows into K rows vs a one-hot split-K batched GEMM
labels = torch.randint(0, K, (V,), device=dev)
def ia():
    S = torch.zeros((K, d), dtype=torch.float32, device=dev)
    S.index_add_(0, labels, X)
    return S
def oh():
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from come_amd import gmm
    return gmm.resp_t_x(torch.nn.functional.one_hot(labels, K).float(), X).float()
ms_ia, s_ia = t(ia)
ms_oh, s_oh = t(oh)
print("index_add_", round(ms_ia, 3), "one-hot split-K", round(ms_oh, 3),
      float((s_ia - s_oh).abs().max() / s_ia.abs().max()))
