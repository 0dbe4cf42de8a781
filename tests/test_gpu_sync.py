"""Fused delta-exchange passes (come_delta_begin / come_delta_end) on the GPU: bit-identical to
the torch arithmetic the gloo tests check (tests/test_distributed.py), and the overlapped
DeltaAllReduce protocol on CUDA tables with a stand-in all-reduce."""
import numpy as np
import pytest
import torch

from come_amd import distributed as cd

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def test_fused_passes_match_torch_ops():
    g = torch.Generator(device=DEV)
    g.manual_seed(0)
    n = 4 * 100003
    W, S, Dsum = (torch.randn(n, device=DEV, generator=g) for _ in range(3))
    D, Down = torch.empty_like(W), torch.empty_like(W)
    cd._native("come_delta_begin", W, S, D, Down)
    assert torch.equal(D, W - S) and torch.equal(Down, W - S)
    W2, S2 = W.clone(), S.clone()
    cd._native("come_delta_end", W2, S2, Dsum, Down)
    assert torch.equal(S2, S + Dsum)
    assert torch.equal(W2, W + (Dsum - Down))


def test_overlapped_protocol_on_cuda_tables():
    """Two ranks simulated in one process (distributed.LocalReplicas: the all-reduce is a sum over
    both ranks' delta buffers) through the fused HIP passes: progress made while the exchange is
    in flight survives, others' deltas land exactly once; a blocking exchange afterwards leaves
    both replicas bit-identical."""
    rng = np.random.RandomState(1)
    base = torch.from_numpy(rng.randn(64, 32).astype(np.float32)).to(DEV)
    group = cd.LocalReplicas(2)
    ranks = [cd.DeltaAllReduce([base.clone()], comm=group.comm(r)) for r in range(2)]
    d0 = [torch.from_numpy(rng.randn(64, 32).astype(np.float32)).to(DEV) for _ in range(2)]
    for s, d in zip(ranks, d0):
        s.tables[0].add_(d)
    for s in ranks:
        s.start()
    later = [torch.from_numpy(rng.randn(64, 32).astype(np.float32)).to(DEV) for _ in range(2)]
    for s, d in zip(ranks, later):
        s.tables[0].add_(d)
    for s in ranks:
        s.finish()
    for r, s in enumerate(ranks):
        expect = base + d0[0] + d0[1] + later[r]
        torch.testing.assert_close(s.tables[0], expect, rtol=0, atol=1e-5)
        torch.testing.assert_close(s.snap[0], base + d0[0] + d0[1], rtol=0, atol=1e-5)
    for s in ranks:
        s.start()
    for s in ranks:
        s.finish()
        s.settle()
    assert torch.equal(ranks[0].tables[0], ranks[1].tables[0])
    torch.testing.assert_close(ranks[0].tables[0], base + d0[0] + d0[1] + later[0] + later[1],
                               rtol=0, atol=2e-5)


def test_row_sparse_passes_match_torch_ops():
    """come_delta_flags / gather / scatter (SparseDeltaAllReduce's device passes) against the
    torch restatement its gloo path uses: bitwise row flags (a -0.0 vs +0.0 change counts), the
    gathered deltas and the scatter update, bit for bit."""
    from come_amd import _lib
    from come_amd._lib import check, ptr, stream_handle
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    for rows, d in ((5000, 128), (333, 256), (17, 4)):
        S = torch.randn(rows, d, device=DEV, generator=g)
        W = S.clone()
        ch = torch.randperm(rows, device=DEV, generator=g)[:rows // 3]
        W[ch] += torch.randn(len(ch), d, device=DEV, generator=g)
        W[0] = S[0]
        S[1, 0], W[1, 0] = 0.0, -0.0
        f = torch.empty(rows, dtype=torch.uint8, device=DEV)
        st = stream_handle(DEV)
        check(_lib.lib().come_delta_flags(ptr(W), ptr(S), rows, d, ptr(f), st), "flags")
        ref = (W.view(torch.int32) != S.view(torch.int32)).any(1).to(torch.uint8)
        assert torch.equal(f, ref) and int(f[1]) == 1 and int(f[0]) == 0
        idx = torch.nonzero(f).view(-1)
        n = idx.numel()
        D, Down = W.new_empty((n, d)), W.new_empty((n, d))
        check(_lib.lib().come_delta_gather(ptr(W), ptr(S), ptr(idx), n, d, ptr(D), ptr(Down), st),
              "gather")
        assert torch.equal(D, W[idx] - S[idx]) and torch.equal(Down, D)
        Dsum = torch.randn(n, d, device=DEV, generator=g)
        W2, S2 = W.clone(), S.clone()
        check(_lib.lib().come_delta_scatter(ptr(W2), ptr(S2), ptr(idx), n, d, ptr(Dsum),
                                            ptr(Down), st), "scatter")
        S3, W3 = S.clone(), W.clone()
        S3[idx] = S[idx] + Dsum
        W3[idx] = W[idx] + (Dsum - Down)
        assert torch.equal(S2, S3) and torch.equal(W2, W3)
