"""Multi-process (world size 2, gloo, CPU) tests of the row-sharded C4 path: the
distributed GMM EM (sufficient-statistics all-reduce) and the sharded community step (row
all-gather).  The HIP kernels need a GPU, so the CPU workers swap them for float64 torch
stand-ins of the same ops (test infrastructure); what is under test is the host-side sharding
and exchange protocol in come_amd.gmm / come_amd.community_embeddings / come_amd.distributed.
The GPU kernels themselves are covered by tests/test_gpu_gmm.py."""
import os
import socket
import types

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from come_amd import community_embeddings as ce
from come_amd import gmm
from come_amd.distributed import all_gather_rows, all_reduce_sum, shard_range
from oracle import oracle as orc

V, D, K = 203, 4, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# ---- CPU stand-ins for the HIP entry points (same maths, float64) ------------------------------
def _cpu_estep(X, prec_chol, mu_prec, log_norm):
    Y = torch.einsum("vd,kde->vke", X.double(), prec_chol.double()) - mu_prec.double()[None]
    logp = -0.5 * (Y ** 2).sum(-1) + log_norm.double()[None]
    lse = torch.logsumexp(logp, 1)
    return torch.exp(logp - lse[:, None]).float(), lse.float()


def _cpu_scatter(X, resp, means, chunks=None):
    Xc = X.double()[:, None, :] - means.double()[None]
    return torch.einsum("vk,vkd,vke->kde", resp.double(), Xc, Xc).float()


def _cpu_params(S, nk, means, weights, reg):
    import math
    d = S.shape[-1]
    cov = S / nk[:, None, None] + reg * torch.eye(d, dtype=torch.float64)
    chol, info = torch.linalg.cholesky_ex(cov)
    eye = torch.eye(d, dtype=torch.float64).expand_as(cov)
    pc = torch.linalg.solve_triangular(chol, eye, upper=False).transpose(-1, -2).contiguous()
    log_det = torch.log(torch.diagonal(pc, dim1=-2, dim2=-1)).sum(-1)
    e_mp = torch.einsum("kd,kde->ke", means, pc).float()
    e_ln = (torch.log(weights) + log_det - 0.5 * d * math.log(2 * math.pi)).float()
    return cov, pc, pc.float(), e_mp, e_ln, info.int()


def _cpu_community_grad(x, pi, mu, inv, beta, lr, iters):
    x.copy_(torch.from_numpy(orc.community_train(x.numpy(), pi.numpy(), mu.numpy(), inv.numpy(),
                                                 beta, lr, iters)))


def _cpu_gmm_resp(x, pc, mp_, ln):
    return _cpu_estep(x, pc, mp_, ln)[0]


def _patch(setattr_=setattr):
    setattr_(gmm, "estep", _cpu_estep)
    setattr_(gmm, "scatter", _cpu_scatter)
    setattr_(gmm, "params", _cpu_params)
    setattr_(gmm.GaussianMixture, "_prepare_x",
             lambda self, X: torch.as_tensor(X, dtype=torch.float32).contiguous())
    setattr_(ce, "community_grad", _cpu_community_grad)
    setattr_(ce, "gmm_resp", _cpu_gmm_resp)


def _data():
    rng = np.random.RandomState(7)
    centres = np.array([[4, 0, 0, 0], [0, 4, 0, 0], [0, 0, 4, 1]], np.float32)
    lab = rng.randint(0, K, V)
    X = (centres[lab] + rng.standard_normal((V, D)) * 0.5).astype(np.float32)
    w0 = np.full(K, 1.0 / K)
    mu0 = centres.astype(np.float64) + 0.3
    prec0 = np.stack([np.eye(D) * 2.0] * K)
    return X, lab, w0, mu0, prec0


def _model(X, rng_seed=3):
    rng = np.random.RandomState(rng_seed)
    m = types.SimpleNamespace()
    m.k, m.vocab_size = K, V
    m.node_embedding = torch.from_numpy(X.copy())
    m.pi = torch.from_numpy(rng.dirichlet(np.ones(K), V).astype(np.float32))
    m.centroid = torch.from_numpy(rng.standard_normal((K, D)).astype(np.float32))
    A = rng.standard_normal((K, D, D)).astype(np.float32)
    m.inv_covariance_mat = torch.from_numpy(
        (np.einsum("kij,klj->kil", A, A) + np.eye(D, dtype=np.float32)).astype(np.float32))
    m.rows_of = lambda ids: np.asarray(ids, np.int64) - 1  # node id i -> row i-1
    return m


def _run(rank, world, out_dir, distributed):
    """Same program on one process (distributed=False) or on each rank."""
    X, lab, w0, mu0, prec0 = _data()
    lo, hi = shard_range(V, rank, world) if distributed else (0, V)
    res = {}
    # 1. EM from fixed initial parameters (sklearn weights_init / means_init / precisions_init)
    g = gmm.GaussianMixture(K, reg_covar=1e-5, max_iter=15, tol=0.0, weights_init=w0,
                            means_init=mu0, precisions_init=prec0, distributed=distributed)
    g.fit(X[lo:hi])
    res.update(weights=g.weights_, means=g.means_, cov=g.covariances_, lb=g.lower_bound_,
               n_iter=g.n_iter_, score=g.score(X[lo:hi]))
    # 2. k-means initialised fit (seeding on rank 0's shard): separated blobs are recovered
    g2 = gmm.GaussianMixture(K, reg_covar=1e-5, n_init=2, random_state=0,
                             distributed=distributed)
    lab_local = g2.fit_predict(X[lo:hi])
    full = torch.zeros(V, dtype=torch.int64)
    full[lo:hi] = lab_local
    if distributed:
        all_gather_rows(full)
    res["kmeans_labels"] = full.numpy()
    # 3. community step: every row, then a subset of nodes
    m = _model(X)
    c2v = ce.Community2Vec.__new__(ce.Community2Vec)
    c2v.lr, c2v.gmm_backend, c2v.distributed, c2v.group = 0.1, "gpu", distributed, None
    c2v.train(np.arange(1, V + 1), m, beta=0.5, iter=3)
    res["x_full"] = m.node_embedding.numpy().copy()
    c2v.train(np.arange(1, V + 1, 3)[::-1], m, beta=0.5, iter=2)
    res["x_sub"] = m.node_embedding.numpy().copy()
    # 4. responsibilities of the fitted mixture, all-gathered
    c2v.g_mixture = g
    res["pi"] = c2v.responsibilities(m).numpy()
    np.savez(os.path.join(out_dir, "res_%s_r%d.npz" % ("dist" if distributed else "single",
                                                     rank)), **res)


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _patch()
    # helpers first: all_reduce_sum over a mixed-shape list, all_gather_rows with ragged shards
    a, b = torch.full((3,), float(rank + 1)), torch.full((2, 2), 10.0 * (rank + 1))
    all_reduce_sum([a, b])
    assert torch.equal(a, torch.full((3,), 3.0)) and torch.equal(b, torch.full((2, 2), 30.0))
    t = torch.full((7, 2), -1.0)
    lo, hi = shard_range(7, rank, world)
    t[lo:hi] = rank
    all_gather_rows(t)
    expect = torch.tensor([0.0] * 4 + [1.0] * 3)[:, None].expand(7, 2)
    assert torch.equal(t, expect), t
    _run(rank, world, out_dir, True)
    dist.destroy_process_group()


def test_c4_row_sharded_world2(tmp_path, monkeypatch):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    _patch(monkeypatch.setattr)  # undone after the test
    _run(0, 1, str(tmp_path), False)
    single = np.load(os.path.join(str(tmp_path), "res_single_r0.npz"))
    r0 = np.load(os.path.join(str(tmp_path), "res_dist_r0.npz"))
    r1 = np.load(os.path.join(str(tmp_path), "res_dist_r1.npz"))
    for key in r0.files:  # every rank ends with the same parameters and replicas, bit for bit
        np.testing.assert_array_equal(r0[key], r1[key], err_msg=key)
    # EM over shards == EM over all rows up to the summation order of the statistics
    for key in ("weights", "means", "cov"):
        np.testing.assert_allclose(r0[key], single[key], rtol=1e-5, atol=1e-6, err_msg=key)
    assert int(r0["n_iter"]) == int(single["n_iter"])
    np.testing.assert_allclose(float(r0["lb"]), float(single["lb"]), rtol=1e-6)
    np.testing.assert_allclose(float(r0["score"]), float(single["score"]), rtol=1e-6)
    # community rows are independent: the sharded step equals the single-process one
    np.testing.assert_array_equal(r0["x_full"], single["x_full"])
    np.testing.assert_array_equal(r0["x_sub"], single["x_sub"])
    np.testing.assert_allclose(r0["pi"], single["pi"], rtol=1e-4, atol=1e-6)
    # k-means seeded on rank 0's shard still recovers the three separated blobs
    _, lab, _, _, _ = _data()
    for labels in (r0["kmeans_labels"], single["kmeans_labels"]):
        pairs = set(zip(lab.tolist(), labels.tolist()))
        assert len(pairs) == K, pairs
