"""Diagnostic: which phase of the GPU ComE flow loses NMI vs the CPU reference flow."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
from sklearn.metrics import normalized_mutual_info_score as NMI
from sklearn.mixture import GaussianMixture as SK
from come_amd.graph import random_walks, sbm
from come_amd.model import Model
from come_amd.node_embeddings import Node2Vec
from come_amd.context_embeddings import Context2Vec
from come_amd import gmm
import come_amd.training_sdg_inner as tsi
from oracle import oracle as orc

blocks, size, dim = 8, 250, 64
g = sbm(blocks, size, 0.04, 0.002, seed=3)
lab = np.arange(g.V) // size
walks = random_walks(g, 4, 30, seed=4, device="cuda")
res = {}
for det in (False, True):
    np.random.seed(3)
    m = Model(g.degree_by_id(), size=dim, table_size=max(10**6, 100*g.V), k=blocks)
    nl = Node2Vec(lr=0.025, negative=5, deterministic=det)
    cl = Context2Vec(lr=0.025, window_size=5, negative=5, deterministic=det)
    ids = torch.where(walks >= 0, walks + 1, walks)
    for _ in range(2):
        nl.train(m, edges=g.edge_ids(), iter=1)
        cl.train(m, paths=ids, total_nodes=walks.numel(), alpha=1.0)
    X = m.node_embedding.cpu().numpy()
    sk = SK(blocks, covariance_type="full", reg_covar=1e-5, n_init=3, random_state=3).fit(X)
    gg = gmm.GaussianMixture(blocks, reg_covar=1e-5, n_init=3, random_state=3).fit(X)
    res["gpu_train_det%d_sklearn_gmm" % det] = NMI(lab, sk.predict(X))
    res["gpu_train_det%d_gpu_gmm" % det] = NMI(lab, gg.predict(X).cpu().numpy())
    res["gpu_train_det%d_lb" % det] = (sk.lower_bound_, gg.lower_bound_)
# CPU-trained embeddings
np.random.seed(3)
node = np.random.uniform(-1, 1, (g.V, dim)).astype(np.float32)
ctx = np.zeros((g.V, dim), np.float32)
table = orc.make_table(g.degree, max(10**6, 100*g.V))
W = walks.cpu().numpy().astype(np.int32)
for _ in range(2):
    orc.sgns_o1(node, g.edges.astype(np.int32), tsi.draw_seeds(g.num_edges), 5, table, 0.025)
    orc.sgns_o2(node, ctx, W, tsi.draw_seeds(len(W)), 5, 5, table, 0.025, 1.0)
sk = SK(blocks, covariance_type="full", reg_covar=1e-5, n_init=3, random_state=3).fit(node)
gg = gmm.GaussianMixture(blocks, reg_covar=1e-5, n_init=3, random_state=3).fit(node)
res["cpu_train_sklearn_gmm"] = NMI(lab, sk.predict(node))
res["cpu_train_gpu_gmm"] = NMI(lab, gg.predict(node).cpu().numpy())
res["cpu_train_lb"] = (sk.lower_bound_, gg.lower_bound_)
for s in range(4):
    gg = gmm.GaussianMixture(blocks, reg_covar=1e-5, n_init=1, random_state=s).fit(node)
    sk = SK(blocks, covariance_type="full", reg_covar=1e-5, n_init=1, random_state=s).fit(node)
    res["cpu_train_seed%d" % s] = (NMI(lab, gg.predict(node).cpu().numpy()), gg.lower_bound_, gg.n_iter_, NMI(lab, sk.predict(node)), sk.lower_bound_, sk.n_iter_)
print(json.dumps(res, default=float))
