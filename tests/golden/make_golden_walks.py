"""Generate tests/golden/walks.npz FROM THE REFERENCE'S OWN utils/graph_utils.py.

Run in the build container only (needs /root/reference and networkx); only the resulting
input/output vectors are committed.  The reference module is imported read-only.

graph_utils was written for networkx 1.x, where ``G.neighbors(n)`` returns a list; under the
installed networkx 3 it returns an iterator and ``len()`` of it fails (graph_utils.py:36).  The
graphs are therefore handed to the reference's functions through ``Nx1View``, which only changes
``neighbors`` back to a list (same order) -- the reference's own code does every draw.

Cases (per case: the edge rows fed to add_edges_from, list(G.nodes()), np.array(G.edges()),
G.degree() values, and walks from the reference functions):
  karate      load_adjacencylist of the shipped Karate graph (graph_utils.py:72-109);
              build_deepwalk_corpus(G, 10, 20, alpha=0, rand=Random(9999999999)) (:172-185);
              write_walks_to_disk(..., num_workers=1 and 4) read back (:122-146, 149-154)
  karate_a03  the same corpus with restart alpha = 0.3
  messy       a random multigraph edge list with duplicates, reversed duplicates, self-loops
              and sparse ids (networkx ordering corner cases), 3 passes, alpha = 0.1
Every case also records the Random state after the corpus (getstate()[1]).
"""
import os
import random
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("COME_REFERENCE", "/root/reference")


class Nx1View(object):
    """networkx-1 surface over a networkx-3 graph: neighbors() as a list."""

    def __init__(self, G):
        self._G = G

    def neighbors(self, n):
        return list(self._G.neighbors(n))

    def nodes(self):
        return self._G.nodes()

    def __len__(self):
        return len(self._G)


def record(out, name, G, edges_in):
    out[name + "_edges_in"] = np.asarray(edges_in, np.int64)
    out[name + "_nodes"] = np.array(list(G.nodes()), np.int64)
    out[name + "_edges"] = np.array(G.edges(), np.int64).reshape(-1, 2)
    out[name + "_degree"] = np.array([d for _, d in G.degree()], np.int64)


def pad(walks, L):
    a = np.full((len(walks), L), -1, np.int64)
    for i, w in enumerate(walks):
        a[i, :len(w)] = w
    return a


def main():
    sys.path.insert(0, REF)
    import networkx as nx
    from utils import graph_utils as gu

    out = {}
    path = os.path.join(REF, "data", "karate", "karate.adjlist")
    G = gu.load_adjacencylist(path, True)
    edges_in = np.loadtxt(path, dtype=np.int64)
    record(out, "karate", G, edges_in)
    rnd = random.Random(9999999999)
    walks = gu.build_deepwalk_corpus(Nx1View(G), 10, 20, alpha=0, rand=rnd)
    out["karate_walks"] = pad(walks, 20)
    out["karate_state"] = np.array(rnd.getstate()[1], np.uint32)
    for workers in (1, 4):
        with tempfile.TemporaryDirectory() as td:
            gu.__dict__["__current_graph"] = None
            files = gu.write_walks_to_disk(Nx1View(G), os.path.join(td, "k.walks"),
                                           num_paths=10, path_length=20, alpha=0,
                                           rand=random.Random(9999999999), num_workers=workers)
            rows = list(gu.combine_files_iter(files))
            out["karate_files_w%d" % workers] = pad(rows, 20)
            out["karate_files_w%d_count" % workers] = np.array(
                [gu.count_lines(f) for f in files], np.int64)
    rnd = random.Random(4242)
    walks = gu.build_deepwalk_corpus(Nx1View(G), 2, 15, alpha=0.3, rand=rnd)
    out["karate_a03_walks"] = pad(walks, 15)
    out["karate_a03_state"] = np.array(rnd.getstate()[1], np.uint32)

    rng = np.random.RandomState(99)
    ids = rng.choice(np.arange(1, 5000), 60, replace=False)
    e = ids[rng.randint(0, 60, (300, 2))]
    e[::17, 1] = e[::17, 0]            # self-loops
    e = np.concatenate([e, e[::5], e[::7, ::-1]])  # duplicates, reversed duplicates
    rng.shuffle(e)
    Gm = nx.Graph()
    Gm.add_edges_from(e)
    record(out, "messy", Gm, e)
    rnd = random.Random(7)
    walks = gu.build_deepwalk_corpus(Nx1View(Gm), 3, 25, alpha=0.1, rand=rnd)
    out["messy_walks"] = pad(walks, 25)
    out["messy_state"] = np.array(rnd.getstate()[1], np.uint32)

    np.savez_compressed(os.path.join(HERE, "walks.npz"), **out)
    print("walks.npz:", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
