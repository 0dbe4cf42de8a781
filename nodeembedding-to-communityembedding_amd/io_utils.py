"""Label / embedding text formats of the reference ``utils/IO_utils.py``.

``load_ground_true`` (:18-47), ``save_ground_true`` (:8-16), ``save_embedding`` (:49-62, one line
per node: ``<node_id>\\t<v1> <v2> ...`` with 1-based ids; native writer, byte-identical to the
reference's str(np.float32) output), ``load_embedding`` (:64-80).  The
reference's pickle ``save``/``load`` (:82-105) are not reproduced (unsafe; Model.save replaces
them).
"""
from os import makedirs
from os.path import dirname, join as path_join

import numpy as np


def save_ground_true(file_name, community_color, path="./data"):
    """IO_utils.save_ground_true (:8-16): "<node id>\t<label>" per line, ids from 1."""
    labels = np.asarray(community_color, np.int64).reshape(-1)
    lines = ["%d\t%d\n" % (i, c) for i, c in zip(range(1, len(labels) + 1), labels.tolist())]
    with open(path_join(path, file_name + ".txt"), "w") as f:
        f.writelines(lines)


def load_ground_true(path='data/', file_name=None, multilabel=False):
    """(labels sorted by node id, number of communities = max label)."""
    labels = {}
    mx = 0
    with open(path_join(path, file_name + '.labels'), 'r') as f:
        for line in f:
            tokens = line.strip().split('\t')
            node_id, label_id = int(tokens[0]), int(tokens[1])
            mx = max(mx, label_id)
            labels.setdefault(node_id, []).append(label_id)
    ret = [labels[k] if multilabel else labels[k][0] for k in sorted(labels)]
    return ret, mx


def _to_numpy(embeddings):
    if hasattr(embeddings, "detach"):
        return embeddings.detach().cpu().numpy()
    return np.asarray(embeddings)


def save_embedding(embeddings, file_name, path='data'):
    """IO_utils.save_embedding (:49-62), written natively (come_save_embedding): the same bytes
    as the reference's str(np.float32) per value, for fp32 tables (host or device)."""
    from . import _lib
    full_path = path_join(path, file_name + '.txt')
    makedirs(dirname(full_path), exist_ok=True)
    emb = np.ascontiguousarray(_to_numpy(embeddings), dtype=np.float32)
    if emb.ndim != 2:
        raise ValueError("embeddings must be 2-D")
    _lib.check(_lib.lib().come_save_embedding(full_path.encode(), _lib.ptr(emb), emb.shape[0],
                                              emb.shape[1], 1), "come_save_embedding")


def load_embedding(file_name, path='data', ext=".txt"):
    """IO_utils.load_embedding (:64-80): the vectors of a save_embedding file, in file order,
    as float32 [V, d] (the id column is not used, as in the reference)."""
    with open(path_join(path, file_name + ext)) as f:
        vecs = [line.partition("\t")[2].split() for line in f if line.strip()]
    return np.array(vecs, dtype=np.float64).astype(np.float32)
