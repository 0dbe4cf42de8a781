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
    with open(path_join(path, "{}.txt".format(file_name)), 'w') as txt_file:
        for node, com in enumerate(community_color):
            txt_file.write('%d\t%d\n' % ((node + 1), com))


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
    ret = []
    with open(path_join(path, file_name + ext), 'r') as f:
        for line in f:
            tokens = line.strip().split('\t')
            ret.append([float(val) for val in tokens[1].strip().split(' ')])
    return np.array(ret, dtype=np.float32)
