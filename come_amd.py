"""come_amd -- MI355X-native ComE hot path (SGNS O1/O2, community gradient, GMM responsibilities).

The package lives in the directory ``nodeembedding-to-communityembedding_amd/`` (a name Python
cannot import directly); this module makes it importable as ``come_amd`` by pointing the package
search path there.  Module map, mirroring the reference layout:

    come_amd.training_sdg_inner   <- utils/training_sdg_inner.pyx (train_o1, train_o2, init,
                                     FAST_VERSION) -- drop-in, backed by libcome.so (HIP, gfx950)
    come_amd.embedding            <- utils/embedding.py (Vocab; prepare_sentences as the
                                     vectorised walks_to_rows)
    come_amd.model                <- ADSCModel/model.py (Model)
    come_amd.node_embeddings      <- ADSCModel/node_embeddings.py (Node2Vec)
    come_amd.context_embeddings   <- ADSCModel/context_embeddings.py (Context2Vec)
    come_amd.community_embeddings <- ADSCModel/community_embeddings.py (Community2Vec)
    come_amd.io_utils             <- utils/IO_utils.py (labels / embedding text formats)
    come_amd.graph                <- synthetic graphs + random walks (inputs of the hot path)
    come_amd.distributed          <- (new) walk sharding + delta all-reduce over RCCL
"""
import os as _os

__path__ = [_os.path.join(_os.path.dirname(_os.path.abspath(__file__)),
                          "nodeembedding-to-communityembedding_amd")]
__version__ = "0.1.0"
