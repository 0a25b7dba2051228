"""MI355X-native MST engine — the GHS fragment-merging hot path of
Trisanu-007/Distributed_GHS_Implementation rebuilt as a level-synchronous Boruvka fragment
contraction in hand-written gfx950 HIP kernels (libghs_mst.so, C-ABI in include/ghs_mst.h).

Entry points mirroring the reference:
  GHSAlgorithm(num_nodes, edges).run()      ghs_implementation.py:416-490
  python -m distributed_ghs_implementation_amd --graph-dir D
                                            ghs_implementation_mpi.py:884-954 (CLI)
Array level: graph.canonicalize -> mst.minimum_spanning_forest; device level: device.DeviceMST;
multi-GPU: distributed.DistributedMST.
"""
from .graph import (CanonicalGraph, canonicalize, read_graph_dir, read_mstbin, write_graph_dir, write_mstbin,
                    write_result)
from .mst import GHSAlgorithm, MSTResult, minimum_spanning_forest

__all__ = [
    "CanonicalGraph", "canonicalize", "read_graph_dir", "read_mstbin", "write_graph_dir", "write_mstbin",
    "write_result", "GHSAlgorithm", "MSTResult", "minimum_spanning_forest",
]
