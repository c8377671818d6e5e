"""raincast_gnn -- MI355X-native (gfx950) GINEConv message-passing engine for the
station-graph precipitation GNN of SohirMaskey/raincast-gnn.

The drop-in is :class:`raincast_gnn.nn.GINEConv` (replaces ``torch_geometric.nn.GINEConv``
at models/gnn.py:5); :mod:`raincast_gnn.models` rebuilds models/gnn.py on top of it.
The compute path is the C-ABI library ``_native/libgine_hip.so`` (include/gine_hip.h).
"""
from . import _lib
from .graph import GineGraph, get_graph, graph_cache
from .nn import GINEConv

__all__ = ["GINEConv", "GineGraph", "get_graph", "graph_cache", "native_library"]


def native_library():
    """Load (if needed) and return the ctypes handle of libgine_hip.so; raises if missing."""
    return _lib.load()
