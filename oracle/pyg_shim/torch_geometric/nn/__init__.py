"""Shim for torch_geometric.nn (PyG 2.0.4 semantics; test infra only)."""
from .conv import MessagePassing, GCNConv, SAGEConv, HeteroConv, GATConv  # noqa: F401
from .linear import Linear  # noqa: F401
