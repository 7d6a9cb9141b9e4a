"""Shim for torch_geometric.utils (PyG 2.0.4 semantics)."""
from .subgraph import k_hop_subgraph, get_num_hops  # noqa: F401
from .loop import add_remaining_self_loops  # noqa: F401
