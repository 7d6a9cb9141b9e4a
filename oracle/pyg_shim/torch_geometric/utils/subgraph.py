"""k_hop_subgraph / get_num_hops restated from PyG 2.0.4 semantics (shim; test infra only).

k_hop_subgraph(node_idx, num_hops, edge_index, relabel_nodes, flow='source_to_target'):
walks *incoming* edges (edge_index[0] -> edge_index[1]) backwards from the seed, num_hops
times; the returned `subset` is the sorted unique union of visited nodes; the returned edge
mask keeps every edge whose two endpoints are both in `subset` (original edge order kept);
`inv` is the position of the seed inside `subset`.
Call site in the reference: data.py:331-333 (with num_hops = model hops + 1, data.py:328).

get_num_hops(model): number of MessagePassing sub-modules (model.py:52).
"""
import torch


def get_num_hops(model):
    from ..nn.conv import MessagePassing

    return sum(1 for m in model.modules() if isinstance(m, MessagePassing))


def k_hop_subgraph(node_idx, num_hops, edge_index, relabel_nodes=False, num_nodes=None,
                   flow="source_to_target"):
    if num_nodes is None:
        num_nodes = int(edge_index.max()) + 1 if edge_index.numel() > 0 else 0
    if flow == "target_to_source":
        row, col = edge_index[0], edge_index[1]
    else:
        col, row = edge_index[0], edge_index[1]

    node_mask = torch.zeros(num_nodes, dtype=torch.bool, device=row.device)
    if isinstance(node_idx, (int, list, tuple)):
        node_idx = torch.tensor([node_idx], device=row.device).flatten()
    else:
        node_idx = node_idx.to(row.device)

    subsets = [node_idx]
    for _ in range(num_hops):
        node_mask.fill_(False)
        node_mask[subsets[-1]] = True
        edge_mask = node_mask[row]
        subsets.append(col[edge_mask])

    subset, inv = torch.cat(subsets).unique(return_inverse=True)
    inv = inv[: node_idx.numel()]

    node_mask.fill_(False)
    node_mask[subset] = True
    edge_mask = node_mask[row] & node_mask[col]
    edge_index = edge_index[:, edge_mask]

    if relabel_nodes:
        mapping = torch.full((num_nodes,), -1, dtype=row.dtype, device=row.device)
        mapping[subset] = torch.arange(subset.size(0), device=row.device)
        edge_index = mapping[edge_index]

    return subset, edge_index, inv, edge_mask
