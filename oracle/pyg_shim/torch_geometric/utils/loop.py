"""add_remaining_self_loops restated from PyG 2.0.4 (shim; test infra only).

Every existing self-loop (row == col) is dropped and exactly one loop per node is appended
(weight `fill_value`, or the weight an existing loop carried).
"""
import torch


def add_remaining_self_loops(edge_index, edge_attr=None, fill_value=None, num_nodes=None):
    N = num_nodes if num_nodes is not None else int(edge_index.max()) + 1
    row, col = edge_index[0], edge_index[1]
    mask = row != col
    loop_index = torch.arange(0, N, dtype=row.dtype, device=row.device)
    loop_index = loop_index.unsqueeze(0).repeat(2, 1)
    edge_index = torch.cat([edge_index[:, mask], loop_index], dim=1)
    if edge_attr is not None:
        if fill_value is None:
            fill_value = 1.0
        loop_attr = edge_attr.new_full((N,) + edge_attr.size()[1:], fill_value)
        inv_mask = ~mask
        loop_attr[row[inv_mask]] = edge_attr[inv_mask]
        edge_attr = torch.cat([edge_attr[mask], loop_attr], dim=0)
    return edge_index, edge_attr
