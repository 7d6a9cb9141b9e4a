"""GCNConv / SAGEConv / HeteroConv restated from PyG 2.0.4 semantics (shim; test infra only).

GCNConv (normalize=True, add_self_loops=True, improved=False, cached=False):
    gcn_norm: add_remaining_self_loops(fill=1) on the given graph, deg = scatter_add(w, col),
    norm_e = deg^-1/2[row] * w_e * deg^-1/2[col] (inf -> 0);
    out = scatter_add(norm_e * (x W^T)[row], col) + bias.     (lin before propagate, bias after)
SAGEConv (aggr='mean', root_weight=True, normalize=False):
    out = lin_l(scatter_mean(x[row], col)) + lin_r(x)          (lin_r has no bias)
HeteroConv(aggr='sum'): one conv per edge type keyed '__'.join(edge_type); outputs summed per
    destination node type in edge_index_dict order.
Messages flow edge_index[0] (source) -> edge_index[1] (target).
"""
import torch
from torch import nn

from ..utils.loop import add_remaining_self_loops
from .linear import Linear


class MessagePassing(nn.Module):
    """Marker base class (get_num_hops counts instances of it)."""


def gcn_norm(edge_index, num_nodes, dtype):
    w = torch.ones(edge_index.size(1), dtype=dtype, device=edge_index.device)
    edge_index, w = add_remaining_self_loops(edge_index, w, 1.0, num_nodes)
    row, col = edge_index[0], edge_index[1]
    deg = torch.zeros(num_nodes, dtype=dtype, device=w.device).index_add_(0, col, w)
    dis = deg.pow(-0.5)
    dis.masked_fill_(dis == float("inf"), 0)
    return edge_index, dis[row] * w * dis[col]


class GCNConv(MessagePassing):
    def __init__(self, in_channels, out_channels, bias=True, **kwargs):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.lin = Linear(in_channels, out_channels, bias=False, weight_initializer="glorot")
        if bias:
            self.bias = nn.Parameter(torch.zeros(out_channels))
        else:
            self.register_parameter("bias", None)

    def forward(self, x, edge_index):
        n = x.size(0)
        ei, norm = gcn_norm(edge_index.long(), n, x.dtype)
        xw = self.lin(x)
        out = torch.zeros(n, xw.size(1), dtype=xw.dtype, device=xw.device)
        out.index_add_(0, ei[1], norm.view(-1, 1) * xw[ei[0]])
        if self.bias is not None:
            out = out + self.bias
        return out

    def __repr__(self):
        return f"GCNConv({self.in_channels}, {self.out_channels})"


class SAGEConv(MessagePassing):
    def __init__(self, in_channels, out_channels, bias=True, **kwargs):
        super().__init__()
        if isinstance(in_channels, int):
            in_channels = (in_channels, in_channels)
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.lin_l = Linear(in_channels[0], out_channels, bias=bias)
        self.lin_r = Linear(in_channels[1], out_channels, bias=False)

    def forward(self, x, edge_index):
        if isinstance(x, torch.Tensor):
            x = (x, x)
        xs, xd = x
        ei = edge_index.long()
        n = xd.size(0)
        s = torch.zeros(n, xs.size(1), dtype=xs.dtype, device=xs.device)
        s.index_add_(0, ei[1], xs[ei[0]])
        cnt = torch.zeros(n, dtype=xs.dtype, device=xs.device)
        cnt.index_add_(0, ei[1], torch.ones(ei.size(1), dtype=xs.dtype, device=xs.device))
        mean = s / cnt.clamp(min=1).view(-1, 1)
        return self.lin_l(mean) + self.lin_r(xd)

    def __repr__(self):
        return f"SAGEConv({self.in_channels}, {self.out_channels})"


class GATConv(MessagePassing):
    def __init__(self, *args, **kwargs):
        super().__init__()

    def forward(self, *args, **kwargs):  # pragma: no cover - not restated
        raise NotImplementedError("GATConv is not restated by the PyG shim")


class HeteroConv(nn.Module):
    def __init__(self, convs, aggr="sum"):
        super().__init__()
        self.convs = nn.ModuleDict({"__".join(k): v for k, v in convs.items()})
        self.aggr = aggr

    def forward(self, x_dict, edge_index_dict):
        out = {}
        for edge_type, ei in edge_index_dict.items():
            key = "__".join(edge_type)
            if key not in self.convs:
                continue
            src, _, dst = edge_type
            conv = self.convs[key]
            if src == dst:
                o = conv(x_dict[src], ei)
            else:
                o = conv((x_dict[src], x_dict[dst]), ei)
            out.setdefault(dst, []).append(o)
        res = {}
        for k, v in out.items():
            if self.aggr == "sum":
                res[k] = torch.stack(v).sum(0)
            elif self.aggr == "mean":
                res[k] = torch.stack(v).mean(0)
            else:
                raise NotImplementedError(self.aggr)
        return res
