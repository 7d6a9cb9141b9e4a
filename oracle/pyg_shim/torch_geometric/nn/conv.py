"""GCNConv / SAGEConv / HeteroConv restated from PyG 2.0.4 semantics (shim; test infra only).

GCNConv (normalize=True, add_self_loops=True, improved=False, cached=False):
    gcn_norm: add_remaining_self_loops(fill=1) on the given graph, deg = scatter_add(w, col),
    norm_e = deg^-1/2[row] * w_e * deg^-1/2[col] (inf -> 0);
    out = scatter_add(norm_e * (x W^T)[row], col) + bias.     (lin before propagate, bias after)
SAGEConv (aggr='mean', root_weight=True, normalize=False):
    out = lin_l(scatter_mean(x[row], col)) + lin_r(x)          (lin_r has no bias)
GATConv: see the class docstring.
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
    """GATConv (PyG 2.0.4 gat_conv.py) restated: lin_src (= lin_dst for an int in_channels;
    separate lin_dst for a tuple, both bias-free, glorot), att_src / att_dst [1, H, C] (glorot),
    bias [H*C] (concat) or [C] (zeros).  forward: a Tensor input is transformed by lin_src for
    BOTH ends (even when a separate lin_dst exists); a tuple by lin_src / lin_dst.  alpha_src =
    (x_src * att_src).sum(-1), alpha_dst likewise; add_self_loops: remove_self_loops then one
    loop per node of min(|src|, |dst|); message alpha_j + alpha_i -> leaky_relu(0.2) -> softmax
    over each target's in-edges (torch_geometric.utils.softmax: minus the per-target max, exp,
    / (sum + 1e-16)) -> dropout (eval: none) -> x_j * alpha; sum per target; concat heads
    (or mean) + bias.  Lazy in_channels (-1) materialise at the first forward."""

    def __init__(self, in_channels, out_channels, heads=1, concat=True, negative_slope=0.2,
                 dropout=0.0, add_self_loops=True, bias=True, **kwargs):
        super().__init__()
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, heads
        self.concat, self.negative_slope, self.dropout = concat, negative_slope, dropout
        self.add_self_loops = add_self_loops
        self.tuple_in = not isinstance(in_channels, int)
        ins = in_channels if self.tuple_in else (in_channels, in_channels)
        self._lazy = ins
        self.lin_src = Linear(ins[0], heads * out_channels, bias=False, weight_initializer="glorot") \
            if ins[0] > 0 else None
        self.lin_dst = (Linear(ins[1], heads * out_channels, bias=False, weight_initializer="glorot")
                        if ins[1] > 0 else None) if self.tuple_in else self.lin_src
        self.att_src = nn.Parameter(torch.empty(1, heads, out_channels))
        self.att_dst = nn.Parameter(torch.empty(1, heads, out_channels))
        bound = (6.0 / (heads + out_channels)) ** 0.5
        with torch.no_grad():
            self.att_src.uniform_(-bound, bound)
            self.att_dst.uniform_(-bound, bound)
        self.bias = nn.Parameter(torch.zeros(heads * out_channels if concat else out_channels)) \
            if bias else None

    def _materialize(self, xs, xd):
        if self.lin_src is None:
            self.lin_src = Linear(xs.size(1), self.heads * self.out_channels, bias=False,
                                  weight_initializer="glorot")
            if not self.tuple_in:
                self.lin_dst = self.lin_src
        if self.tuple_in and self.lin_dst is None and xd is not None:
            self.lin_dst = Linear(xd.size(1), self.heads * self.out_channels, bias=False,
                                  weight_initializer="glorot")

    def forward(self, x, edge_index):
        H, C = self.heads, self.out_channels
        if isinstance(x, torch.Tensor):
            self._materialize(x, None)
            x_src = x_dst = self.lin_src(x).view(-1, H, C)
        else:
            xs, xd = x
            self._materialize(xs, xd)
            x_src = self.lin_src(xs).view(-1, H, C)
            x_dst = self.lin_dst(xd).view(-1, H, C) if xd is not None else None
        a_src = (x_src * self.att_src).sum(-1)
        a_dst = (x_dst * self.att_dst).sum(-1) if x_dst is not None else None
        ei = edge_index.long()
        n_dst = x_dst.size(0) if x_dst is not None else x_src.size(0)
        if self.add_self_loops:
            n = min(x_src.size(0), n_dst)
            ei = ei[:, ei[0] != ei[1]]
            loop = torch.arange(n, device=ei.device)
            ei = torch.cat([ei, torch.stack([loop, loop])], 1)
        src, dst = ei[0], ei[1]
        alpha = a_src[src] if a_dst is None else a_src[src] + a_dst[dst]
        alpha = torch.nn.functional.leaky_relu(alpha, self.negative_slope)
        amax = torch.full((n_dst, H), float("-inf"), dtype=alpha.dtype)
        amax = amax.scatter_reduce(0, dst.view(-1, 1).expand(-1, H), alpha, reduce="amax")
        ex = (alpha - amax[dst]).exp()
        den = torch.zeros((n_dst, H), dtype=alpha.dtype).index_add_(0, dst, ex)
        alpha = ex / (den[dst] + 1e-16)
        out = torch.zeros((n_dst, H, C), dtype=x_src.dtype).index_add_(0, dst,
                                                                       x_src[src] * alpha.unsqueeze(-1))
        out = out.reshape(n_dst, H * C) if self.concat else out.mean(dim=1)
        if self.bias is not None:
            out = out + self.bias
        return out

    def __repr__(self):
        return f"GATConv({self.in_channels}, {self.out_channels}, heads={self.heads})"


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
