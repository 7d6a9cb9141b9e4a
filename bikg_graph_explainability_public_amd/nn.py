"""PyG-2.0.4-compatible graph layers (GCNConv, SAGEConv, HeteroConv, Linear).

PyTorch Geometric is not available on ROCm boxes here; these modules carry the same
`state_dict` keys as torch_geometric 2.0.4 (`lin.weight` / `bias` for GCNConv, `lin_l.*` /
`lin_r.weight` for SAGEConv, `convs.<src>__<rel>__<dst>.*` for HeteroConv, `weight` / `bias`
for Linear) so the reference checkpoints (test_data/*.pth.tar, tests/test_utils.py:10-83) load
unchanged.  Their torch `forward` is the semantics the HIP engine compiles (engine.py); the
engine recognises these classes and the real PyG classes by name and attributes.
"""
import math

import torch
from torch import nn
import torch.nn.functional as F


class MessagePassing(nn.Module):
    """Marker base class: `Model.get_hops` counts instances (PyG get_num_hops semantics)."""


def _uniform_(t, bound):
    with torch.no_grad():
        t.uniform_(-bound, bound)


class Linear(nn.Module):
    def __init__(self, in_channels, out_channels, bias=True, weight_initializer=None,
                 bias_initializer=None):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        if weight_initializer == "glorot":
            _uniform_(self.weight, math.sqrt(6.0 / (in_channels + out_channels)))
        else:
            _uniform_(self.weight, 1.0 / math.sqrt(max(in_channels, 1)))
        if self.bias is not None:
            if bias_initializer == "zeros":
                with torch.no_grad():
                    self.bias.zero_()
            else:
                _uniform_(self.bias, 1.0 / math.sqrt(max(in_channels, 1)))

    def forward(self, x):
        return F.linear(x, self.weight, self.bias)

    def extra_repr(self):
        return f"{self.in_channels}, {self.out_channels}, bias={self.bias is not None}"


class GCNConv(MessagePassing):
    """GCNConv(normalize=True, add_self_loops=True): D^-1/2 (A + I) D^-1/2 X W^T + b, where
    existing self-loops are replaced by one weight-1 loop per node."""

    def __init__(self, in_channels, out_channels, bias=True, improved=False, cached=False,
                 add_self_loops=True, normalize=True, **kwargs):
        super().__init__()
        if improved or not add_self_loops or not normalize:
            raise NotImplementedError("only GCNConv(improved=False, add_self_loops=True, "
                                      "normalize=True) is supported")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.improved, self.add_self_loops, self.normalize = improved, add_self_loops, normalize
        self.lin = Linear(in_channels, out_channels, bias=False, weight_initializer="glorot")
        self.bias = nn.Parameter(torch.zeros(out_channels)) if bias else None

    def forward(self, x, edge_index):
        n = x.size(0)
        ei = edge_index.long()
        keep = ei[0] != ei[1]
        src = torch.cat([ei[0][keep], torch.arange(n, device=x.device)])
        dst = torch.cat([ei[1][keep], torch.arange(n, device=x.device)])
        deg = torch.zeros(n, dtype=x.dtype, device=x.device)
        deg.index_add_(0, dst, torch.ones_like(dst, dtype=x.dtype))
        dis = deg.pow(-0.5)
        dis.masked_fill_(torch.isinf(dis), 0)
        xw = self.lin(x)
        out = torch.zeros_like(xw)
        out.index_add_(0, dst, (dis[src] * dis[dst]).unsqueeze(1) * xw[src])
        if self.bias is not None:
            out = out + self.bias
        return out

    def extra_repr(self):
        return f"{self.in_channels}, {self.out_channels}"


class SAGEConv(MessagePassing):
    """SAGEConv(aggr='mean', root_weight=True, normalize=False): lin_l(mean_j x_j) + lin_r(x)."""

    def __init__(self, in_channels, out_channels, bias=True, normalize=False, root_weight=True,
                 aggr="mean", **kwargs):
        super().__init__()
        if normalize or not root_weight or aggr != "mean":
            raise NotImplementedError("only SAGEConv(aggr='mean', root_weight=True, "
                                      "normalize=False) is supported")
        if isinstance(in_channels, int):
            in_channels = (in_channels, in_channels)
        self.in_channels, self.out_channels = in_channels, out_channels
        self.aggr, self.root_weight, self.normalize = aggr, root_weight, normalize
        self.lin_l = Linear(in_channels[0], out_channels, bias=bias)
        self.lin_r = Linear(in_channels[1], out_channels, bias=False)

    def forward(self, x, edge_index):
        xs, xd = (x, x) if isinstance(x, torch.Tensor) else x
        ei = edge_index.long()
        n = xd.size(0)
        s = torch.zeros(n, xs.size(1), dtype=xs.dtype, device=xs.device)
        s.index_add_(0, ei[1], xs[ei[0]])
        cnt = torch.zeros(n, dtype=xs.dtype, device=xs.device)
        cnt.index_add_(0, ei[1], torch.ones(ei.size(1), dtype=xs.dtype, device=xs.device))
        return self.lin_l(s / cnt.clamp(min=1).unsqueeze(1)) + self.lin_r(xd)

    def extra_repr(self):
        return f"{self.in_channels}, {self.out_channels}, aggr={self.aggr}"


class HeteroConv(nn.Module):
    """HeteroConv(convs, aggr='sum'): per edge type conv, outputs summed per destination type."""

    def __init__(self, convs, aggr="sum"):
        super().__init__()
        if aggr != "sum":
            raise NotImplementedError("only HeteroConv(aggr='sum') is supported")
        self.convs = nn.ModuleDict({"__".join(k): v for k, v in convs.items()})
        self.aggr = aggr

    def forward(self, x_dict, edge_index_dict):
        out = {}
        for et, ei in edge_index_dict.items():
            key = "__".join(et)
            if key not in self.convs:
                continue
            src, _, dst = et
            conv = self.convs[key]
            o = conv(x_dict[src], ei) if src == dst else conv((x_dict[src], x_dict[dst]), ei)
            out[dst] = o if dst not in out else out[dst] + o
        return out


class ConvStack(nn.Module):
    """Model family of the reference tests/notebooks (tests/test_utils.py:10-83,
    examples/toy_example-caseA.ipynb cell 9): `conv` = ModuleList[Conv, ReLU]*, `fc` =
    ModuleList[Linear, act]* ending in Sigmoid.  `kind` in {"gcn", "sage"}; `hetero_rels`
    wraps each conv in HeteroConv over the given edge types (single node type)."""

    def __init__(self, kind, dims, fc_dims, hetero_rels=None, final_act="sigmoid"):
        super().__init__()
        mk = GCNConv if kind == "gcn" else SAGEConv
        convs = []
        for i in range(len(dims) - 1):
            if hetero_rels is not None:
                convs.append(HeteroConv({tuple(r): mk(dims[i], dims[i + 1])
                                         for r in hetero_rels}))
            else:
                convs.append(mk(dims[i], dims[i + 1]))
            convs.append(nn.ReLU())
        self.conv = nn.ModuleList(convs)
        fcs = []
        for i in range(len(fc_dims) - 1):
            fcs.append(Linear(fc_dims[i], fc_dims[i + 1]))
            last = i == len(fc_dims) - 2
            fcs.append((nn.Sigmoid() if final_act == "sigmoid" else nn.Identity()) if last
                       else nn.ReLU())
        self.fc = nn.ModuleList(fcs)

    def forward(self, x, edge_index):
        for i, c in enumerate(self.conv):
            if i % 2 == 0:
                x = c(x, edge_index)
            elif isinstance(x, dict):
                x = {k: c(v) for k, v in x.items()}
            else:
                x = c(x)
        if isinstance(x, dict):
            x = x[list(x.keys())[0]]
        for layer in self.fc:
            x = layer(x)
        return x
