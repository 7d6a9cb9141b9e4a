"""PyG-2.0.4-compatible graph layers (GCNConv, SAGEConv, GATConv, HeteroConv, Linear).

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
    """PyG Linear; in_channels <= 0 is lazy (shape taken from the first input or checkpoint)."""

    def __init__(self, in_channels, out_channels, bias=True, weight_initializer=None,
                 bias_initializer=None):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.weight_initializer, self.bias_initializer = weight_initializer, bias_initializer
        if in_channels > 0:
            self.weight = nn.Parameter(torch.empty(out_channels, in_channels))
        else:
            self.weight = nn.parameter.UninitializedParameter()
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        if in_channels > 0:
            self.reset_parameters()
        elif self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()

    def reset_parameters(self):
        fan_in = self.weight.shape[1]
        if self.weight_initializer == "glorot":
            _uniform_(self.weight, math.sqrt(6.0 / (fan_in + self.out_channels)))
        else:
            _uniform_(self.weight, 1.0 / math.sqrt(max(fan_in, 1)))
        if self.bias is not None:
            if self.bias_initializer == "zeros":
                with torch.no_grad():
                    self.bias.zero_()
            else:
                _uniform_(self.bias, 1.0 / math.sqrt(max(fan_in, 1)))

    def _materialize(self, in_channels, device, dtype):
        if isinstance(self.weight, nn.parameter.UninitializedParameter):
            self.weight.materialize((self.out_channels, in_channels), device=device, dtype=dtype)
            self.in_channels = in_channels
            self.reset_parameters()

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        w = state_dict.get(prefix + "weight")
        if w is not None:
            self._materialize(w.shape[1], w.device, w.dtype)
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)

    def forward(self, x):
        self._materialize(x.shape[-1], x.device, x.dtype)
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


class GATConv(MessagePassing):
    """GATConv (PyG 2.0.4): h = x W (W_src / W_dst for bipartite inputs), attention
    softmax over each target's in-edges of leaky_relu(a_src . h_j + a_dst . h_i, 0.2), heads
    concatenated (or averaged), + bias.  The conv of the reference's multi-node-type test arch
    (tests/test_utils.py:86-182: HeteroConv of GATConv((-1, -1), c, add_self_loops=False)).
    The engine does not compile it: archs using it run on the generic (batched) path."""

    def __init__(self, in_channels, out_channels, heads=1, concat=True, negative_slope=0.2,
                 dropout=0.0, add_self_loops=True, bias=True, **kwargs):
        super().__init__()
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, heads
        self.concat, self.negative_slope, self.dropout = concat, negative_slope, dropout
        self.add_self_loops = add_self_loops
        if isinstance(in_channels, int):
            self.lin_src = Linear(in_channels, heads * out_channels, bias=False,
                                  weight_initializer="glorot")
            self.lin_dst = self.lin_src
        else:
            self.lin_src = Linear(in_channels[0], heads * out_channels, bias=False,
                                  weight_initializer="glorot")
            self.lin_dst = Linear(in_channels[1], heads * out_channels, bias=False,
                                  weight_initializer="glorot")
        self.att_src = nn.Parameter(torch.empty(1, heads, out_channels))
        self.att_dst = nn.Parameter(torch.empty(1, heads, out_channels))
        _uniform_(self.att_src, math.sqrt(6.0 / (heads + out_channels)))
        _uniform_(self.att_dst, math.sqrt(6.0 / (heads + out_channels)))
        n_bias = heads * out_channels if concat else out_channels
        self.bias = nn.Parameter(torch.zeros(n_bias)) if bias else None

    def forward(self, x, edge_index):
        H, C = self.heads, self.out_channels
        # gat_conv.py (2.0.4): a Tensor input is transformed by lin_src for BOTH ends, also when a
        # separate lin_dst exists (tuple in_channels: HeteroConv hands same-type relations a
        # Tensor); a tuple input by lin_src / lin_dst
        if isinstance(x, torch.Tensor):
            hs = hd = self.lin_src(x).view(-1, H, C)
        else:
            hs = self.lin_src(x[0]).view(-1, H, C)
            hd = self.lin_dst(x[1]).view(-1, H, C)
        a_s = (hs * self.att_src).sum(-1)
        a_d = (hd * self.att_dst).sum(-1)
        ei = edge_index.long()
        n = hd.size(0)
        if self.add_self_loops:
            loop = torch.arange(min(hs.size(0), n), device=ei.device)
            ei = torch.cat([ei[:, ei[0] != ei[1]], torch.stack([loop, loop])], 1)
        src, dst = ei[0], ei[1]
        alpha = F.leaky_relu(a_s[src] + a_d[dst], self.negative_slope)          # [E, H]
        idx = dst.unsqueeze(1).expand(-1, H)
        amax = torch.zeros((n, H), dtype=alpha.dtype, device=alpha.device).scatter_reduce(
            0, idx, alpha, reduce="amax", include_self=False)
        ex = (alpha - amax[dst]).exp()
        den = torch.zeros((n, H), dtype=alpha.dtype, device=alpha.device).index_add_(0, dst, ex)
        alpha = ex / (den[dst] + 1e-16)
        alpha = F.dropout(alpha, p=self.dropout, training=self.training)
        out = torch.zeros((n, H, C), dtype=hs.dtype, device=hs.device)
        out.index_add_(0, dst, hs[src] * alpha.unsqueeze(-1))
        out = out.reshape(n, H * C) if self.concat else out.mean(dim=1)
        if self.bias is not None:
            out = out + self.bias
        return out

    def extra_repr(self):
        return f"{self.in_channels}, {self.out_channels}, heads={self.heads}"


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


class HeteroSageStack(nn.Module):
    """Multi-node-type model family: [HeteroConv({(src, rel, dst): SAGEConv}) -> ReLU]* then
    Linear layers on the first output node type — the layout of the reference's multi-type
    test arch (tests/test_utils.py:86-182) with SAGEConv relations (bipartite layer-1 inputs
    (F_src, F_dst)).  state_dict keys: conv.<2l>.convs.<src>__<rel>__<dst>.lin_l/lin_r.*,
    fc.<2i>.weight/bias."""

    def __init__(self, rels, in_dims, hidden, n_layers, fc_dims):
        super().__init__()
        convs = []
        for li in range(n_layers):
            convs.append(HeteroConv({tuple(r): SAGEConv((in_dims[r[0]], in_dims[r[-1]])
                                                        if li == 0 else (hidden, hidden), hidden)
                                     for r in rels}))
            convs.append(nn.ReLU())
        self.conv = nn.ModuleList(convs)
        fcs = []
        for i in range(len(fc_dims) - 1):
            fcs.append(Linear(fc_dims[i], fc_dims[i + 1]))
            fcs.append(nn.Sigmoid() if i == len(fc_dims) - 2 else nn.ReLU())
        self.fc = nn.ModuleList(fcs)

    def forward(self, x, edge_index):
        for i, c in enumerate(self.conv):
            x = c(x, edge_index) if i % 2 == 0 else {k: c(v) for k, v in x.items()}
        x = x[list(x.keys())[0]]
        for layer in self.fc:
            x = layer(x)
        return x


class HeteroGATStack(nn.Module):
    """Multi-node-type model family of the reference's own multi-type test arch
    (tests/test_utils.py:86-182: HeteroConv({(src, rel, dst): GATConv((-1, -1), c,
    add_self_loops=False)}, aggr="sum") -> ReLU, then Linear layers on the first output node
    type), with explicit input widths per layer and `heads` per layer (concatenated).  The
    engine does not compile GAT: it runs on the generic (batched) torch path.  state_dict keys:
    conv.<2l>.convs.<src>__<rel>__<dst>.{lin_src,lin_dst}.weight / att_src / att_dst / bias."""

    def __init__(self, rels, in_dims, hidden, heads, fc_dims, add_self_loops=False):
        super().__init__()
        convs, width = [], None
        for li, h in enumerate(heads):
            convs.append(HeteroConv({tuple(r): GATConv((in_dims[r[0]], in_dims[r[-1]]) if li == 0
                                                       else (width, width), hidden, heads=h,
                                                       add_self_loops=add_self_loops)
                                     for r in rels}))
            convs.append(nn.ReLU())
            width = hidden * h
        self.conv = nn.ModuleList(convs)
        fcs = []
        for i in range(len(fc_dims) - 1):
            fcs.append(Linear(fc_dims[i], fc_dims[i + 1]))
            fcs.append(nn.Sigmoid() if i == len(fc_dims) - 2 else nn.ReLU())
        self.fc = nn.ModuleList(fcs)

    def forward(self, x, edge_index):
        for i, c in enumerate(self.conv):
            x = c(x, edge_index) if i % 2 == 0 else {k: c(v) for k, v in x.items()}
        x = x[list(x.keys())[0]]
        for layer in self.fc:
            x = layer(x)
        return x


class LinkModel(nn.Module):
    """Edge-level model for edge problems: a node encoder (e.g. ConvStack with
    final_act="identity") and a dot-product link decoder, score(u, v) = act(<z_u, z_v>).

    forward(x, edge_index, edge_label_index=None) runs the encoder's message passing over
    `edge_index` and scores the edges of `edge_label_index` (default: every edge of
    `edge_index`) — the per-edge output the reference's edge problem extracts
    (model.py:295-328).  Scoring a separate label index keeps the query edge's output defined
    when Data.perturb_edge (data.py:500-554) removes that edge from the message passing."""

    def __init__(self, encoder, act="sigmoid"):
        super().__init__()
        if act not in ("sigmoid", "identity", None):
            raise ValueError("LinkModel act must be 'sigmoid' or 'identity'")
        self.encoder = encoder
        self.act = act or "identity"

    def forward(self, x, edge_index, edge_label_index=None):
        z = self.encoder(x, edge_index)
        eli = edge_index if edge_label_index is None else edge_label_index
        s = (z[eli[0]] * z[eli[1]]).sum(-1, keepdim=True)
        return torch.sigmoid(s) if self.act == "sigmoid" else s
