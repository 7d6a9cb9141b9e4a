"""Compile a black-box GNN `arch` (nn.Module) into the engine's layer program.

The reference treats `arch` as a black box and calls `arch(feat, edge_index)` on the B-fold
union graph (model.py:62-116).  The engine instead recognises the supported module family —
GCNConv / SAGEConv (mean) / HeteroConv(sum) conv layers, each optionally followed by an
elementwise activation, then Linear layers with activations (the layout of
tests/test_utils.py:10-83 and the notebooks) — and lowers it to:

    ConvLayer(terms=[(kind, relation, W_k)], bias_sum, act)   per conv layer
    HeadLayer(W, b, act)                                       per Linear

Multi-node-type graphs (HeteroConv over relations (src, rel, dst) between several node types,
model.py:118-253): every term carries its relation's destination type (the engine applies it
only to targets of that type), SAGE root weights and biases are summed per destination type,
and layer-1 weights are zero-padded to the widest input (the homogenised features are padded the
same way, data.py:825-878).  The head reads the first output node type of the last HeteroConv
(the `x[list(x.keys())[0]]` convention of the reference's hetero archs, tests/test_utils.py:176-178).

Modules are matched by class name + attributes, so both torch_geometric 2.0.4 modules and
bikg_graph_explainability_public_amd.nn modules compile.  Anything else raises
UnsupportedArch (callers then use the generic torch path, model.py).
"""
from dataclasses import dataclass, field
from typing import List, Optional

import torch
from torch import nn


class UnsupportedArch(ValueError):
    pass


@dataclass
class Term:
    kind: str          # "gcn" | "mean" | "root"
    rel: int           # relation index (ignored for root)
    weight: torch.Tensor  # [f_out, f_in]
    dst_type: int = -1    # multi-node-type: destination node type of the relation


@dataclass
class ConvLayer:
    terms: List[Term]
    bias: torch.Tensor    # [f_out] (sum over relations); multi-node-type: [n_types, f_out]
    act: Optional[str]
    f_in: int
    f_out: int


@dataclass
class HeadLayer:
    weight: torch.Tensor  # [n, k]
    bias: Optional[torch.Tensor]
    act: Optional[str]


@dataclass
class ModelProgram:
    convs: List[ConvLayer] = field(default_factory=list)
    head: List[HeadLayer] = field(default_factory=list)
    out_col: int = 0
    n_types: int = 1               # > 1: multi-node-type program (node-type-gated terms)
    out_type: Optional[int] = None  # multi-node-type: node type whose rows feed the head
    link_act: Optional[str] = None  # LinkModel: the program is its encoder; decoder act(<z_u, z_v>)

    @property
    def hops(self):
        return len(self.convs)


_ACTS = {"ReLU": "relu", "Sigmoid": "sigmoid", "Tanh": "tanh", "ELU": "elu",
         "LeakyReLU": "leaky_relu"}
_SKIP = {"Dropout", "Identity", "AlphaDropout"}


def _act_name(m):
    name = type(m).__name__
    if name not in _ACTS:
        return None
    if name == "LeakyReLU" and abs(getattr(m, "negative_slope", 0.01) - 0.01) > 0:
        raise UnsupportedArch("LeakyReLU(negative_slope != 0.01)")
    if name == "ELU" and getattr(m, "alpha", 1.0) != 1.0:
        raise UnsupportedArch("ELU(alpha != 1)")
    return _ACTS[name]


def _is_conv(m):
    return type(m).__name__ in ("GCNConv", "SAGEConv", "HeteroConv")


def _is_linear(m):
    return type(m).__name__ == "Linear" and hasattr(m, "weight")


def _leaf_units(module):
    """Registration-order walk yielding conv / linear / activation units (convs not entered)."""
    for child in module.children():
        if _is_conv(child) or _is_linear(child) or _act_name(child) is not None:
            yield child
        elif type(child).__name__ in _SKIP:
            continue
        elif len(list(child.children())) == 0:
            if any(True for _ in child.parameters(recurse=False)):
                raise UnsupportedArch(f"unsupported parameterised module {type(child).__name__}")
            continue
        else:
            yield from _leaf_units(child)


def _f32(t):
    return t.detach().to(torch.float32)


def _single_conv_terms(conv, rel):
    name = type(conv).__name__
    if name == "GCNConv":
        if getattr(conv, "improved", False) or not getattr(conv, "add_self_loops", True) \
                or not getattr(conv, "normalize", True):
            raise UnsupportedArch("GCNConv with improved/add_self_loops=False/normalize=False")
        W = _f32(conv.lin.weight)
        if getattr(conv.lin, "bias", None) is not None:
            raise UnsupportedArch("GCNConv.lin with bias")
        b = _f32(conv.bias) if getattr(conv, "bias", None) is not None else None
        return [Term("gcn", rel, W)], b, None, W.shape[1], W.shape[0]
    if name == "SAGEConv":
        aggr = getattr(conv, "aggr", "mean")
        if isinstance(aggr, str) and aggr != "mean" or getattr(conv, "normalize", False) \
                or not getattr(conv, "root_weight", True) or getattr(conv, "project", False):
            raise UnsupportedArch("SAGEConv other than aggr='mean', root_weight, no normalize")
        Wl = _f32(conv.lin_l.weight)
        bl = _f32(conv.lin_l.bias) if getattr(conv.lin_l, "bias", None) is not None else None
        Wr = _f32(conv.lin_r.weight)
        return [Term("mean", rel, Wl)], bl, Wr, Wl.shape[1], Wl.shape[0]
    raise UnsupportedArch(f"unsupported conv {name}")


def _conv_layer(conv, rel_index):
    """Lower one conv (or HeteroConv) to terms.  rel_index maps edge-type tuples to relations."""
    if type(conv).__name__ == "HeteroConv":
        if getattr(conv, "aggr", "sum") != "sum":
            raise UnsupportedArch("HeteroConv(aggr != 'sum')")
        if rel_index is None:
            raise UnsupportedArch("HeteroConv on a homogeneous graph")
        terms, bias, root = [], None, None
        f_in = f_out = None
        for key, sub in conv.convs.items():
            et = tuple(key.split("__"))
            if et not in rel_index:
                continue  # relation absent from the graph: HeteroConv skips it too
            if et[0] != et[-1]:
                raise UnsupportedArch("bipartite relations need the multi-node-type path")
            t, b, wr, fi, fo = _single_conv_terms(sub, rel_index[et])
            terms += t
            if b is not None:
                bias = b.clone() if bias is None else bias + b
            if wr is not None:
                root = wr.clone() if root is None else root + wr
            f_in, f_out = fi, fo
        if not terms:
            raise UnsupportedArch("HeteroConv with no relation present in the graph")
    else:
        if rel_index is not None and len(rel_index) != 1:
            raise UnsupportedArch("homogeneous conv on a multi-relation graph")
        terms, bias, root, f_in, f_out = _single_conv_terms(conv, 0)
    if root is not None:
        terms.append(Term("root", -1, root))
    if bias is None:
        bias = torch.zeros(f_out)
    return terms, bias, f_in, f_out


def _pad_cols(w, n):
    return w if w.shape[1] == n else torch.nn.functional.pad(w, (0, n - w.shape[1]))


def _conv_layer_multi(conv, rel_index, node_type_names):
    """HeteroConv over several node types: terms gated by destination type, SAGE root weights
    and biases summed per destination type.  Returns (terms, bias [n_types, f_out], f_in, f_out,
    destination type of the first present relation)."""
    if type(conv).__name__ != "HeteroConv" or getattr(conv, "aggr", "sum") != "sum":
        raise UnsupportedArch("multi-node-type graphs need HeteroConv(aggr='sum') layers")
    nt = len(node_type_names)
    terms, roots, biases = [], {}, {}
    f_out, first_dst, f_ins = None, None, []
    for key, sub in conv.convs.items():
        et = tuple(key.split("__"))
        if et not in rel_index:
            continue
        s_t, d_t = node_type_names.index(et[0]), node_type_names.index(et[-1])
        if type(sub).__name__ == "GCNConv" and s_t != d_t:
            raise UnsupportedArch("GCNConv on a bipartite relation")
        t, b, wr, fi, fo = _single_conv_terms(sub, rel_index[et])
        if f_out is not None and fo != f_out:
            raise UnsupportedArch("HeteroConv relations with different output widths")
        f_out = fo
        first_dst = d_t if first_dst is None else first_dst
        for term in t:
            term.dst_type = d_t
            f_ins.append(term.weight.shape[1])
        terms += t
        if b is not None:
            biases[d_t] = b.clone() if d_t not in biases else biases[d_t] + b
        if wr is not None:
            f_ins.append(wr.shape[1])
            if d_t in roots and roots[d_t].shape != wr.shape:
                raise UnsupportedArch("root weights of one destination type differ in shape")
            roots[d_t] = wr.clone() if d_t not in roots else roots[d_t] + wr
    if not terms:
        raise UnsupportedArch("HeteroConv with no relation present in the graph")
    # HeteroConv's output dict is keyed in edge_index_dict order (the graph's relation order)
    for et in rel_index:
        if "__".join(et) in conv.convs:
            first_dst = node_type_names.index(et[-1])
            break
    for d_t in sorted(roots):
        terms.append(Term("root", -1, roots[d_t], d_t))
    f_in = max(f_ins)
    for term in terms:
        term.weight = _pad_cols(term.weight, f_in)
    bias = torch.zeros(nt, f_out)
    for d_t, b in biases.items():
        bias[d_t] = b
    return terms, bias, f_in, f_out, first_dst


def compile_arch(arch: nn.Module, edge_type_names=None, node_type_names=None) -> ModelProgram:
    """Lower `arch` to a ModelProgram.  `edge_type_names` (list of (src, rel, dst) tuples in
    homogenised edge-type order, data.py:743-822) enables HeteroConv relations;
    `node_type_names` with two or more types selects the multi-node-type lowering."""
    if type(arch).__name__ == "LinkModel" and hasattr(arch, "encoder"):
        prog = compile_arch(arch.encoder, edge_type_names, node_type_names)
        prog.link_act = getattr(arch, "act", "identity") or "identity"
        return prog
    rel_index = None
    if edge_type_names is not None:
        rel_index = {tuple(et): i for i, et in enumerate(edge_type_names)}
    multi = node_type_names is not None and len(node_type_names) >= 2
    if multi and rel_index is None:
        raise UnsupportedArch("multi-node-type graphs need edge types")
    units = list(_leaf_units(arch))
    prog = ModelProgram()
    if multi:
        prog.n_types = len(node_type_names)
    i = 0
    while i < len(units) and _is_conv(units[i]):
        if multi:
            terms, bias, f_in, f_out, prog.out_type = _conv_layer_multi(units[i], rel_index,
                                                                        list(node_type_names))
        else:
            terms, bias, f_in, f_out = _conv_layer(units[i], rel_index)
        act = None
        if i + 1 < len(units) and _act_name(units[i + 1]) is not None:
            act = _act_name(units[i + 1])
            i += 1
        prog.convs.append(ConvLayer(terms, bias, act, f_in, f_out))
        i += 1
    if not prog.convs:
        raise UnsupportedArch("arch has no GCNConv/SAGEConv/HeteroConv layer first")
    while i < len(units) and _is_linear(units[i]):
        lin = units[i]
        act = None
        if i + 1 < len(units) and _act_name(units[i + 1]) is not None:
            act = _act_name(units[i + 1])
            i += 1
        b = _f32(lin.bias) if getattr(lin, "bias", None) is not None else None
        prog.head.append(HeadLayer(_f32(lin.weight), b, act))
        i += 1
    if i != len(units):
        raise UnsupportedArch(f"unexpected module order at {type(units[i]).__name__}")
    # width consistency
    prev = prog.convs[0].f_in
    for c in prog.convs:
        if c.f_in != prev:
            raise UnsupportedArch("conv widths do not chain")
        prev = c.f_out
    for h in prog.head:
        if h.weight.shape[1] != prev:
            raise UnsupportedArch("head widths do not chain")
        prev = h.weight.shape[0]
    return prog


def count_message_passing(arch: nn.Module) -> int:
    """PyG get_num_hops (model.py:52): number of MessagePassing modules."""
    n = 0
    for m in arch.modules():
        if any(c.__name__ == "MessagePassing" for c in type(m).__mro__):
            n += 1
        elif type(m).__name__ in ("GCNConv", "SAGEConv", "GATConv", "GINConv", "GraphConv"):
            n += 1
    return n
