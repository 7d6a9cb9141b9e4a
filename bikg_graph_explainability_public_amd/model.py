"""Black-box model adapter: the reference's `Model` class (model.py:11-328).

`get_hops` counts message-passing layers (PyG get_num_hops semantics) divided by the relation
count for heterogeneous models (model.py:28-60).  `infer` runs the user's module in torch on a
(union) graph — it is the generic path for architectures the engine cannot compile
(program.compile_arch); supported architectures never go through it (engine.ForwardPlan).
"""
import inspect

import torch

from .data import Data
from .program import count_message_passing


class Model:
    def __init__(self, arch):
        self.arch = arch

    def get_hops(self, num_relations=0):
        """model.py:28-60."""
        hops = count_message_passing(self.arch)
        if num_relations > 0:
            hops //= num_relations
        return hops

    def infer(self, feat, edge_index, node_types=None, edge_types=None):
        """model.py:62-116 — call convention picked from the forward signature."""
        nargs = len(inspect.signature(self.arch.forward).parameters)
        with torch.no_grad():
            if nargs == 2:
                return self.arch(feat, edge_index)
            if nargs == 4 and node_types is not None and edge_types is not None:
                return self.arch(feat, edge_index, node_types, edge_types)
        raise TypeError("arch.forward must take (x, edge_index) or "
                        "(x, edge_index, node_types, edge_types)")

    def predict_hetero_output(self, feat, edge_index, node_types, edge_types, node_type_names,
                              edge_type_names, num_perturbs, num_nodes, sub_ind=None,
                              padded_dims=None, problem="node_prediction"):
        """model.py:118-253 — multi-node-type graphs: one forward per perturbation copy, edge
        indices re-based per node type; returns the query output per copy."""
        uniq = torch.unique(node_types)
        outs = []
        src_vals = edge_index[0, :]
        pointers = None
        for b in range(num_perturbs):
            idx = torch.arange(b * num_nodes, (b + 1) * num_nodes, device=feat.device)
            pf, pt = feat[idx], node_types[idx]
            sel = torch.where((src_vals >= b * num_nodes) & (src_vals < (b + 1) * num_nodes))[0]
            pei = edge_index[:, sel] - idx[0]
            pet = edge_types[sel]
            if pet.shape[0] == 0:
                outs.append(0)
                continue
            if pointers is None:
                pointers = [torch.where(node_types == u)[0][0] for u in uniq]
            dc = Data(pf, pei)
            fd = dc.homo2hetero(pf, pt, node_type_names, padded_dims)
            ed = dc.homo2hetero(pei, pet, edge_type_names)
            for et in edge_type_names:
                m = ed[et]
                m[0] -= pointers[node_type_names.index(et[0])]
                m[1] -= pointers[node_type_names.index(et[-1])]
                ed[et] = m
            with torch.no_grad():
                out = self.arch(fd, ed)
            if "node" in problem and sub_ind is not None:
                out = out[sub_ind, 0].item()
            outs.append(out)
        return torch.tensor(outs, device=feat.device)

    def predict_hetero_output_batched(self, feat, edge_index, node_types, edge_types,
                                      node_type_names, edge_type_names, num_perturbs, num_nodes,
                                      sub_ind=None, padded_dims=None, problem="node_prediction"):
        """predict_hetero_output (model.py:118-253) with ONE `arch` call instead of one per copy
        (SURVEY.md §8f2): the B copies become a disjoint union per node type — copy b's nodes of
        type t are rows [b*n_t, (b+1)*n_t) of x_dict[t], relation edges are re-based the same
        way — so every node-wise message-passing layer (GCN/SAGE/GAT, HeteroConv, Linear)
        computes exactly the per-copy outputs.  Copies without edges give 0 as in the reference.
        Returns None when the layout is not the contiguous per-type blocks the reference's
        pointer arithmetic assumes (callers then use the per-copy loop)."""
        if "node" not in problem or sub_ind is None:
            return None
        B, S = int(num_perturbs), int(num_nodes)
        dev = feat.device
        nt = node_types[:S]
        uniq = torch.unique(node_types)
        pointers = [int(torch.where(node_types == u)[0][0]) for u in uniq]
        f3 = feat.reshape(B, S, feat.shape[1])
        x_dict, n_of = {}, {}
        for i, name in enumerate(node_type_names):
            idx = torch.where(nt == i)[0]
            n_of[name] = int(idx.numel())
            if idx.numel() and int(idx[-1] - idx[0]) + 1 != idx.numel():
                return None  # type rows not one contiguous block
            block = f3[:, idx, :].reshape(B * idx.numel(), feat.shape[1])
            if padded_dims is not None and padded_dims[i] > 0:
                block = block[:, :-padded_dims[i]]
            x_dict[name] = block
        ei = edge_index.long()
        copy = torch.div(ei[0], S, rounding_mode="floor")
        e_dict = {}
        for k, et in enumerate(edge_type_names):
            sel = torch.where(edge_types == k)[0]
            b = copy[sel]
            out_e = []
            for row, tname in ((0, et[0]), (1, et[-1])):
                p = pointers[node_type_names.index(tname)]
                loc = ei[row, sel] - b * S - p
                if loc.numel() and (int(loc.min()) < 0 or int(loc.max()) >= n_of[tname]):
                    return None
                out_e.append(b * n_of[tname] + loc)
            e_dict[et] = torch.stack(out_e) if sel.numel() else \
                torch.zeros((2, 0), dtype=torch.long, device=dev)
        with torch.no_grad():
            out = self.arch(x_dict, e_dict)
        if out.shape[0] % B:
            return None
        y = out.reshape(B, out.shape[0] // B, -1)[:, sub_ind, 0]
        has_edges = torch.bincount(copy, minlength=B)[:B] > 0
        return torch.where(has_edges, y, torch.zeros_like(y))

    @staticmethod
    def hetero2homo_output(hetero_output):
        """model.py:256-292."""
        if isinstance(hetero_output, torch.Tensor):
            return hetero_output, None
        vals = list(hetero_output.values())
        types = torch.cat([torch.full((len(v),), i, dtype=torch.int, device=v.device)
                           for i, v in enumerate(vals)])
        return torch.cat(vals, dim=0), types

    @staticmethod
    def extract_node_edge_output(output, ind, n):
        """model.py:295-328 — output[ind::n]."""
        return output[torch.arange(ind, output.shape[0], n, device=output.device)]
