"""Graph data utilities: the reference's `Data` class (data.py:19-878), same names and outputs.

* Heterogeneous <-> homogeneous layout (data.py:39-232, 695-878) and names: host torch ops.
* `comp_graph` (data.py:281-361): PyG-2.0.4 k_hop_subgraph semantics (L+1 hops, relabel).  On a
  device graph (the Explainer.run path) it is the HIP frontier/compaction kernels
  (`engine.khop_subgraph`, §8f1); a host graph (Data used on CPU tensors) uses torch ops.
* Perturbation seams (`build_edge_mask`, `perturb_node`, `perturbator`, data.py:390-648): the
  edge keep test runs in the HIP kernel `xpg_edge_keep` on bit-packed masks (device tensors
  only; no CPU fallback).  The engine path never materialises the B-fold union graph at all.
"""
import itertools
import operator

import numpy as np
import torch
import torch.nn.functional as F

from . import engine
from .frames import sorted_frame


def k_hop_subgraph(node_idx, num_hops, edge_index, num_nodes=None):
    """PyG 2.0.4 k_hop_subgraph(flow='source_to_target', relabel_nodes=True): walk incoming
    edges num_hops times from the seed; subset = sorted unique visited nodes; keep every edge
    with both ends in subset (original order); relabel.  Returns (subset, edge_index, inv,
    edge_mask)."""
    if num_nodes is None:
        num_nodes = int(edge_index.max()) + 1 if edge_index.numel() else 1
    if edge_index.device.type == "cuda":
        return engine.khop_subgraph(int(node_idx), num_hops, edge_index, num_nodes)
    src, dst = edge_index[0], edge_index[1]
    dev = edge_index.device
    seed = torch.tensor([int(node_idx)], device=dev)
    visited = [seed]
    mark = torch.zeros(num_nodes, dtype=torch.bool, device=dev)
    for _ in range(num_hops):
        mark.fill_(False)
        mark[visited[-1]] = True
        visited.append(src[mark[dst]])
    subset, inv = torch.cat(visited).unique(return_inverse=True)
    mark.fill_(False)
    mark[subset] = True
    emask = mark[src] & mark[dst]
    remap = torch.full((num_nodes,), -1, dtype=torch.long, device=dev)
    remap[subset] = torch.arange(subset.numel(), device=dev)
    return subset, remap[edge_index[:, emask]], inv[:1], emask


def take_names(names, idx):
    """np.array(names, dtype=str)[idx].tolist() without converting every name: the selected
    names as numpy's str conversion gives them."""
    if not len(idx):
        return []
    ii = idx.tolist() if hasattr(idx, "tolist") else [int(i) for i in idx]  # one host copy
    picked = (names[ii[0]],) if len(ii) == 1 else operator.itemgetter(*ii)(names)
    if set(map(type, picked)) == {str} and "\x00" not in "".join(picked):
        return list(picked)  # str names: numpy's str conversion returns them unchanged
    return np.array(picked, dtype=str).tolist()


def pad_feat_tensors(feat_tensors):
    """data.py:825-878 — zero-pad feature widths to the maximum; returns (padded tensors,
    padding per type, start pointer per type)."""
    widths = [t.shape[1] for t in feat_tensors]
    wmax = max(widths)
    padded, pads, pointers, p = [], [], [], 0
    for t in feat_tensors:
        d = wmax - t.shape[1]
        pads.append(d)
        pointers.append(p)
        p += t.shape[0]
        padded.append(F.pad(t, (0, d)) if d > 0 else t)
    return padded, pads, pointers


class Data:
    def __init__(self, feat, edge_index):
        self.feat = feat
        self.edge_index = edge_index

    # -------------------------------------------------------------- hetero layout (host)
    def preprocess_hetero_graph(self):
        """data.py:39-93."""
        res = [None, None, self.feat, self.edge_index, None, None, None, None, None]
        if isinstance(self.edge_index, dict) and isinstance(self.feat, dict):
            ntypes, etypes = list(self.feat.keys()), list(self.edge_index.keys())
            fh, eh, nt, et, npt, ept, pads = self.hetero2homo()
            res = [ntypes, etypes, fh, eh, nt, et, npt, ept, pads]
        return tuple(res)

    def hetero2homo(self):
        """data.py:95-147."""
        feat, node_types, pads, node_ptrs = self.concatenate_hetero_features()
        ei, edge_types, edge_ptrs = self.concatenate_hetero_edge_indices(node_ptrs)
        return feat, ei, node_types, edge_types, node_ptrs, edge_ptrs, pads

    @staticmethod
    def homo2hetero(matrix, element_type, element_type_names, padded_dims=None):
        """data.py:150-232 — split a homogeneous matrix back into {type name: block}."""
        out = {}
        node_mode = isinstance(element_type_names[0], str)
        for i, name in enumerate(element_type_names):
            idx = torch.where(element_type == i)[0]
            if node_mode:
                block = matrix[idx]
                if padded_dims is not None and padded_dims[i] > 0:
                    block = block[:, :-padded_dims[i]]
                out[name] = block
            else:
                out[name] = matrix[:, idx].long()
        return out

    @staticmethod
    def hetero2homo_names(names):
        """data.py:235-279."""
        if not isinstance(names, dict):
            return names, None
        device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        lists = list(names.values())
        types = torch.cat([torch.full((len(v),), float(i), device=device)
                           for i, v in enumerate(lists)])
        return list(itertools.chain.from_iterable(lists)), types

    def concatenate_hetero_features(self):
        """data.py:695-741."""
        tensors = list(self.feat.values())
        padded, pads, pointers = pad_feat_tensors(tensors)
        dev = tensors[0].device
        types = torch.cat([torch.full((t.shape[0],), float(i), device=dev)
                           for i, t in enumerate(padded)])
        return torch.cat(padded, dim=0), types, pads, pointers

    def concatenate_hetero_edge_indices(self, node_pointers):
        """data.py:743-822 — offset each relation's endpoints by its node types' pointers."""
        ntypes = list(self.feat.keys())
        mapped, types, pointers, p = [], [], [], 0
        for i, (rel, ei) in enumerate(self.edge_index.items()):
            pointers.append(p)
            add = torch.tensor([[node_pointers[ntypes.index(rel[0])]],
                                [node_pointers[ntypes.index(rel[-1])]]], device=ei.device)
            mapped.append(ei + add)
            types.append(torch.full((ei.shape[-1],), float(i), device=ei.device))
            p += ei.shape[-1]
        return torch.cat(mapped, dim=1), torch.cat(types), pointers

    # -------------------------------------------------------------- computational graph
    def comp_graph(self, ind, n_hops, problem, names, node_types=None, edge_types=None,
                   return_pos=False):
        """data.py:281-361 — k-hop computational subgraph with one hop more than the model.
        `return_pos` appends the positions of `sub_names` in `names` (int64 numpy array)."""
        hops = n_hops + 1
        n = self.feat.shape[0]
        subset, sub_ei, sub_ind, emask = k_hop_subgraph(ind, hops, self.edge_index, n)
        if sub_ei.shape[1] == 0:  # no kept edge (sub_ei has one column per kept edge)
            sub_ei = torch.tensor([[int(sub_ind)], [int(sub_ind)]], dtype=torch.long,
                                  device=self.edge_index.device)
        sub_feat = self.feat[subset]
        sub_nt = node_types[subset] if node_types is not None else None
        sub_et = edge_types[torch.where(emask)[0]] if edge_types is not None else None
        pos = subset if "node" in problem or "graph" in problem else torch.where(emask)[0]
        # the reference indexes np.array(names, dtype=str) (data.py:341-356); only the subgraph's
        # names are converted here, not every name of the graph (1M of them at c3)
        pos = pos.cpu().numpy()
        sub_names = take_names(names, pos)
        if return_pos:
            return sub_feat, sub_ei, sub_names, sub_ind, sub_nt, sub_et, pos
        return sub_feat, sub_ei, sub_names, sub_ind, sub_nt, sub_et

    def edge_comp_graph(self, ind, n_hops, names, return_pos=False):
        """Computational graph of an edge problem (edge masks mode; the reference's data.py:281-361
        hands the edge index to k_hop_subgraph as a node id, so its edge path is broken): nodes
        within n_hops + 1 hops of either endpoint of edge `ind`, every edge with both ends inside
        (original order), relabelled.  Returns (sub_feat, sub_edge_index, sub_names = the kept
        edges' names, sub_ind = position of edge `ind` among them, (u, v) relabelled)."""
        hops = n_hops + 1
        ei = self.edge_index
        n = self.feat.shape[0]
        if not 0 <= int(ind) < ei.shape[1]:
            raise IndexError(f"edge {ind} out of range for {ei.shape[1]} edges")
        u, v = int(ei[0, ind]), int(ei[1, ind])
        node = torch.zeros(n, dtype=torch.bool, device=ei.device)
        for seed in (u, v):
            subset, _, _, _ = k_hop_subgraph(seed, hops, ei, n)
            node[subset] = True
        subset = torch.nonzero(node).reshape(-1)
        remap = torch.full((n,), -1, dtype=torch.long, device=ei.device)
        remap[subset] = torch.arange(subset.numel(), device=ei.device)
        keep = node[ei[0]] & node[ei[1]]
        pos = torch.nonzero(keep).reshape(-1)
        sub_ind = int(torch.nonzero(pos == int(ind)).reshape(-1)[0])
        pos = pos.cpu().numpy()
        sub_names = take_names(names, pos)
        out = (self.feat[subset], remap[ei[:, keep]], sub_names, sub_ind,
               (int(remap[u]), int(remap[v])))
        return out + (pos,) if return_pos else out

    def element_size(self, problem):
        """data.py:363-388."""
        return self.edge_index.shape[1] if "edge" in problem else self.feat.shape[0]

    # -------------------------------------------------------------- perturbation seams (HIP)
    def build_edge_mask(self, mask):
        """data.py:390-451 — (edge keep [B*E] bool, tiled edge index [2, B*E] int32)."""
        B, S = mask.shape
        bits = engine.pack_masks(mask)
        ei = self.edge_index.to(mask.device)
        keep = engine.edge_keep(bits, S, ei[0], ei[1])
        off = (torch.arange(B, device=mask.device, dtype=torch.int32) * S).repeat_interleave(
            ei.shape[1])
        tiled = ei.int().repeat(1, B) + off
        return keep, tiled

    def perturb_node(self, mask, edge_type=None):
        """data.py:453-498."""
        keep, tiled = self.build_edge_mask(mask)
        et = None
        if edge_type is not None:
            et = edge_type.int().repeat(mask.shape[0])[keep]
        return tiled[:, keep], et

    def perturb_edge(self, mask, edge_type=None):
        """data.py:500-554 — edge masks: keep the edges whose mask entry is set."""
        flat = mask.reshape(-1)
        B = mask.shape[0]
        n = self.feat.shape[0]
        off = (torch.arange(B, device=mask.device, dtype=torch.int32) * n).repeat_interleave(
            self.edge_index.shape[1])
        tiled = self.edge_index.int().to(mask.device).repeat(1, B) + off
        active = torch.where(flat)[0]
        et = edge_type.int().repeat(B)[active] if edge_type is not None else None
        return tiled[:, active], et

    def concat_features(self, n, node_type=None):
        """data.py:556-589."""
        return self.feat.repeat(n, 1), (node_type.repeat(n) if node_type is not None else None)

    def perturbator(self, mask, problem, node_type=None, edge_type=None):
        """data.py:591-648 — B-fold union graph of the masked copies (generic black-box path)."""
        feat, nt = self.concat_features(mask.shape[0], node_type)
        if "edge" in problem:
            ei, et = self.perturb_edge(mask, edge_type)
        else:
            ei, et = self.perturb_node(mask, edge_type)
        return feat.float(), nt, ei, et

    # -------------------------------------------------------------- output table
    @staticmethod
    def config_val_dataframe(config_val_mean, config_val_std, names):
        """data.py:651-693."""
        ms = torch.stack([config_val_mean.detach(), config_val_std.detach()]).cpu().numpy()
        return sorted_frame(names, {"config_value_mean": ms[0], "config_value_std": ms[1]},
                            "config_value_mean")
