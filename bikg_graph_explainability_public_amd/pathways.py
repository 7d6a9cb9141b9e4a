"""Communities ("pathways"): the reference's `Pathways` class (pathways.py:8-429), same names,
arguments and outputs.

Host-side bookkeeping (filtering, name -> index, hetero flattening, DataFrames) is plain
Python / torch.  The random community coalitions (`mask_generator`, `activate_dead_mask`) draw
from torch's CPU generator in exactly the reference's call order so that compat-mode masks are
bit-identical to the reference CPU path; `aggregate` runs as one segmented mean on the device.
"""
import itertools

import numpy as np
import pandas as pd
import torch

from .frames import sorted_frame


class Pathways:
    """Graph communities.  communities: list of lists of names or indices (or a dict per
    element type for heterogeneous graphs); community_names: list (or dict); community_types:
    per-community type tensor for hetero graphs."""

    def __init__(self, communities, community_names, community_types=None):
        self.communities = communities
        self.community_names = community_names
        self.community_types = community_types
        if self.community_names is None:
            self.community_names = list(range(len(self.communities)))

    # -------------------------------------------------------------- preprocessing (host)
    def comp_graph(self, names):
        """pathways.py:33-102 — keep communities that overlap the computational graph; members
        become the (sorted, string) intersection with `names`."""
        names_arr = np.array(names, dtype=str)
        subs, sub_names = [], []
        sub_types = [] if self.community_types is not None else None
        for i, (community, cname) in enumerate(zip(self.communities, self.community_names)):
            common = np.intersect1d(np.array(community, dtype=str), names_arr)
            if len(common) > 0:
                subs.append(common.tolist())
                sub_names.append(cname)
                if sub_types is not None:
                    sub_types.append(self.community_types[i])
        if sub_types is not None:
            sub_types = torch.tensor(sub_types, device=self.community_types.device)
        return subs, sub_names, sub_types

    def names2inds(self, names):
        """pathways.py:104-136 — member names -> positions in `names` (string-sorted order)."""
        if isinstance(self.communities[0][0], (int, np.integer)):
            return self.communities
        names_arr = np.array(names, dtype=str)
        out = []
        for community in self.communities:
            _, pos, _ = np.intersect1d(names_arr, np.array(community, dtype=str),
                                       return_indices=True)
            out.append(pos.tolist())
        return out

    def shift_hetero_pathways(self, pointers):
        """pathways.py:138-160 — add each type's homogeneous offset to integer members."""
        for key, pointer in zip(list(self.communities.keys()), pointers):
            for i in range(len(self.communities[key])):
                self.communities[key][i] = (np.array(self.communities[key][i]) +
                                            int(pointer)).tolist()

    def hetero2homo(self, problem, node_pointers=None, edge_pointers=None):
        """pathways.py:162-232 — flatten {type: [communities]} into one list (+ type tensor).
        Integer members are shifted only for problem == 'node' / 'edge' exactly (as the
        reference does)."""
        homo, homo_names, types = self.communities, self.community_names, None
        if isinstance(self.communities, dict):
            keys = list(self.communities.keys())
            first = self.communities[keys[0]][0][0]
            if isinstance(first, (int, float, np.integer)):
                if problem == "node":
                    self.shift_hetero_pathways(node_pointers)
                elif problem == "edge":
                    self.shift_hetero_pathways(edge_pointers)
            device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
            types, homo, homo_names = [], [], []
            for t, key in enumerate(keys):
                value = self.communities[key]
                types.append(torch.full((len(value),), float(t), device=device))
                homo.extend(value)
                homo_names.append(self.community_names[key])
            types = torch.cat(types)
            homo_names = list(itertools.chain.from_iterable(homo_names))
        return homo, homo_names, types

    # -------------------------------------------------------------- random coalitions (CPU RNG)
    def mask_generator(self, half_size, size, size_internal, device):
        """pathways.py:234-283 — antithetic community coalitions: `half_size` random rows, their
        complements, plus one extra random row when size - size_internal is odd."""
        n = len(self.communities)
        half = torch.randint(0, 2, (half_size, n), dtype=torch.bool)
        out = torch.cat([half, ~half], dim=0)
        if (size - size_internal) % 2 != 0:
            out = torch.cat([out, torch.randint(0, 2, (1, n), dtype=torch.bool)], dim=0)
        return out.to(device)

    def activate_dead_mask(self, pathway_mask, pathway_ind):
        """pathways.py:285-334 — when no community is on, switch one on per row, cycling through a
        random permutation of the other communities."""
        fixed = pathway_mask.clone()
        order = torch.randperm(len(self.communities))
        order = order[order != pathway_ind]
        rows = pathway_mask.shape[0]
        if rows > len(order) and len(order) > 0:
            order = torch.cat([order] * (rows // len(order) + 1))
        order = order[:rows]
        fixed[torch.arange(rows), order.to(fixed.device)] = True
        return fixed

    def pathway_mask2node_mask(self, pathway_mask):
        """pathways.py:336-385 — expand community flags to member columns.
        Returns (element_mask [rows, J], tiled member ids [rows, J]), J = sum of sizes."""
        device = pathway_mask.device
        members = torch.tensor(list(itertools.chain.from_iterable(self.communities)),
                               device=device, dtype=torch.long)
        sizes = torch.tensor([len(c) for c in self.communities], device=device)
        rows = pathway_mask.shape[0]
        element = torch.repeat_interleave(pathway_mask.reshape(-1), sizes.repeat(rows))
        return element.reshape(rows, members.numel()), members.repeat(rows, 1)

    # -------------------------------------------------------------- scoring
    def aggregate(self, config_val, community_inds):
        """pathways.py:387-429 — community score = mean member score; DataFrame indexed by
        community name, sorted descending, NaN rows dropped.  One segmented mean (index_add)
        on the scores' device (member / segment index tensors cached while the communities are
        unchanged), one host transfer, and the frame built once from the sorted arrays."""
        dev = config_val.device
        flat, seg, cnt = self._segments(community_inds, dev)
        vals = config_val.reshape(-1).float()[flat]
        sums = torch.zeros(cnt.numel(), dtype=torch.float32, device=dev).index_add_(0, seg, vals)
        scores = (sums / cnt).cpu().numpy().astype(np.float64)
        return sorted_frame(self.community_names, {"score": scores}, "score", dropna=True)

    def _segments(self, community_inds, dev):
        lens = np.fromiter((len(c) for c in community_inds), dtype=np.int64,
                           count=len(community_inds))
        flat = np.fromiter(itertools.chain.from_iterable(community_inds), dtype=np.int64,
                           count=int(lens.sum()))
        c = getattr(self, "_seg_cache", None)
        if c is not None and c[0] == dev and np.array_equal(c[1], lens) and np.array_equal(c[2], flat):
            return c[3]
        seg = np.repeat(np.arange(len(lens), dtype=np.int64), lens)
        t = (torch.from_numpy(flat).to(dev), torch.from_numpy(seg).to(dev),
             torch.from_numpy(lens.astype(np.float32)).to(dev))
        self._seg_cache = (dev, lens, flat, t)
        return t

