"""Perturbation masks: the reference's `Mask` class (masks.py:10-397) plus the device sampler.

Two samplers share one output contract (bool [R, S] rows + per-row community index):

* compat (default, `params["mask_sampler"] = "compat"`): restates masks.py:262-397 with torch's
  CPU generator in the reference's exact call order — per community in length-descending order:
  internal randint, external antithetic randint (+ extra row), optional dead-mask randperm; then
  the row shuffle randperm — so masks are bit-identical to the reference CPU path for the same
  RNG state (tests/test_host_cpu.py::test_compat_sampler_reproduces_reference_masks).  Rows
  are then bit-packed on the device.
* device (`"device"`): counter-based Philox bits generated directly in HBM by the HIP samplers
  — same distribution, no host work; used for throughput.  Without communities:
  engine.sample_shapley; with communities: engine.sample_communities over the block plan of
  `Mask.community_plan` (same block sizes, antithetic coalitions, dead-mask activation and
  own-community internal bits; the row shuffle is a seeded bijection instead of randperm).
"""
import itertools
import math

import numpy as np
import torch
from torch.utils.data import DataLoader

from .data import Data
from .pathways import Pathways


def dataloader_seed_draw():
    """The reference iterates its mask DataLoader once per repeat (wlm.py:210); creating the
    iterator draws a base seed from torch's global CPU generator
    (torch.utils.data.dataloader._BaseDataLoaderIter.__init__).  Compat mode replays that
    draw so the next repeat's masks stay on the reference's random stream."""
    torch.empty((), dtype=torch.int64).random_()


class Mask(Data):
    def __init__(self, feat, edge_index, pathways, params, problem):
        super().__init__(feat, edge_index)
        self.pathways = pathways
        self.params = params
        self.problem = problem

    @staticmethod
    def assertions_mask_generator(params):
        """masks.py:37-60."""
        n_perturbs = params["interpret_samples"]
        epochs = params["epochs"]
        assert isinstance(n_perturbs, (int, float)), \
            "Number of perturbations in batch is not numeric"
        assert isinstance(epochs, (int, float)), "Number of epochs in batch is not numeric"
        return abs(n_perturbs), abs(epochs)

    def obtain_device(self):
        """masks.py:62-78."""
        if isinstance(self.feat, dict):
            return self.feat[list(self.feat.keys())[0]].device
        return self.feat.device

    @staticmethod
    def internal_sizes(n_members, len_pathways, total_size):
        """masks.py:98-118 — (block rows, internal-only rows) of one community."""
        fraction = n_members / torch.sum(len_pathways)
        size = math.ceil(fraction * total_size)
        size_internal = math.ceil(fraction * size)
        if size_internal < 3:
            size_internal, size = 1, 2
        return size, size_internal

    @staticmethod
    def get_internal_mask(pathway, len_pathways, total_size, device):
        """masks.py:81-136 — rows proportional to the community size; random member bits."""
        size, size_internal = Mask.internal_sizes(len(pathway), len_pathways, total_size)
        internal = torch.randint(0, 2, (size, len(pathway)), dtype=torch.bool)
        return internal.to(device), size_internal

    def community_plan(self):
        """Host plan of the device community sampler (engine.sample_communities): the block
        loop of `generate` without its random draws.  Returns (blocks int32 [P', 5] =
        {row_start, size, size_internal, own, off}, src_rows, out_rows, shuffle) — the
        reference truncates to the `total` rows of the largest communities instead of
        shuffling when S > 4000 (masks.py:340-380)."""
        n_perturbs, epochs = self.assertions_mask_generator(self.params)
        total = n_perturbs * epochs
        S = self.element_count()
        lens = torch.tensor([len(p) for p in self.pathways])
        order = torch.argsort(lens, descending=True)
        # internal_sizes for every community at once, in the same float32 tensor arithmetic:
        # `n / tensor` is Tensor.__rtruediv__ = reciprocal() * n (not a correctly rounded
        # quotient), then ceil(fraction * total) and ceil(fraction * size), elementwise
        frac = torch.sum(lens).reciprocal() * lens[order]
        sizes = torch.ceil(frac * total)
        sizes_int = torch.ceil(frac * sizes)
        small = sizes_int < 3
        sizes = torch.where(small, torch.full_like(sizes, 2), sizes).long().tolist()
        sizes_int = torch.where(small, torch.ones_like(sizes_int), sizes_int).long().tolist()
        order_l = order.tolist()
        blocks, start = [], 0
        for e in range(len(order_l)):
            size, size_internal = sizes[e], sizes_int[e]
            blocks.append((start, size, size_internal, order_l[e], e))
            start += size
            if start - size > total and S > 4000:
                break
        out_rows, shuffle = start, True
        if S > 4000 and start > total:
            out_rows, shuffle = int(total), False
        return torch.tensor(blocks, dtype=torch.int32), start, out_rows, shuffle

    def get_external_indices(self, full_mask, ind_pathway, size_internal):
        """masks.py:138-194 — external coalitions for rows size_internal..end.  Column
        `ind_pathway` (the position in length-sorted order, as the reference passes it) is
        switched off in the community mask."""
        pw = Pathways(self.pathways, None)
        device = full_mask.device
        pmask = pw.mask_generator((full_mask.shape[0] - size_internal) // 2, full_mask.shape[0],
                                  size_internal, torch.device("cpu"))
        pmask[:, ind_pathway] = False
        if len(self.pathways) - 1 > 0 and pmask.sum() == 0:
            pmask = pw.activate_dead_mask(pmask, ind_pathway)
        element, members = pw.pathway_mask2node_mask(pmask)
        rows = torch.where(element)[0] + size_internal
        out = full_mask.cpu()
        out[rows, members[element]] = True
        return out.to(device)

    @staticmethod
    def mask_loader(mask, pieces):
        """masks.py:197-229 — DataLoader with batch_size = rows // pieces."""
        return DataLoader(mask, batch_size=mask.shape[0] // pieces, num_workers=0)

    def shapley_mask(self, size, device):
        """masks.py:231-260."""
        return torch.randint(0, 2, size, dtype=torch.bool).to(device)

    def element_count(self):
        if "edge" in self.problem:
            # masks.py:292-294 reads a non-existent attribute for edge problems; mirror it.
            return self.edge_size.shape[1]
        return self.feat.shape[0]

    def generate(self):
        """Compat sampler: (mask bool [R, S] on CPU, pathway_rows int32 [R] or None).
        Community masks come from the native replay of the reference's draws
        (`_community_bits`), unpacked; Shapley masks are the reference's torch.randint."""
        n_perturbs, epochs = self.assertions_mask_generator(self.params)
        total = n_perturbs * epochs
        S = self.element_count()
        if self.pathways is not None:
            bits, prow = self._community_bits()
            return _unpack_host(bits, S), prow
        mask = self.shapley_mask((total, S), "cpu")
        return mask[torch.randperm(mask.shape[0])], None

    def _community_bits(self):
        """The community compat draw as bit-packed host rows: (bits int32 [R, W], pathway_rows
        int32 [R]).  The block plan (`community_plan`: the reference's per-community sizes,
        length-descending order and early stop, masks.py:299-348) is built here; every random
        draw of the block loop -- internal randint, antithetic external randint (+ extra row),
        dead-mask randperm -- is replayed natively from torch's generator state
        (engine.compat_community_bits); the row shuffle is torch.randperm on the advanced
        generator, or the S > 4000 truncation to the rows of the largest communities
        (masks.py:367-390).  Bit-identical to `_generate_torch` and the reference."""
        from . import engine
        n_perturbs, epochs = self.assertions_mask_generator(self.params)
        total = n_perturbs * epochs
        S = self.element_count()
        blocks, src_rows, _, shuffle = self.community_plan()
        for o in blocks[:, 3].tolist():
            self.pathways[o].sort()  # the reference sorts the caller's lists in place
        bits = engine.compat_community_bits(S, [sorted(p) for p in self.pathways], blocks)
        # host bookkeeping in numpy (torch's threaded kernels cost more than they save here)
        b = blocks.numpy()
        prow = np.repeat(b[:, 3], b[:, 1]).astype(np.int32)
        if shuffle:
            ii = torch.randperm(src_rows).numpy()
        else:
            lens = torch.tensor([len(p) for p in self.pathways], dtype=torch.int)
            ii = torch.argsort(lens[torch.from_numpy(prow).long()], descending=True)[:total].numpy()
        return torch.from_numpy(bits.numpy()[ii]), torch.from_numpy(prow[ii])

    def _generate_torch(self):
        """The reference's community block loop (masks.py:299-390) in torch calls, draw for draw
        (kept as the restatement the native replay `_community_bits` is tested against)."""
        n_perturbs, epochs = self.assertions_mask_generator(self.params)
        total = n_perturbs * epochs
        S = self.element_count()
        lens = torch.tensor([len(p) for p in self.pathways])
        order = torch.argsort(lens, descending=True)
        blocks, rows_of, sizes_of = [], [], []
        cumulative = 0
        for e in range(order.shape[0]):
            pathway = self.pathways[order[e]]
            pathway.sort()  # the reference sorts the caller's lists in place
            internal, size_internal = self.get_internal_mask(pathway, lens, total, "cpu")
            block = torch.zeros((internal.shape[0], S), dtype=torch.bool)
            block = self.get_external_indices(block, e, size_internal)
            block[:, pathway] = internal
            rows_of.append([int(order[e])] * block.shape[0])
            sizes_of.append([len(pathway)] * block.shape[0])
            blocks.append(block)
            if cumulative > total and S > 4000:
                break
            cumulative += block.shape[0]
        mask = torch.cat(blocks, dim=0)
        prow = torch.tensor(list(itertools.chain.from_iterable(rows_of)), dtype=torch.int)
        psize = torch.tensor(list(itertools.chain.from_iterable(sizes_of)), dtype=torch.int)
        if S > 4000 and mask.shape[0] > total:
            ind = torch.argsort(psize, descending=True)[:total]
        else:
            ind = torch.randperm(mask.shape[0])
        return mask[ind], prow[ind]

    def generate_bits(self, device):
        """Compat sampler straight to bit-packed device rows: (bits int32 [R, W], pathway_rows).
        Community masks: the native replay of the reference's draws (`_community_bits`), then
        uploaded.  Shapley masks (no communities):
        the same torch CPU draws replayed natively as packed rows (engine.compat_shapley_bits),
        then the reference's randperm row shuffle applied on the device -- bit-identical rows
        and the same generator state afterwards, without the [R, S] bool tensor and its host
        row gather (masks.py:231-260, 375-380)."""
        from . import engine
        if self.pathways is not None:
            bits, prow = self._community_bits()
            dev = torch.device(device)
            if dev.type == "cpu":
                return bits, prow
            return bits.to(dev, non_blocking=True), prow.to(dev, non_blocking=True)
        n_perturbs, epochs = self.assertions_mask_generator(self.params)
        size = torch.Size((n_perturbs * epochs, self.element_count()))  # torch.randint's checks
        host = engine.compat_shapley_bits(size[0], size[1])
        ind = torch.randperm(host.shape[0])
        dev = torch.device(device)
        if dev.type == "cpu":
            return host[ind], None
        return host.to(dev, non_blocking=True)[ind.to(dev)], None

    def mask_generator(self):
        """masks.py:262-397 — (DataLoader over the shuffled mask, pathway_rows)."""
        _, epochs = self.assertions_mask_generator(self.params)
        mask, prow = self.generate()
        device = self.obtain_device()
        mask = mask.to(device)
        if prow is not None:
            prow = prow.to(device)
        return self.mask_loader(mask, epochs), prow


def _unpack_host(bits, cols):
    """Bit-packed int32 [R, W] host rows -> bool [R, cols] (bit c % 32 of word c // 32)."""
    b = bits.contiguous().numpy().view(np.uint8).reshape(bits.shape[0], -1)
    return torch.from_numpy(np.unpackbits(b, axis=1, bitorder="little")[:, :cols].copy()).bool()
