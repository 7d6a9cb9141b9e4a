"""Diagnostic (not part of the product): frontier / term sizes of the c5 plan (bench.c5_section's
graph and arch) — what the multi-kernel forward's kernels iterate over per mask row."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bikg_graph_explainability_public_amd import _lib, pipeline  # noqa: E402
from bikg_graph_explainability_public_amd.data import Data  # noqa: E402
from bikg_graph_explainability_public_amd.nn import HeteroSageStack  # noqa: E402


def main():
    _lib.load()
    dev = torch.device("cuda", 0)
    sizes = {"gene": 500_000, "protein": 300_000, "drug": 200_000}
    F = 256
    g = torch.Generator(device=dev).manual_seed(5)
    feat = {t: torch.randn((n, F), generator=g, device=dev) for t, n in sizes.items()}
    ei = {r: torch.stack([torch.randint(0, sizes[r[0]], (2_000_000,), generator=g, device=dev),
                          torch.randint(0, sizes[r[-1]], (2_000_000,), generator=g, device=dev)])
          for r in bench.C5_RELS}
    torch.manual_seed(0)
    arch = HeteroSageStack(bench.C5_RELS, {t: F for t in sizes}, 64, 2, [64, 16, 1]).to(dev).eval()
    fh, eh, nt, et, _, _, pads = Data(feat, ei).hetero2homo()
    ntn, etn = list(feat), list(ei)
    sub_x, sub_ei, _, sub_ind, sub_nt, sub_et = Data(fh, eh).comp_graph(
        7, 2, "node", [str(i) for i in range(fh.shape[0])], nt, et)
    plan = pipeline.build_plan(arch, sub_x, sub_ei, [int(sub_ind)], sub_nt.long(), sub_et, ntn, etn, pads)
    print("S", sub_x.shape[0], "E", sub_ei.shape[1], "n0", plan.n0, "n_rel", plan.n_rel,
          "frontiers", [len(f) for f in plan.frontiers], "deg_edges", int(plan.desc.n_deg_edges))
    for li in range(plan.desc.n_layers):
        ld = plan._layers[li]
        print(f"layer {li}: n_tgt {ld.n_tgt} n_edges {ld.n_edges} n_terms {ld.n_terms} "
              f"f_out_pad {ld.f_out_pad} kinds {[ld.terms[k].kind for k in range(ld.n_terms)]}")

if __name__ == "__main__":
    main()
