"""Rebuild the golden cases' inputs with the product package (CPU tensors)."""
import copy

import torch

from bikg_graph_explainability_public_amd.explainer import Explainer
from bikg_graph_explainability_public_amd.nn import ConvStack, HeteroSageStack, HeteroGATStack
from golden_utils import case_inputs, load_case, state_dict


def _t(x):
    if isinstance(x, dict):
        return {k: torch.as_tensor(v) for k, v in x.items()}
    return torch.as_tensor(x)


def build_arch(meta, z):
    a = meta["arch_spec"]
    if a["kind"] == "hetero_gat":
        arch = HeteroGATStack([tuple(r) for r in a["rels"]], a["in_dims"], a["hidden"],
                              a["heads"], a["fc"])
        arch.load_state_dict({k: torch.as_tensor(v) for k, v in state_dict(z).items()})
        return arch.eval()
    if a["kind"] == "hetero_sage":
        arch = HeteroSageStack([tuple(r) for r in a["rels"]], a["in_dims"], a["hidden"],
                               a["layers"], a["fc"])
        arch.load_state_dict({k: torch.as_tensor(v) for k, v in state_dict(z).items()})
        return arch.eval()
    rels = a.get("hetero_rels")
    arch = ConvStack(a["kind"], a["dims"], a["fc"],
                     hetero_rels=[tuple(r) for r in rels] if rels else None)
    arch.load_state_dict({k: torch.as_tensor(v) for k, v in state_dict(z).items()})
    return arch.eval()


def build_explainer(name, params_override=None):
    """Explainer over a golden case's inputs; returns (explainer, z, meta)."""
    z, meta = load_case(name)
    feat, ei = case_inputs(z)
    feat, ei = _t(feat), _t(ei)
    if isinstance(ei, dict):
        ei = {k: v.long() for k, v in ei.items()}
    else:
        ei = ei.long()
    arch = build_arch(meta, z)
    params = dict(meta["params"])
    if params_override:
        params.update(params_override)
    names = meta["names"]
    pathways = copy.deepcopy(meta["pathways"])
    exp = Explainer(feat, ei, arch, params, names, pathways, meta["pathway_names"],
                    meta["element_type"], problem=meta["problem"])
    return exp, z, meta
