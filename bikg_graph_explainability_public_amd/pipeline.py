"""One repeat of the explanation hot path on the device (explainer.py:490-519 loop body):

    mask rows (compat host sampler -> bit-pack, or device Philox sampler)
      -> per-row query logit      (ForwardPlan.forward: masked receptive-field message passing)
      -> KernelSHAP fp64 weights  (xpg_popcount_rows + xpg_shap_kernel)
      -> surrogate Adam epochs    (xpg_wlm_fit, one persistent workgroup)

Architectures the engine cannot compile run through `generic_outputs` (the user's torch module
on the B-fold union graph built with the HIP edge-keep kernel) — still on the GPU, with the
KernelSHAP and surrogate stages unchanged.
"""
import os
import warnings

import torch

from . import engine
from .data import Data
from .model import Model
from .program import UnsupportedArch, compile_arch


def relation_edges(edge_index, edge_type, n_rel):
    if edge_type is None:
        return [edge_index]
    et = edge_type.to(edge_index.device)
    return [edge_index[:, et == r] for r in range(n_rel)]


def build_plan(arch, feat, edge_index, queries, node_type=None, edge_type=None,
               node_type_names=None, edge_type_names=None, padded_dims=None):
    """ForwardPlan for `arch` on the (sub)graph, or None when the engine cannot run it."""
    if node_type_names is not None and node_type is not None and \
            len(torch.unique(node_type)) >= 2:
        return None  # multi-node-type graphs: per-copy generic path (model.py:118-253)
    hetero = edge_type_names is not None and edge_type is not None
    try:
        prog = compile_arch(arch, edge_type_names if hetero else None)
    except UnsupportedArch as e:
        warnings.warn(f"engine cannot compile arch ({e}); using the generic torch path")
        return None
    x = feat
    if hetero and padded_dims is not None and padded_dims[0] > 0:
        x = feat[:, :feat.shape[1] - padded_dims[0]]
    rels = relation_edges(edge_index, edge_type if hetero else None,
                          len(edge_type_names) if hetero else 1)
    try:
        return engine.ForwardPlan(prog, x, rels, queries)
    except ValueError as e:
        warnings.warn(f"engine plan rejected ({e}); using the generic torch path")
        return None


def generic_outputs(arch, feat, edge_index, mask, element_index, problem, node_type=None,
                    edge_type=None, node_type_names=None, edge_type_names=None,
                    padded_dims=None, batch=None):
    """wlm.py:349-436 semantics per batch of mask rows with the user's module in torch.
    Returns y [R] (the regression target of each row; for multi-node-type graphs the
    reference's output[ind::S] collapse, quirk Q4, broadcast over its batch)."""
    data = Data(feat, edge_index)
    mc = Model(arch)
    R, S = mask.shape
    batch = R if batch is None else batch
    ys = []
    for r0 in range(0, R, batch):
        mb = mask[r0:r0 + batch]
        B = mb.shape[0]
        cf, cnt, pei, pet = data.perturbator(mb, problem, node_type, edge_type)
        pei = pei.long()
        n_types = 1 if node_type_names is None else len(torch.unique(node_type))
        if node_type is not None and edge_type is not None and node_type_names is not None \
                and edge_type_names is not None and n_types < 2:
            cf = data.homo2hetero(cf, cnt, node_type_names, padded_dims)
            pei = data.homo2hetero(pei, pet, edge_type_names)
        if n_types < 2:
            out = mc.infer(cf, pei, cnt, pet)
        else:
            # one arch call over the disjoint union per node type (§8f2); XPG_HETERO_LOOP=1
            # restores the reference's per-copy loop
            out = None
            if os.environ.get("XPG_HETERO_LOOP", "0") != "1":
                out = mc.predict_hetero_output_batched(cf, pei, cnt, pet, node_type_names,
                                                       edge_type_names, B, S, element_index,
                                                       padded_dims, problem)
            if out is None:
                out = mc.predict_hetero_output(cf, pei, cnt, pet, node_type_names,
                                               edge_type_names, B, S, element_index,
                                               padded_dims, problem)
        if node_type is not None and edge_type is not None and isinstance(out, dict):
            out, _ = mc.hetero2homo_output(out)
        if element_index is not None:
            out = mc.extract_node_edge_output(out, element_index, S)
        out = out.reshape(-1).float()
        if out.numel() == B:
            ys.append(out)
        elif out.numel() == 1:
            ys.append(out.expand(B))
        else:
            raise RuntimeError("model output does not broadcast against the mask batch "
                               "(the reference's weighted_mse_loss would fail here too)")
    return torch.cat(ys)


def verify_plan(plan, arch, feat, edge_index, query, node_type=None, edge_type=None,
                node_type_names=None, edge_type_names=None, padded_dims=None, rows=8, tol=1e-4):
    """Check the compiled program against the user's module on a few random masks (guards the
    registration-order lowering in program.compile_arch)."""
    g = torch.Generator(device="cpu").manual_seed(1234)
    S = feat.shape[0]
    mask = (torch.rand((rows, S), generator=g) < 0.5).to(feat.device)
    mask[0] = True
    ref = generic_outputs(arch, feat, edge_index, mask, query, "node", node_type, edge_type,
                          node_type_names, edge_type_names, padded_dims)
    got = plan.forward(engine.pack_masks(mask))[:, 0]
    err = (ref - got).abs().max().item()
    return err <= tol * max(1.0, ref.abs().max().item()), err


def fit_repeat(bits, cols, batch, y, w0, params):
    """KernelSHAP + surrogate fit for one repeat; returns (w_final, losses[list], best_epoch,
    kernel)."""
    kern = engine.shap_kernel(bits, cols)
    w, losses, best, _, _ = engine.wlm_fit(bits, cols, batch, y, kern, w0, params)
    return w, losses, best, kern
