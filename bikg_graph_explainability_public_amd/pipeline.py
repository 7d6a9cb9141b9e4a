"""One repeat of the explanation hot path on the device (explainer.py:490-519 loop body):

    mask rows (compat host sampler -> bit-pack, or device Philox sampler)
      -> per-row query logit      (ForwardPlan.forward: masked receptive-field message passing)
      -> KernelSHAP fp64 weights  (xpg_popcount_rows + xpg_shap_kernel)
      -> surrogate Adam epochs    (xpg_wlm_fit, one persistent workgroup)

Architectures the engine cannot compile run through `generic_outputs` (the user's torch module
on the B-fold union graph built with the HIP edge-keep kernel) — still on the GPU, with the
KernelSHAP and surrogate stages unchanged.
"""
import collections
import warnings
import weakref

import torch

from . import engine
from .data import Data
from .model import Model
from .program import UnsupportedArch, compile_arch


# generic multi-node-type path: one arch call over the per-type disjoint union of the copies
# (False: the reference's per-copy loop, model.py:118-253)
HETERO_BATCHED = True

def relation_edges(edge_index, edge_type, n_rel):
    if edge_type is None:
        return [edge_index]
    et = edge_type.to(edge_index.device)
    return [edge_index[:, et == r] for r in range(n_rel)]


_PROGRAMS = collections.OrderedDict()  # compiled_program's cache: key -> (weakref(arch), program)


def clear_programs():
    """Drop every cached compiled program and its padded device weights (compiled_program)."""
    _PROGRAMS.clear()


def compiled_program(arch, edge_type_names=None, node_type_names=None, state=None):
    """compile_arch(arch, ...) once per module state: keyed by the module (identity, checked by
    weak reference), every parameter and buffer (storage + in-place version counter: an
    optimizer step, load_state_dict or a replaced tensor compiles again) and the type names.
    The program carries the plans' weight-derived device tensors (ForwardPlan._program_tensor),
    so a new query's plan neither lowers the module nor re-pads its weights.  8 programs kept.
    `state`: the caller's (parameters, buffers) state tuples of this walk (Explainer.run reads
    them once per call); None reads them here.  An edit through `param.data` (e.g.
    `p.data.copy_(w)`) bumps no version counter and is not seen: call clear_programs() (or
    Explainer.clear_cache()) after one."""
    if state is None:
        state = (tuple((t.data_ptr(), t._version) for t in arch.parameters()),
                 tuple((t.data_ptr(), t._version) for t in arch.buffers()))
    key = (id(arch), state,
           tuple(tuple(e) for e in edge_type_names) if edge_type_names is not None else None,
           tuple(node_type_names) if node_type_names is not None else None)
    hit = _PROGRAMS.get(key)
    if hit is not None and hit[0]() is arch:
        _PROGRAMS.move_to_end(key)
        return hit[1]
    prog = compile_arch(arch, edge_type_names, node_type_names)
    _PROGRAMS[key] = (weakref.ref(arch), prog)
    while len(_PROGRAMS) > 8:
        _PROGRAMS.popitem(last=False)
    return prog


def build_plan(arch, feat, edge_index, queries, node_type=None, edge_type=None,
               node_type_names=None, edge_type_names=None, padded_dims=None, module_state=None):
    """ForwardPlan for `arch` on the (sub)graph, or None when the engine cannot run it.

    Multi-node-type graphs (model.py:118-253): the program's terms are gated by destination
    node type and the query is the reference's `out[sub_ind, 0]` — row sub_ind of the output
    node type's block — so `queries` are positions inside that type and are mapped to subgraph
    nodes here.  The plan is marked `multi_type` (its per-row outputs then go through
    `multi_type_targets`)."""
    multi = node_type_names is not None and node_type is not None and \
        len(torch.unique(node_type)) >= 2
    hetero = edge_type_names is not None and edge_type is not None
    try:
        prog = compiled_program(arch, edge_type_names if hetero else None,
                                node_type_names if multi else None, module_state)
    except UnsupportedArch as e:
        warnings.warn(f"engine cannot compile arch ({e}); using the generic torch path")
        return None
    if prog.link_act is not None:
        raise ValueError("a LinkModel scores edges: explain it with problem='edge_prediction' "
                         "and params['edge_masks'] = True")
    x = feat
    nt = None
    if multi:
        nt = node_type.long().reshape(-1)
        rows_t = torch.where(nt == prog.out_type)[0].cpu()
        queries = [int(q) for q in queries]
        if any(q >= rows_t.numel() for q in queries):
            raise IndexError("query index beyond the output node type's rows (model.py:247)")
        queries = [int(rows_t[q]) for q in queries]
    elif hetero and padded_dims is not None and padded_dims[0] > 0:
        x = feat[:, :feat.shape[1] - padded_dims[0]]
    rels = relation_edges(edge_index, edge_type if hetero else None,
                          len(edge_type_names) if hetero else 1)
    try:
        plan = engine.ForwardPlan(prog, x, rels, queries, node_type=nt)
    except ValueError as e:
        warnings.warn(f"engine plan rejected ({e}); using the generic torch path")
        return None
    plan.multi_type = multi
    return plan


def build_edge_plan(arch, feat, edge_index, u, v, module_state=None):
    """ForwardPlan of an edge problem (edge masks, Data.perturb_edge data.py:500-554): mask
    columns = the subgraph's edges, output = the LinkModel decoder's score of edge (u, v).
    None when the engine cannot compile `arch` (generic torch path)."""
    try:
        prog = compiled_program(arch, state=module_state)
    except UnsupportedArch as e:
        warnings.warn(f"engine cannot compile arch ({e}); using the generic torch path")
        return None
    if prog.link_act is None:
        warnings.warn("edge masks need an edge-level model (nn.LinkModel); using the generic "
                      "torch path")
        return None
    queries, link = ([u, v], (0, 1, prog.link_act)) if u != v else ([u], (0, 0, prog.link_act))
    cols = torch.arange(edge_index.shape[1], device=edge_index.device)
    try:
        return engine.ForwardPlan(prog, feat, [edge_index], queries, edge_cols=[cols], link=link)
    except ValueError as e:
        warnings.warn(f"engine plan rejected ({e}); using the generic torch path")
        return None


def generic_edge_outputs(arch, feat, edge_index, mask, u, v, max_rows=None):
    """Edge problem through the user's module (torch, on the device): the B-fold union graph of
    Data.perturbator with perturb_edge (data.py:591-648, 500-554: copy b keeps edge e iff
    mask[b, e], copy-major order, node ids shifted by b * N) and `arch(x, ei,
    edge_label_index=...)` scoring each copy's (u, v) -> y [B]."""
    B, _ = mask.shape
    N = feat.shape[0]
    step = B if max_rows is None else max_rows
    ys = []
    for b0 in range(0, B, step):
        m = mask[b0:b0 + step]
        nb = m.shape[0]
        rows, cols = torch.nonzero(m, as_tuple=True)
        ei = edge_index[:, cols] + rows * N
        x = feat.repeat(nb, 1).float()
        off = torch.arange(nb, device=feat.device) * N
        eli = torch.stack([off + u, off + v])
        with torch.no_grad():
            ys.append(arch(x, ei, edge_label_index=eli).reshape(-1).float())
    return torch.cat(ys)


def verify_edge_plan(plan, arch, feat, edge_index, u, v, rows=8, tol=1e-4):
    """The compiled edge plan against the user's module on a few random edge masks."""
    g = torch.Generator(device="cpu").manual_seed(1234)
    mask = (torch.rand((rows, edge_index.shape[1]), generator=g) < 0.5).to(feat.device)
    mask[0] = True
    ref = generic_edge_outputs(arch, feat, edge_index, mask, u, v)
    got = plan.forward(engine.pack_masks(mask))[:, 0]
    err = (ref - got).abs().max().item()
    return err <= tol * max(1.0, ref.abs().max().item()), err


def empty_copy_rows(bits, cols, edge_index):
    """bool [rows]: mask rows that keep no edge of the (sub)graph — the reference's
    multi-node-type loop outputs 0 for such copies instead of running the model
    (model.py:213-215).  One HIP pass over the rows (engine.rows_no_edge)."""
    rows, E = bits.shape[0], edge_index.shape[1]
    if E == 0:
        return torch.ones(rows, dtype=torch.bool, device=bits.device)
    return engine.rows_no_edge(bits, cols, edge_index[0], edge_index[1])


def multi_type_targets(y_rows, empty, batch, sub_ind, S, q4=True):
    """Regression targets of a multi-node-type repeat from per-row engine outputs.
    Copies without edges give 0 (model.py:213-215).  With q4 (the reference's behaviour,
    SURVEY.md quirk Q4) each batch's [B] outputs are cut again by
    extract_node_edge_output(out, sub_ind, S) (wlm.py:435-436): the one surviving value is
    the target of every row of the batch; q4=False keeps the per-copy outputs."""
    y = torch.where(empty, torch.zeros_like(y_rows), y_rows)
    if not q4:
        return y
    out = torch.empty_like(y)
    nfull = y.shape[0] // batch
    if nfull and sub_ind < batch <= S + sub_ind:
        # every full batch keeps exactly one value, row sub_ind: one vectorised broadcast
        out[:nfull * batch] = y[:nfull * batch].view(nfull, batch)[:, sub_ind:sub_ind + 1] \
            .expand(nfull, batch).reshape(-1)
        start = nfull * batch
    else:
        start = 0
    for r0 in range(start, y.shape[0], batch):
        yb = y[r0:r0 + batch]
        sel = yb[sub_ind::S]
        if sel.numel() == yb.numel():
            out[r0:r0 + batch] = sel
        elif sel.numel() == 1:
            out[r0:r0 + batch] = sel.expand(yb.numel())
        else:
            raise RuntimeError("model output does not broadcast against the mask batch "
                               "(the reference's weighted_mse_loss would fail here too)")
    return out


def generic_outputs(arch, feat, edge_index, mask, element_index, problem, node_type=None,
                    edge_type=None, node_type_names=None, edge_type_names=None,
                    padded_dims=None, batch=None, q4=True):
    """wlm.py:349-436 semantics per batch of mask rows with the user's module in torch.
    Returns y [R] (the regression target of each row; for multi-node-type graphs the
    reference's output[ind::S] collapse, quirk Q4, broadcast over its batch).  A list of
    element indices (single-node-type graphs) returns y [R, Q]: every query's extraction from
    the same union-graph forward."""
    if isinstance(element_index, (list, tuple)):
        return _generic_multi(arch, feat, edge_index, mask, element_index, problem, node_type,
                              edge_type, node_type_names, edge_type_names, padded_dims, batch)
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
            # one arch call over the disjoint union per node type (§8f2); HETERO_BATCHED =
            # False restores the reference's per-copy loop
            out = None
            if HETERO_BATCHED:
                out = mc.predict_hetero_output_batched(cf, pei, cnt, pet, node_type_names,
                                                       edge_type_names, B, S, element_index,
                                                       padded_dims, problem)
            if out is None:
                out = mc.predict_hetero_output(cf, pei, cnt, pet, node_type_names,
                                               edge_type_names, B, S, element_index,
                                               padded_dims, problem)
        if node_type is not None and edge_type is not None and isinstance(out, dict):
            out, _ = mc.hetero2homo_output(out)
        if element_index is not None and (q4 or n_types < 2):
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


def _generic_multi(arch, feat, edge_index, mask, queries, problem, node_type, edge_type,
                   node_type_names, edge_type_names, padded_dims, batch):
    """generic_outputs for several queries of a single-node-type graph: [R, Q]."""
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
        if node_type is not None and edge_type is not None and node_type_names is not None \
                and edge_type_names is not None:
            cf = data.homo2hetero(cf, cnt, node_type_names, padded_dims)
            pei = data.homo2hetero(pei, pet, edge_type_names)
        out = mc.infer(cf, pei, cnt, pet)
        if isinstance(out, dict):
            out, _ = mc.hetero2homo_output(out)
        ys.append(torch.stack([mc.extract_node_edge_output(out, int(q), S).reshape(-1).float()
                               for q in queries], 1).reshape(B, len(queries)))
    return torch.cat(ys)


def verify_plan(plan, arch, feat, edge_index, query, node_type=None, edge_type=None,
                node_type_names=None, edge_type_names=None, padded_dims=None, rows=8, tol=1e-4):
    """Check the compiled program against the user's module on a few random masks (guards the
    registration-order lowering in program.compile_arch).  `query` may be the list of a
    multi-query plan's queries: every output column is then checked."""
    g = torch.Generator(device="cpu").manual_seed(1234)
    S = feat.shape[0]
    mask = (torch.rand((rows, S), generator=g) < 0.5).to(feat.device)
    mask[0] = True
    multi = getattr(plan, "multi_type", False)
    if isinstance(query, (list, tuple)):
        assert not multi, "multi-query plans are single-node-type"
        ref = generic_outputs(arch, feat, edge_index, mask, list(query), "node", node_type,
                              edge_type, node_type_names, edge_type_names, padded_dims)
        got = plan.forward(engine.pack_masks(mask))[:, :len(query)]
        err = (ref - got).abs().max().item()
        return err <= tol * max(1.0, ref.abs().max().item()), err
    ref = generic_outputs(arch, feat, edge_index, mask, query, "node", node_type, edge_type,
                          node_type_names, edge_type_names, padded_dims, q4=not multi)
    bits = engine.pack_masks(mask)
    got = plan.forward(bits)[:, 0]
    if multi:  # per-copy outputs on both sides (zero for copies without edges)
        got = torch.where(empty_copy_rows(bits, S, edge_index), torch.zeros_like(got), got)
    err = (ref - got).abs().max().item()
    return err <= tol * max(1.0, ref.abs().max().item()), err


def fit_repeat(bits, cols, batch, y, w0, params):
    """KernelSHAP + surrogate fit for one repeat; returns (w_final, losses[list], best_epoch,
    kernel)."""
    kern = engine.shap_kernel(bits, cols)
    w, losses, best, _, _ = engine.wlm_fit(bits, cols, batch, y, kern, w0, params)
    return w, losses, best, kern
