"""Helpers to load the golden fixtures (tests/golden/*.npz|json) produced by running the
reference (tests/golden/make_golden.py) and to turn them into oracle specs / product inputs."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

CASES = ["test_run", "test_run_t1", "toy", "hetero_single", "sage_shapley", "gcn2_graph",
         "gcn2_medium"]


def load_case(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    meta = json.load(open(os.path.join(GOLDEN, name + ".json")))
    return z, meta


def _unpack_dict(z, prefix):
    if prefix in z.files:
        return z[prefix]
    keys = [str(k) for k in z[prefix + "__keys"]]
    out = {}
    for i, k in enumerate(keys):
        kk = tuple(k.split("|")) if "|" in k else k
        out[kk] = z[f"{prefix}__{i}"]
    return out


def case_inputs(z):
    return _unpack_dict(z, "feat"), _unpack_dict(z, "edge_index")


def state_dict(z):
    return {k[3:]: z[k] for k in z.files if k.startswith("w__")}


def repeat_masks(z, meta):
    out = []
    for i in range(meta["n_repeats"]):
        shp = tuple(int(v) for v in z[f"r{i}_mask_shape"])
        m = np.unpackbits(z[f"r{i}_mask_bits"], axis=1, bitorder="little")[:, :shp[1]]
        out.append(m.astype(bool))
    return out


def oracle_spec(meta, sd):
    """Build the oracle's model spec from the fixture's arch_spec + state dict (ConvStack layout
    in make_golden.py == tests/test_utils.py:10-83 layout)."""
    a = meta["arch_spec"]
    rels = a.get("hetero_rels")
    convs = []
    for li in range(len(a["dims"]) - 1):
        base = f"conv.{2 * li}."
        if rels:
            rkeys = [tuple(r) for r in rels]
            params = {}
            for r in rkeys:
                p = base + "convs." + "__".join(r) + "."
                params[r] = _conv_params(a["kind"], sd, p)
            convs.append({"kind": a["kind"], "rels": rkeys, "params": params, "act": "relu"})
        else:
            convs.append({"kind": a["kind"], "rels": [None],
                          "params": {None: _conv_params(a["kind"], sd, base)}, "act": "relu"})
    fc = []
    nfc = len(a["fc"]) - 1
    for i in range(nfc):
        fc.append({"W": sd[f"fc.{2 * i}.weight"], "b": sd[f"fc.{2 * i}.bias"],
                   "act": "sigmoid" if i == nfc - 1 else "relu"})
    return {"convs": convs, "fc": fc}


def _conv_params(kind, sd, p):
    if kind == "gcn":
        return {"W": sd[p + "lin.weight"], "b": sd.get(p + "bias")}
    return {"Wl": sd[p + "lin_l.weight"], "bl": sd.get(p + "lin_l.bias"),
            "Wr": sd[p + "lin_r.weight"]}


def hetero_multi_setup(z, meta):
    """The multi-node-type golden case as the reference sees it after Explainer's host steps
    (see multi_type_setup)."""
    feat, ei = case_inputs(z)
    a = meta["arch_spec"]
    return multi_type_setup(feat, ei, meta["names"], meta["element"], meta["element_type"],
                            a["layers"], state_dict(z), a["fc"], conv=a["kind"])


def multi_type_setup(feat, ei, names_by_type, element, element_type, n_layers, sd, fc_dims,
                     conv="hetero_sage"):
    """hetero2homo (type blocks in feat-dict order, features zero-padded to the widest type,
    relation edges shifted by the node-type pointers, data.py:95-147,695-822), the L+1-hop
    computational subgraph of the element, and sub_ind = the element's position among the
    subgraph nodes of its type (explainer.py:449-463); oracle spec of a HeteroSageStack state
    dict.  Returns a dict."""
    import oracle
    ntypes = list(feat.keys())
    rels = list(ei.keys())
    wmax = max(v.shape[1] for v in feat.values())
    pads = [wmax - feat[t].shape[1] for t in ntypes]
    ptr = np.cumsum([0] + [feat[t].shape[0] for t in ntypes])[:-1]
    x = np.vstack([np.pad(feat[t], ((0, 0), (0, wmax - feat[t].shape[1]))) for t in ntypes])
    nt = np.concatenate([np.full(feat[t].shape[0], i) for i, t in enumerate(ntypes)])
    e = np.hstack([ei[r] + np.array([[ptr[ntypes.index(r[0])]], [ptr[ntypes.index(r[-1])]]])
                   for r in rels])
    et = np.concatenate([np.full(ei[r].shape[1], i) for i, r in enumerate(rels)])
    names = [n for t in ntypes for n in names_by_type[t]]
    q = names.index(element)
    subset, sub_ei, _, emask = oracle.comp_graph(q, n_layers, e, x.shape[0])
    sub_nt, sub_et = nt[subset], et[emask]
    sub_names = [names[i] for i in subset]
    etype = ntypes.index(element_type)
    filt = [n for n, t in zip(sub_names, sub_nt) if t == etype]
    layers = []
    for li in range(n_layers):
        if conv == "hetero_gat":  # GATConv((F_src, F_dst), c, heads, add_self_loops=False)
            pre = lambda r: f"conv.{2 * li}.convs.{'__'.join(r)}."
            layers.append({r: {"Ws": sd[pre(r) + "lin_src.weight"],
                               "Wd": sd.get(pre(r) + "lin_dst.weight"),
                               "att_s": sd[pre(r) + "att_src"], "att_d": sd[pre(r) + "att_dst"],
                               "bias": sd.get(pre(r) + "bias"), "concat": True,
                               "self_loops": False} for r in rels})
            continue
        layers.append({r: {"Wl": sd[f"conv.{2 * li}.convs.{'__'.join(r)}.lin_l.weight"],
                           "bl": sd.get(f"conv.{2 * li}.convs.{'__'.join(r)}.lin_l.bias"),
                           "Wr": sd[f"conv.{2 * li}.convs.{'__'.join(r)}.lin_r.weight"]}
                       for r in rels})
    nfc = len(fc_dims) - 1
    fc = [{"W": sd[f"fc.{2 * i}.weight"], "b": sd[f"fc.{2 * i}.bias"],
           "act": "sigmoid" if i == nfc - 1 else "relu"} for i in range(nfc)]
    return {"x": x[subset], "nt": sub_nt, "ei": sub_ei, "et": sub_et, "ntypes": ntypes,
            "rels": rels, "pads": pads, "sub_ind": filt.index(element),
            "spec": {"layers": layers, "fc": fc}, "sub_names": sub_names, "feat": feat,
            "edge_index": ei}
