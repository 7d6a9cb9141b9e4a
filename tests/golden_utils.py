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
