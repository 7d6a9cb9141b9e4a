"""Generate golden vectors by running the REFERENCE implementation in this container.

    python tests/golden/make_golden.py            # writes tests/golden/*.npz / *.json

Imports `pathway_explanations` from /root/reference/src (read-only) with the PyG 2.0.4 shim in
oracle/pyg_shim on sys.path, runs the reference pipeline on small cases and records inputs,
every intermediate the hot path produces (masks + pathway rows per repeat, per-batch KernelSHAP
weights and GNN outputs, initial/final surrogate weights, losses) and the two output DataFrames.

Two behaviour-preserving harness patches are applied:
  * torch.optim.lr_scheduler.ReduceLROnPlateau is wrapped to drop `verbose=` (removed in the
    torch shipped here; the reference builds the scheduler but never steps it, wlm.py:250);
  * checkpoints are loaded with torch.load(weights_only=True) and converted to plain arrays.

Nothing here is needed at run time: the committed fixtures are data (inputs + expected outputs).
"""
import json
import os
import sys

import numpy as np
import torch
from torch import nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SRC = "/root/reference/src"
REF_DATA = "/root/reference/test_data"
sys.path.insert(0, os.path.join(REPO, "oracle", "pyg_shim"))
sys.path.insert(0, REF_SRC)

_RLR = torch.optim.lr_scheduler.ReduceLROnPlateau


class _RLRNoVerbose(_RLR):
    def __init__(self, *a, **kw):
        kw.pop("verbose", None)
        super().__init__(*a, **kw)


torch.optim.lr_scheduler.ReduceLROnPlateau = _RLRNoVerbose

import pathway_explanations as pe  # noqa: E402
from pathway_explanations import explainer as pe_explainer  # noqa: E402
from pathway_explanations import wlm as pe_wlm  # noqa: E402
from pathway_explanations.masks import Mask as PeMask  # noqa: E402
from pathway_explanations.kernels import Kernel as PeKernel  # noqa: E402
from torch_geometric.nn import GATConv, GCNConv, SAGEConv, HeteroConv, Linear  # noqa: E402

torch.set_num_threads(8)

PARAMS = {"seed": 1, "interpret_samples": 20, "epochs": 50, "optimizer": "adam", "lr": 0.01,
          "lr_patience": 10, "l1_lambda": 1e-4}  # /root/reference/config/configs.json


# ----------------------------------------------------------------------------- model zoo
class ConvStack(nn.Module):
    """conv ModuleList [Conv, ReLU]* + fc ModuleList [Linear, act]* (tests/test_utils.py:10-83
    layout, so checkpoint keys conv.0.lin.weight / fc.4.bias etc. match)."""

    def __init__(self, kind, dims, fc_dims, hetero_rels=None):
        super().__init__()
        convs = []
        for i in range(len(dims) - 1):
            if hetero_rels is not None:
                mk = GCNConv if kind == "gcn" else SAGEConv
                convs.append(HeteroConv({r: mk(dims[i], dims[i + 1]) for r in hetero_rels},
                                        aggr="sum"))
            elif kind == "gcn":
                convs.append(GCNConv(dims[i], dims[i + 1]))
            else:
                convs.append(SAGEConv(dims[i], dims[i + 1]))
            convs.append(nn.ReLU())
        self.conv = nn.ModuleList(convs)
        fcs = []
        for i in range(len(fc_dims) - 1):
            fcs.append(Linear(fc_dims[i], fc_dims[i + 1]))
            fcs.append(nn.Sigmoid() if i == len(fc_dims) - 2 else nn.ReLU())
        self.fc = nn.ModuleList(fcs)
        self.hetero = hetero_rels is not None

    def forward(self, x, edge_index):
        for i, c in enumerate(self.conv):
            if i % 2 == 0:
                x = c(x, edge_index)
            elif isinstance(x, dict):
                x = {k: c(v) for k, v in x.items()}
            else:
                x = c(x)
        if isinstance(x, dict):
            x = x[list(x.keys())[0]]
        for l in self.fc:
            x = l(x)
        return x


class HeteroSage(nn.Module):
    """Multi-node-type [HeteroConv(SAGEConv) -> ReLU]* + Linear head on the first output node
    type (the reference's multi-type arch layout, tests/test_utils.py:164-182, with SAGEConv in
    place of GATConv — the shim restates SAGE; bipartite relations take (F_src, F_dst) inputs)."""

    def __init__(self, rels, in_dims, hidden, n_layers, fc_dims):
        super().__init__()
        convs = []
        for li in range(n_layers):
            convs.append(HeteroConv({r: SAGEConv((in_dims[r[0]], in_dims[r[-1]]) if li == 0
                                                 else (hidden, hidden), hidden) for r in rels},
                                    aggr="sum"))
            convs.append(nn.ReLU())
        self.conv = nn.ModuleList(convs)
        fcs = []
        for i in range(len(fc_dims) - 1):
            fcs.append(Linear(fc_dims[i], fc_dims[i + 1]))
            fcs.append(nn.Sigmoid() if i == len(fc_dims) - 2 else nn.ReLU())
        self.fc = nn.ModuleList(fcs)

    def forward(self, x, edge_index):
        for i, c in enumerate(self.conv):
            x = c(x, edge_index) if i % 2 == 0 else {k: c(v) for k, v in x.items()}
        x = x[list(x.keys())[0]]
        for l in self.fc:
            x = l(x)
        return x


class HeteroGat(nn.Module):
    """The reference's multi-type test arch (tests/test_utils.py:86-182: HeteroConv of
    GATConv(.., add_self_loops=False) per relation, sum, -> ReLU, then Linear layers on the first
    output node type) with explicit input widths and `heads` per layer (concatenated)."""

    def __init__(self, rels, in_dims, hidden, heads, fc_dims):
        super().__init__()
        convs, width = [], None
        for li, h in enumerate(heads):
            convs.append(HeteroConv({r: GATConv((in_dims[r[0]], in_dims[r[-1]]) if li == 0
                                                else (width, width), hidden, heads=h,
                                                add_self_loops=False) for r in rels},
                                    aggr="sum"))
            convs.append(nn.ReLU())
            width = hidden * h
        self.conv = nn.ModuleList(convs)
        fcs = []
        for i in range(len(fc_dims) - 1):
            fcs.append(Linear(fc_dims[i], fc_dims[i + 1]))
            fcs.append(nn.Sigmoid() if i == len(fc_dims) - 2 else nn.ReLU())
        self.fc = nn.ModuleList(fcs)

    def forward(self, x, edge_index):
        for i, c in enumerate(self.conv):
            x = c(x, edge_index) if i % 2 == 0 else {k: c(v) for k, v in x.items()}
        x = x[list(x.keys())[0]]
        for l in self.fc:
            x = l(x)
        return x


def load_ckpt(name):
    sd = torch.load(os.path.join(REF_DATA, name), weights_only=True, map_location="cpu")["model"]
    return {k: v.clone() for k, v in sd.items()}


# ----------------------------------------------------------------------------- recording
class Recorder:
    def __init__(self):
        self.repeats = []  # one dict per mask_generator call
        self.cur = None

    def install(self):
        rec = self
        orig_mg = PeMask.mask_generator
        orig_ko = pe_wlm.kernel_output
        orig_tm = pe_explainer.train_model

        def mask_generator(self_):
            loader, rows = orig_mg(self_)
            full = loader.dataset.clone()
            rec.cur = {"mask": full.cpu().numpy().astype(bool),
                       "pathway_rows": None if rows is None else rows.cpu().numpy(),
                       "batch_size": loader.batch_size, "kernels": [], "outputs": []}
            rec.repeats.append(rec.cur)
            return loader, rows

        def kernel_output(mask, *a, **kw):
            k, out = orig_ko(mask, *a, **kw)
            rec.cur["kernels"].append(k.detach().cpu().numpy().astype(np.float64))
            rec.cur["outputs"].append(out.detach().cpu().numpy().astype(np.float32).reshape(-1))
            return k, out

        def train_model(loader, params, feat, ei, lin, *a, **kw):
            rec.cur["w0"] = lin.layer.weight.detach().cpu().numpy().reshape(-1).copy()
            res = orig_tm(loader, params, feat, ei, lin, *a, **kw)
            rec.cur["w_final"] = res[0][0].detach().cpu().numpy().reshape(-1).copy()
            rec.cur["losses"] = np.asarray(res[1], dtype=np.float64)
            rec.cur["best_epoch"] = int(res[2])
            return res

        PeMask.mask_generator = mask_generator
        pe_wlm.kernel_output = kernel_output
        pe_explainer.train_model = train_model
        self._orig = (orig_mg, orig_ko, orig_tm)

    def uninstall(self):
        PeMask.mask_generator, pe_wlm.kernel_output, pe_explainer.train_model = self._orig


def tensor_dict_to_np(prefix, d, out):
    if isinstance(d, dict):
        keys = list(d.keys())
        out[prefix + "__keys"] = np.array(["|".join(k) if isinstance(k, tuple) else k
                                           for k in keys])
        for i, k in enumerate(keys):
            out[f"{prefix}__{i}"] = d[k].cpu().numpy()
    else:
        out[prefix] = d.cpu().numpy()


def run_case(name, feat, edge_index, arch, params, names, pathways=None, pathway_names=None,
             element_type=None, problem="node_prediction", element="0", times=1,
             state_dict=None, arch_spec=None):
    out = {}
    meta = {"name": name, "problem": problem, "element": element, "times": times,
            "params": params, "names": names, "pathways": pathways,
            "pathway_names": pathway_names, "element_type": element_type,
            "arch_spec": arch_spec}
    tensor_dict_to_np("feat", feat, out)
    tensor_dict_to_np("edge_index", edge_index, out)
    for k, v in (state_dict or arch.state_dict()).items():
        out["w__" + k] = v.detach().cpu().numpy()
    out["rng_state"] = torch.get_rng_state().numpy()

    rec = Recorder()
    rec.install()
    try:
        exp = pe.Explainer(feat, edge_index, arch, params, names,
                           None if pathways is None else [list(p) for p in pathways],
                           pathway_names, element_type, problem=problem)
        df, pdf = exp.run(element, times)
    finally:
        rec.uninstall()

    meta["n_repeats"] = len(rec.repeats)
    for i, r in enumerate(rec.repeats):
        m = r["mask"]
        out[f"r{i}_mask_bits"] = np.packbits(m, axis=1, bitorder="little")
        out[f"r{i}_mask_shape"] = np.array(m.shape)
        if r["pathway_rows"] is not None:
            out[f"r{i}_pathway_rows"] = r["pathway_rows"]
        out[f"r{i}_kernel"] = np.concatenate(r["kernels"])
        out[f"r{i}_output"] = np.concatenate(r["outputs"])
        out[f"r{i}_w0"] = r["w0"]
        out[f"r{i}_w_final"] = r["w_final"]
        out[f"r{i}_losses"] = r["losses"]
        meta[f"r{i}_batch_size"] = r["batch_size"]
        meta[f"r{i}_best_epoch"] = r["best_epoch"]
    meta["df"] = {"index": [str(x) for x in df.index.tolist()],
                  "config_value_mean": df["config_value_mean"].astype(float).tolist(),
                  "config_value_std": df["config_value_std"].astype(float).tolist()}
    if pdf is not None:
        meta["pathway_df"] = {"index": [str(x) for x in pdf.index.tolist()],
                              "score": pdf["score"].astype(float).tolist()}
    else:
        meta["pathway_df"] = None
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    with open(os.path.join(HERE, name + ".json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"[golden] {name}: repeats={len(rec.repeats)} rows={rec.repeats[0]['mask'].shape}"
          f" df={len(df)} pdf={None if pdf is None else len(pdf)}")


# ----------------------------------------------------------------------------- cases
TEST_RUN_EDGES = None  # filled from the fixture file below


def case_test_run(times, name):
    """tests/test_explainer.py:303-647 fixture: 36x84 graph, 4 communities, query '10',
    gcn_homo_1hop checkpoint."""
    ei = np.load(os.path.join(HERE, "inputs_test_run_edges.npy"))
    torch.manual_seed(2)  # == set_seed(0): torch seed + 2
    feat = torch.randn((36, 84))
    arch = ConvStack("gcn", [84, 16], [16, 16, 32, 1])
    arch.load_state_dict(load_ckpt("gcn_homo_1hop_lungCancer.pth.tar"))
    arch.eval()
    pathways = [list(range(0, 11)), [10] + list(range(11, 19)),
                [10] + list(range(19, 28)), [10] + list(range(28, 36))]
    names = [str(i) for i in range(36)]
    torch.manual_seed(1234)
    run_case(name, feat, torch.tensor(ei, dtype=torch.long), arch, dict(PARAMS), names,
             pathways, ["west", "north", "south", "east"], problem="node", element="10",
             times=times, arch_spec={"kind": "gcn", "dims": [84, 16], "fc": [16, 16, 32, 1]})


def case_hetero_single():
    """gcn_hetero_1hop checkpoint on a single-node-type, 3-relation synthetic graph."""
    g = torch.Generator().manual_seed(11)
    n = 60
    rels = [("gene", "interacts", "gene"), ("gene", "modifies", "gene"),
            ("gene", "regulates", "gene")]
    feat = {"gene": torch.randn((n, 84), generator=g)}
    ei = {r: torch.randint(0, n, (2, 90 + 10 * i), generator=g) for i, r in enumerate(rels)}
    arch = ConvStack("gcn", [84, 16], [16, 16, 32, 1], hetero_rels=rels)
    arch.load_state_dict(load_ckpt("gcn_hetero_1hop_lungCancer.pth.tar"))
    arch.eval()
    names = {"gene": [f"g{i}" for i in range(n)]}
    pathways = [[f"g{i}" for i in range(0, 20)], [f"g{i}" for i in range(15, 40)],
                [f"g{i}" for i in range(35, 60)]]
    torch.manual_seed(77)
    run_case("hetero_single", feat, ei, arch, dict(PARAMS, interpret_samples=16, epochs=12),
             names, pathways, ["pa", "pb", "pc"], element_type="gene", problem="node",
             element="g5", times=2,
             arch_spec={"kind": "gcn", "dims": [84, 16], "fc": [16, 16, 32, 1],
                        "hetero_rels": [list(r) for r in rels]})


HM_RELS = [("A", "ab", "B"), ("B", "ba", "A"), ("A", "aa", "A"), ("C", "ca", "A"),
           ("A", "ac", "C")]
HM_SIZES = {"A": 50, "B": 30, "C": 20}
HM_DIMS = {"A": 8, "B": 6, "C": 5}


def case_hetero_multi():
    """Three node types with different feature widths (padded by hetero2homo), five relations
    (three bipartite), 2-layer HeteroConv(SAGEConv) — the multi-node-type path
    (model.py:118-253, including quirk Q4: the per-copy outputs re-cut by
    extract_node_edge_output)."""
    g = torch.Generator().manual_seed(41)
    feat = {t: torch.randn((n, HM_DIMS[t]), generator=g) for t, n in HM_SIZES.items()}
    ei = {r: torch.stack([torch.randint(0, HM_SIZES[r[0]], (m,), generator=g),
                          torch.randint(0, HM_SIZES[r[-1]], (m,), generator=g)])
          for r, m in zip(HM_RELS, (60, 50, 70, 30, 30))}
    torch.manual_seed(12)
    arch = HeteroSage(HM_RELS, HM_DIMS, 16, 2, [16, 8, 1])
    arch.eval()
    names = {t: [f"{t.lower()}{i}" for i in range(n)] for t, n in HM_SIZES.items()}
    torch.manual_seed(5)
    run_case("hetero_multi", feat, ei, arch, dict(PARAMS, interpret_samples=16, epochs=4),
             names, None, None, element_type="B", problem="node", element="b2", times=2,
             arch_spec={"kind": "hetero_sage", "rels": [list(r) for r in HM_RELS],
                        "sizes": HM_SIZES, "in_dims": HM_DIMS, "hidden": 16, "layers": 2,
                        "fc": [16, 8, 1]})


def case_hetero_gat():
    """The multi-node-type path with the reference's own conv family (GATConv, tests/test_utils.py
    :86-182): the hetero_multi graph (3 node types, 5 relations incl. the same-type 'aa', whose
    conv gets a Tensor input), 2-layer HeteroConv(GAT) with 2 then 1 heads, add_self_loops=False.
    GAT numerics come from the shim's PyG 2.0.4 restatement (parity pinned to it, as for GCN /
    SAGE)."""
    g = torch.Generator().manual_seed(41)
    feat = {t: torch.randn((n, HM_DIMS[t]), generator=g) for t, n in HM_SIZES.items()}
    ei = {r: torch.stack([torch.randint(0, HM_SIZES[r[0]], (m,), generator=g),
                          torch.randint(0, HM_SIZES[r[-1]], (m,), generator=g)])
          for r, m in zip(HM_RELS, (60, 50, 70, 30, 30))}
    torch.manual_seed(13)
    arch = HeteroGat(HM_RELS, HM_DIMS, 8, [2, 1], [8, 4, 1])
    arch.eval()
    names = {t: [f"{t.lower()}{i}" for i in range(n)] for t, n in HM_SIZES.items()}
    torch.manual_seed(6)
    run_case("hetero_gat", feat, ei, arch, dict(PARAMS, interpret_samples=16, epochs=4),
             names, None, None, element_type="B", problem="node", element="b2", times=2,
             arch_spec={"kind": "hetero_gat", "rels": [list(r) for r in HM_RELS],
                        "sizes": HM_SIZES, "in_dims": HM_DIMS, "hidden": 8, "heads": [2, 1],
                        "layers": 2, "fc": [8, 4, 1]})


def case_sage_shapley():
    g = torch.Generator().manual_seed(5)
    n, e = 300, 1500
    feat = torch.randn((n, 16), generator=g)
    ei = torch.randint(0, n, (2, e), generator=g)
    torch.manual_seed(3)
    arch = ConvStack("sage", [16, 16, 16], [16, 1])
    arch.eval()
    names = [f"n{i}" for i in range(n)]
    run_case("sage_shapley", feat, ei, arch, dict(PARAMS, interpret_samples=24, epochs=10),
             names, None, None, problem="node_prediction", element="n7", times=1,
             arch_spec={"kind": "sage", "dims": [16, 16, 16], "fc": [16, 1]})


def case_gcn2_graph():
    g = torch.Generator().manual_seed(8)
    n, e = 40, 160
    feat = torch.randn((n, 12), generator=g)
    ei = torch.randint(0, n, (2, e), generator=g)
    torch.manual_seed(4)
    arch = ConvStack("gcn", [12, 8, 8], [8, 8, 1])
    arch.eval()
    names = [str(i) for i in range(n)]
    pathways = [[0, 1, 2, 3, 4, 5], [5, 6, 7, 8, 9, 10, 11, 12], list(range(20, 40))]
    torch.manual_seed(99)
    run_case("gcn2_graph", feat, ei, arch, dict(PARAMS, interpret_samples=10, epochs=8),
             names, pathways, ["a", "b", "c"], problem="graph_prediction", element="3",
             times=2, arch_spec={"kind": "gcn", "dims": [12, 8, 8], "fc": [8, 8, 1]})


def case_toy():
    """examples/toy_example-caseA.ipynb cells 5/9/13/15 graph + model shape (random init)."""
    ei = torch.tensor([[0, 1], [1, 0], [1, 2], [2, 1], [1, 3], [3, 1], [1, 4], [4, 1]]).T
    torch.manual_seed(2)
    feat = torch.randn((5, 16))
    torch.manual_seed(0)
    arch = ConvStack("gcn", [16, 16, 8, 8], [8, 8, 16, 1])
    arch.eval()
    names = [str(i) for i in range(5)]
    torch.manual_seed(2)
    run_case("toy", feat, ei, arch, dict(PARAMS, seed=0), names, [[0], [2, 3, 4]],
             ["blue", "red"], problem="node_prediction", element="1", times=3,
             arch_spec={"kind": "gcn", "dims": [16, 16, 8, 8], "fc": [8, 8, 16, 1]})


def case_gcn2_medium():
    """c2-shaped (2-layer GCN 64->64->64->1) on a scaled-down random graph."""
    g = torch.Generator().manual_seed(21)
    n, e = 2000, 20000
    feat = torch.randn((n, 64), generator=g)
    ei = torch.randint(0, n, (2, e), generator=g)
    torch.manual_seed(6)
    arch = ConvStack("gcn", [64, 64, 64], [64, 1])
    arch.eval()
    names = [str(i) for i in range(n)]
    run_case("gcn2_medium", feat, ei, arch, dict(PARAMS, interpret_samples=8, epochs=10),
             names, None, None, problem="node_prediction", element="7", times=1,
             arch_spec={"kind": "gcn", "dims": [64, 64, 64], "fc": [64, 1]})


def case_kernels():
    """Kernel.compute on exact (M<=1000) and approximate (M>1000) paths (kernels.py:115-174)."""
    out = {}
    g = torch.Generator().manual_seed(31)
    for cols in (9, 200, 1001, 1002, 1500, 3000, 20000):
        m = torch.rand((64, cols), generator=g) < torch.rand((64, 1), generator=g)
        m[0] = False
        m[1] = True
        if cols > 5:
            m[2] = False
            m[2, :1] = True
        k = PeKernel(m).compute()
        out[f"c{cols}_mask_bits"] = np.packbits(m.numpy(), axis=1, bitorder="little")
        out[f"c{cols}_kernel"] = k.numpy().astype(np.float64)
    np.savez_compressed(os.path.join(HERE, "kernels.npz"), **out)
    print("[golden] kernels")


def extract_test_run_edges():
    """Pull the 2x122 edge-index literal of test_run (tests/test_explainer.py:320-562) out of the
    reference test file as DATA (ast literal evaluation; no reference code is executed)."""
    import ast

    src = open("/root/reference/tests/test_explainer.py").read()
    tree = ast.parse(src)
    for node in ast.walk(tree):
        if isinstance(node, ast.FunctionDef) and node.name == "test_run":
            for sub in ast.walk(node):
                if (isinstance(sub, ast.Assign) and isinstance(sub.targets[0], ast.Name)
                        and sub.targets[0].id == "mock_edge_index"):
                    lit = ast.literal_eval(sub.value.args[0])
                    arr = np.asarray(lit, dtype=np.int64)
                    np.save(os.path.join(HERE, "inputs_test_run_edges.npy"), arr)
                    return arr
    raise RuntimeError("edge literal not found")


if __name__ == "__main__":
    if len(sys.argv) > 1:  # regenerate selected cases only: make_golden.py hetero_multi ...
        for c in sys.argv[1:]:
            globals()["case_" + c]()
        sys.exit(0)
    extract_test_run_edges()
    case_kernels()
    case_test_run(3, "test_run")
    case_test_run(1, "test_run_t1")
    case_toy()
    case_hetero_single()
    case_sage_shapley()
    case_gcn2_graph()
    case_gcn2_medium()
    case_hetero_multi()
    case_hetero_gat()
