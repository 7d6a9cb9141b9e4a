"""Benchmark: perturbation-samples/s of the XP-GNN hot path on MI355X (BASELINE.json metric).

Workload (configs[1] of BASELINE.json, "c2"): synthetic homogeneous graph, 100k nodes / 1M
edges, 64-dim fp32 features, 2-layer GCN 64->64->64 + Linear(64->1) + sigmoid (random init),
interpret_samples=256, epochs=50 -> 12,800 mask rows per repeat, query node 7 (node_prediction:
its 3-hop computational subgraph, as the reference extracts it).

One step = one full repeat of the hot path per rank, inputs resident in HBM:
  device mask sampling (Philox Shapley rows) -> masked receptive-field forward (all rows) ->
  KernelSHAP weights -> surrogate Adam loop (ceil(R / (R // epochs)) steps) ->
  (N > 1) all-gather of the per-repeat weights for the mean/std over repeats.
Repeats are independent, so ranks shard repeats (weak scaling, one repeat per rank per step).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "perturbation-samples/sec (masked GNN fwd) per query node; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--nodes", type=int, default=100_000)
    p.add_argument("--edges", type=int, default=1_000_000)
    p.add_argument("--feat", type=int, default=64)
    p.add_argument("--interpret-samples", type=int, default=256)
    p.add_argument("--epochs", type=int, default=50)
    p.add_argument("--query", type=int, default=7)
    p.add_argument("--repeats", type=int, default=1,
                   help="Explainer.run(times=...) repeats per rank per step (batched fits)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-rows", type=int, default=12800)
    p.add_argument("--full-graph-rows", type=int, default=64,
                   help="regime (ii): mask rows of the c3-shaped full-graph forward (0 = skip)")
    p.add_argument("--no-hetero", action="store_true", help="skip the c4 multi-type section")
    p.add_argument("--no-communities", action="store_true",
                   help="skip the c2 community-sampler section")
    p.add_argument("--no-graph-prediction", action="store_true",
                   help="skip the c3 graph_prediction per-query pipeline section")
    return p.parse_args()


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def build_workload(args, dev):
    from bikg_graph_explainability_public_amd import pipeline
    from bikg_graph_explainability_public_amd.data import Data
    from bikg_graph_explainability_public_amd.nn import ConvStack

    g = torch.Generator().manual_seed(0)
    feat = torch.randn((args.nodes, args.feat), generator=g)
    ei = torch.randint(0, args.nodes, (2, args.edges), generator=g)
    torch.manual_seed(0)
    arch = ConvStack("gcn", [args.feat, 64, 64], [64, 1]).eval().to(dev)
    data = Data(feat.to(dev), ei.to(dev))
    names = [str(i) for i in range(args.nodes)]
    sub_feat, sub_ei, _, sub_ind, _, _ = data.comp_graph(args.query, 2, "node", names)
    q = int(sub_ind.reshape(-1)[0])
    plan = pipeline.build_plan(arch, sub_feat, sub_ei, [q])
    return arch, sub_feat, sub_ei, q, plan


def forward_bytes(plan, rows):
    """Algorithmic HBM bytes of the masked forward per launch chain: per row,
    per layer: CSR pointers + columns of the targets, the row's mask words, the gathered
    source rows of kept edges + self rows (F_out wide, layer-1 tables), the written outputs."""
    arr = plan.arrays
    W = (plan.cols + 31) // 32
    b = 4 * (plan.n0 + 1) + 4 * arr["deg_src"].size + 4 * W  # degree pass
    for li, conv in enumerate(plan.program.convs):
        lay = arr["layers"][li]
        n_t = arr["frontiers"][li + 1].size
        e = lay["agg_src"].size
        width = conv.f_out if li == 0 else conv.f_in
        b += 4 * (n_t + 1) + 8 * e + 4 * width * (0.25 * e + n_t) + 4 * conv.f_out * n_t
    return b * rows


def wlm_bytes(rows, cols, batch):
    W = (cols + 31) // 32
    return rows * W * 4 + rows * (4 + 8) + cols * 4 * 6 + 8 * math.ceil(rows / batch)


def pmc_traffic(kernels, args):
    """HBM bytes per launch of the dominant launch chain from the committed PMC passes
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py from rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE runs of this bench at its default configuration), or None."""
    fn = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    default = (args.nodes, args.edges, args.feat, args.interpret_samples, args.epochs,
               args.repeats) == (100_000, 1_000_000, 64, 256, 50, 1)
    if not default or not os.path.exists(fn):
        return None, None
    data = json.load(open(fn))
    tot, hit = 0.0, False
    for name, d in data.items():
        if name.startswith(kernels) and d.get("traffic_bytes") is not None:
            tot += d["traffic_bytes"]
            hit = True
    return (tot if hit else None), ("profiles/pmc_traffic.json (2 x FETCH_SIZE + WRITE_SIZE, "
                                    "summed over the chain's kernels)" if hit else None)


def pmc_traffic_counts(counts):
    """HBM bytes of one operation = sum over kernels of (dispatches per operation) x (measured
    bytes per dispatch) from profiles/pmc_traffic.json (2 x FETCH_SIZE + WRITE_SIZE of this bench's
    default run, tools/pmc_traffic.py), or None when a kernel is missing."""
    fn = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(fn):
        return None
    data = json.load(open(fn))
    tot = 0.0
    for prefix, n in counts.items():
        hits = [d["traffic_bytes"] for name, d in data.items()
                if name.startswith(prefix) and d.get("traffic_bytes") is not None]
        if not hits:
            return None
        tot += n * sum(hits) / len(hits)
    return tot


def cpu_baseline(args, arch, sub_feat, sub_ei, q):
    """The numpy oracle (CPU restatement of the reference path, 1 thread) on a bounded sample
    of the same workload: cpu_rows mask rows through forward + KernelSHAP + surrogate."""
    import oracle
    try:
        from threadpoolctl import threadpool_limits
    except Exception:  # pragma: no cover
        threadpool_limits = None
    S = sub_feat.shape[0]
    rows = args.cpu_rows
    rng = np.random.default_rng(0)
    m = rng.random((rows, S)) < 0.5
    spec = {"convs": [{"kind": "gcn", "rels": [None], "act": "relu",
                       "params": {None: {"W": arch.conv[2 * i].lin.weight.detach().cpu().numpy(),
                                         "b": arch.conv[2 * i].bias.detach().cpu().numpy()}}}
                      for i in range(2)],
            "fc": [{"W": arch.fc[0].weight.detach().cpu().numpy(),
                    "b": arch.fc[0].bias.detach().cpu().numpy(), "act": "sigmoid"}]}
    x = sub_feat.cpu().numpy()
    e = {None: sub_ei.cpu().numpy()}
    ctx = threadpool_limits(limits=1) if threadpool_limits else None
    try:
        t0 = time.perf_counter()
        y = oracle.masked_query_outputs(spec, x, e, m, q, dtype=np.float32)
        k = oracle.shap_kernel(m)
        oracle.train_wlm(m, args.interpret_samples, y, k, np.zeros(S, np.float32),
                         {"lr": 0.01, "l1_lambda": 1e-4}, dtype=np.float32)
        dt = time.perf_counter() - t0
    finally:
        if ctx is not None:
            ctx.unregister() if hasattr(ctx, "unregister") else None
    return {"value": rows / dt, "unit": "samples/s", "cores": 1, "kind": "port",
            "sample": f"{rows} mask rows of the same workload (S={S}) through the numpy oracle "
                      f"(union-graph forward + KernelSHAP + surrogate fit), {dt:.1f} s"}


def c3_graph(dev, nodes=1_000_000, edges=10_000_000, feat=128, seed=0):
    """synthetic homogeneous graph, 2-layer SAGEConv(mean) 128-128-128, head
    Linear(128, 1) + sigmoid (random init, ConvStack layout of the reference tests)."""
    from bikg_graph_explainability_public_amd.nn import ConvStack
    g = torch.Generator().manual_seed(seed)
    x = torch.randn((nodes, feat), generator=g)
    ei = torch.randint(0, nodes, (2, edges), generator=g)
    torch.manual_seed(seed)
    arch = ConvStack("sage", [feat, feat, feat], [feat, 1]).eval()
    return x, ei, arch


def full_graph_bytes(n, e_kept_per_row, e, f_in, f_out, rows, layers=2):
    """SURVEY.md §8d algorithmic bytes per sample of the full-graph masked forward, summed over
    the rows: per layer 4(N+1) + 4E (CSR) + N/8 (mask bits) + 4 F_g E_kept (gathered rows,
    F_g = min(F_in, F_out)) + 4 F_root N (SAGE self rows) + 4 F_out N (layer output)."""
    per_layer_fixed = 4 * (n + 1) + 4 * e + n / 8 + 4 * f_in * n + 4 * f_out * n
    return layers * (per_layer_fixed * rows + 4 * min(f_in, f_out) * e_kept_per_row.sum())


def full_graph_section(args, dev):
    """Regime (ii): every node a target of the masked forward on the c3 graph
    (1M nodes / 10M edges / 128 features / 2-layer SAGE), `rows` mask rows (32-sample passes)."""
    from bikg_graph_explainability_public_amd import engine, pipeline
    x, ei, arch = c3_graph(dev)
    N, E = x.shape[0], ei.shape[1]
    xd, eid = x.to(dev), ei.to(dev)
    arch = arch.to(dev)
    plan = pipeline.build_plan(arch, xd, eid, list(range(N)))
    rows = args.full_graph_rows
    bits = engine.sample_shapley(77, rows, N, dev)
    y = plan.forward(bits)  # warm-up (workspace, code objects)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 3
    a.record(stream)
    for _ in range(reps):
        y = plan.forward(bits)
    b.record(stream)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    # kept edges per row (both endpoints active), for the algorithmic byte count
    m = engine.unpack_masks(bits, N)
    kept = (m[:, eid[0]] & m[:, eid[1]]).sum(1).double().cpu().numpy()
    del m
    bytes_ = full_graph_bytes(N, kept, E, 128, 128, rows)
    flops = rows * N * 2.0 * (2 * 128 * 128 + 128)  # layer-2 dense (l and r) + head, per target
    achieved = bytes_ / (ms * 1e-3) / 1e9
    passes = -(-rows // 32)
    traffic = pmc_traffic_counts({"k_wide_bits": passes, "k_wide_f0": passes,
                                  "k_wide_degree": passes, "k_wide_tgt<8, false": passes,
                                  "k_wide_tgt<8, true": passes}) if rows == 64 else None
    out = {
        "workload": "c3 full-graph masked forward (SURVEY.md §8d regime (ii)): 1M nodes / 10M "
                    "edges, 128 feats, 2-layer SAGEConv(mean) + Linear(128,1) + sigmoid, every "
                    "node a target (all 1M outputs per mask row)",
        "rows": rows, "ms": ms, "ms_per_row": ms / rows,
        "samples_per_s": rows / (ms * 1e-3),
        "node_outputs_per_s": rows * N / (ms * 1e-3),
        "roofline": {"kernel": "wide forward chain (k_wide_bits, k_wide_f0, k_wide_tgt<layer 1>, "
                               "k_wide_tgt<layer 2 + head>)",
                     "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "bytes_per_launch": bytes_,
                     "traffic": traffic,
                     "traffic_source": "profiles/pmc_traffic.json" if traffic else None,
                     "bytes_formula": "SURVEY.md §8d B_alg per sample, E_kept measured per row"},
        "mfma": {"tflops": flops / (ms * 1e-3) / 1e12, "peak_fp32_tflops": 157.3,
                 "frac": flops / (ms * 1e-3) / 1e12 / 157.3},
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = full_graph_cpu(arch)
    return out


def full_graph_cpu(arch):
    """The numpy oracle (1 thread) on ONE mask row of the same model on a 1/10-scale c3 graph
    (100k nodes / 1M edges, same degree and widths): the forward is linear in N and E, so the
    per-sample rate at full scale is the measured one / 10 (reported as such)."""
    import oracle
    try:
        from threadpoolctl import threadpool_limits
    except Exception:  # pragma: no cover
        threadpool_limits = None
    x, ei, _ = c3_graph("cpu", nodes=100_000, edges=1_000_000)
    sd = {k: v.detach().cpu().numpy() for k, v in arch.state_dict().items()}
    spec = {"convs": [{"kind": "sage", "rels": [None], "act": "relu",
                       "params": {None: {"Wl": sd[f"conv.{2 * i}.lin_l.weight"],
                                         "bl": sd[f"conv.{2 * i}.lin_l.bias"],
                                         "Wr": sd[f"conv.{2 * i}.lin_r.weight"]}}}
                      for i in range(2)],
            "fc": [{"W": sd["fc.0.weight"], "b": sd["fc.0.bias"], "act": "sigmoid"}]}
    rng = np.random.default_rng(0)
    m = rng.random(x.shape[0]) < 0.5
    e = ei.numpy()
    keep = m[e[0]] & m[e[1]]
    ctx = threadpool_limits(limits=1) if threadpool_limits else None
    try:
        t0 = time.perf_counter()
        oracle.forward_union(spec, x.numpy(), {None: (e[0][keep], e[1][keep])}, dtype=np.float32)
        dt = time.perf_counter() - t0
    finally:
        if ctx is not None and hasattr(ctx, "unregister"):
            ctx.unregister()
    return {"value": 1.0 / (dt * 10), "unit": "samples/s", "cores": 1, "kind": "port",
            "sample": f"1 mask row through the numpy oracle on a 1/10-scale c3 graph (100k nodes / "
                      f"1M edges) in {dt:.1f} s; full-scale rate = 1 / (10 x {dt:.1f} s)"}


def graph_prediction_section(args, dev):
    """The reference's graph_prediction semantics on the c3 graph (explainer.py:427-447: no
    subgraph, S = N = 1M mask columns) for one query node, one repeat of interpret_samples=512,
    epochs=50 (25,600 rows): device sampler with fused row counts -> receptive-field forward ->
    KernelSHAP -> many-column surrogate fit (k_gw_*: streams the step's mask bits twice)."""
    from bikg_graph_explainability_public_amd import engine, pipeline
    x, ei, arch = c3_graph(dev)
    N = x.shape[0]
    plan = pipeline.build_plan(arch.to(dev), x.to(dev), ei.to(dev), [7])
    R, epochs = 512 * 50, 50
    batch = R // epochs
    w0 = torch.zeros(N, device=dev)
    params = {"lr": 0.01, "l1_lambda": 1e-4}
    stream = torch.cuda.current_stream()

    def rep(i, ev=None):
        if ev:
            ev[0].record(stream)
        bits, cnt = engine.sample_shapley(500 + i, R, N, dev, with_counts=True)
        if ev:
            ev[1].record(stream)
        y = plan.forward(bits)[:, 0]
        if ev:
            ev[2].record(stream)
        k = engine.shap_kernel(bits, N, counts=cnt)
        if ev:
            ev[3].record(stream)
        engine.wlm_fit(bits, N, batch, y, k, w0, params)
        if ev:
            ev[4].record(stream)

    rep(0)
    torch.cuda.synchronize()
    reps = 3
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(reps)]
    for i in range(reps):
        rep(1 + i, evs[i])
    torch.cuda.synchronize()
    ph = {name: float(np.mean([e[j].elapsed_time(e[j + 1]) for e in evs]))
          for j, name in enumerate(("sample", "forward", "shap", "wlm"))}
    total = sum(ph.values())
    W = (N + 31) // 32
    wbytes = 2 * R * W * 4 + epochs * 6 * N * 4  # mask bits twice per step + Adam state r/w
    traffic = pmc_traffic_counts({"k_gw_p": epochs, "k_gw_g": epochs, "k_gw_grad": epochs,
                                  "k_gw_loss": 1})
    return {"workload": "c3 graph_prediction, one query (node 7), S = 1M mask columns, "
                        "interpret_samples=512 x epochs=50 = 25,600 rows, one repeat",
            "ms_per_repeat": total, "samples_per_s": R / (total * 1e-3), "phases_ms": ph,
            "roofline": {"kernel": "many-column surrogate fit (k_wlm_stats, k_gw_p, k_gw_g, "
                                   "k_gw_grad, k_gw_loss)", "bound": "hbm",
                         "achieved": wbytes / (ph["wlm"] * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s",
                         "frac": wbytes / (ph["wlm"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "bytes_per_launch": wbytes, "traffic": traffic,
                         "traffic_source": "profiles/pmc_traffic.json" if traffic else None,
                         "bytes_formula": "2 x R x ceil(S/32) x 4 (bits, p and grad passes) + "
                                          "steps x 24 S (w, m, v read + write)"},
            "sampler_GBps": R * W * 4 / (ph["sample"] * 1e-3) / 1e9}


C4_RELS = [("gene", "interacts", "gene"), ("gene", "encodes", "protein"),
           ("protein", "binds", "protein"), ("drug", "targets", "protein"),
           ("protein", "regulates", "gene")]


def hetero_c4_section(args, dev):
    """c4 (BASELINE.json configs[3]): 3 node types (200k gene / 200k protein / 100k drug,
    84 / 64 / 32 features), 5 relations (3 bipartite), 5M edges, one HeteroConv(SAGE) layer
    (gcn_hetero_1hop shape: 84 -> 16, head 16 -> 16 -> 32 -> 1; GCNConv cannot take bipartite
    relations), node_prediction of gene 7 through Explainer's host steps (hetero2homo, k-hop
    subgraph on the GPU), then per repeat: device Shapley masks -> node-type-gated forward ->
    empty-copy / Q4 targets -> KernelSHAP -> surrogate fit.  Regime (i): the subgraph is
    cache-resident, so samples/s is the figure (no HBM fraction).  `reference_loop` times the
    reference's own per-copy multi-type loop (model.py:196-249, one arch call + host sync per
    row) on the same GPU for one batch."""
    from bikg_graph_explainability_public_amd import engine, pipeline
    from bikg_graph_explainability_public_amd.data import Data
    from bikg_graph_explainability_public_amd.model import Model
    from bikg_graph_explainability_public_amd.nn import HeteroSageStack
    sizes = {"gene": 200_000, "protein": 200_000, "drug": 100_000}
    dims = {"gene": 84, "protein": 64, "drug": 32}
    g = torch.Generator(device=dev).manual_seed(4)
    feat = {t: torch.randn((n, dims[t]), generator=g, device=dev) for t, n in sizes.items()}
    ei = {r: torch.stack([torch.randint(0, sizes[r[0]], (1_000_000,), generator=g, device=dev),
                          torch.randint(0, sizes[r[-1]], (1_000_000,), generator=g, device=dev)])
          for r in C4_RELS}
    torch.manual_seed(0)
    arch = HeteroSageStack(C4_RELS, dims, 16, 1, [16, 16, 32, 1]).to(dev).eval()
    d = Data(feat, ei)
    fh, eh, nt, et, _, _, pads = d.hetero2homo()
    ntn, etn = list(feat), list(ei)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sub_x, sub_ei, _, sub_ind, sub_nt, sub_et = Data(fh, eh).comp_graph(
        7, 1, "node", [str(i) for i in range(fh.shape[0])], nt, et)
    torch.cuda.synchronize()
    t_khop = time.perf_counter() - t0
    sub_nt = sub_nt.long()
    q = int(sub_ind)  # gene = type 0 comes first in the sorted subset: position among genes
    plan = pipeline.build_plan(arch, sub_x, sub_ei, [q], sub_nt, sub_et, ntn, etn, pads)
    assert plan is not None and plan.multi_type
    S = sub_x.shape[0]
    R, epochs = 256 * 50, 50
    batch = R // epochs
    params = {"lr": 0.01, "l1_lambda": 1e-4}
    w0 = torch.zeros(S, device=dev)
    stream = torch.cuda.current_stream()

    def rep(i, ev=None):
        if ev:
            ev[0].record(stream)
        bits, cnt = engine.sample_shapley(900 + i, R, S, dev, with_counts=True)
        if ev:
            ev[1].record(stream)
        y = plan.forward(bits)[:, 0]
        empty = pipeline.empty_copy_rows(bits, S, sub_ei)
        y = pipeline.multi_type_targets(y, empty, batch, q, S, q4=False)
        if ev:
            ev[2].record(stream)
        k = engine.shap_kernel(bits, S, counts=cnt)
        if ev:
            ev[3].record(stream)
        engine.wlm_fit(bits, S, batch, y, k, w0, params)
        if ev:
            ev[4].record(stream)

    rep(0)
    torch.cuda.synchronize()
    reps = 5
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(reps)]
    t0 = time.perf_counter()
    for i in range(reps):
        rep(1 + i, evs[i])
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    ph = {name: float(np.mean([e[j].elapsed_time(e[j + 1]) for e in evs]))
          for j, name in enumerate(("sample", "forward", "shap", "wlm"))}
    # the reference's per-copy loop on the same GPU, one batch of rows
    mask = engine.unpack_masks(engine.sample_shapley(77, batch, S, dev), S)
    cf, cnt_t, pei, pet = Data(sub_x, sub_ei).perturbator(mask, "node", sub_nt, sub_et)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    Model(arch).predict_hetero_output(cf, pei.long(), cnt_t, pet, ntn, etn, batch, S, q, pads, "node")
    torch.cuda.synchronize()
    loop_rate = batch / (time.perf_counter() - t0)
    return {"workload": "c4: 3 node types (200k/200k/100k, 84/64/32 feats), 5 relations (3 "
                        "bipartite), 5M edges, HeteroConv(SAGE) 1 layer 84->16 + head "
                        "16->16->32->1, node_prediction of gene 7, interpret_samples=256 x "
                        "epochs=50 = 12,800 rows, one repeat, per-copy targets (hetero_q4=False)",
            "subgraph_nodes": S, "subgraph_edges": int(sub_ei.shape[1]),
            "khop_ms": t_khop * 1e3, "ms_per_repeat": wall * 1e3,
            "samples_per_s": R / wall, "phases_ms": ph,
            "reference_loop_gpu_samples_per_s": loop_rate}


def communities_section(args, dev, plan, sub_feat, sub_ei, reps=10):
    """c2 with 20 random communities over the subgraph (SURVEY.md §8d c5-style communities):
    the device community sampler (k_communities) inside the full repeat pipeline, and the
    compat CPU sampler (the reference's masks.py:262-397 algorithm and RNG order) beside it."""
    from bikg_graph_explainability_public_amd import engine
    from bikg_graph_explainability_public_amd.masks import Mask
    S = plan.cols
    rng = np.random.default_rng(20)
    cuts = np.sort(rng.choice(np.arange(1, S), 19, replace=False))
    pathways = [c.tolist() for c in np.split(rng.permutation(S), cuts)]
    params = {"interpret_samples": args.interpret_samples, "epochs": args.epochs}
    m = Mask(sub_feat, sub_ei, pathways, params, "node_prediction")
    cplan = m.community_plan()
    tabs = engine.community_tables(cplan, pathways, S, dev)
    R = cplan[2]
    batch = R // args.epochs
    w0 = torch.zeros((1, S), device=dev)
    fit = {"lr": 0.01, "l1_lambda": 1e-4}
    stream = torch.cuda.current_stream()

    def rep(i):
        bits, _ = engine.sample_communities(4000 + i, cplan, pathways, S, dev, tables=tabs)
        y = plan.forward(bits)[:, 0]
        k = engine.shap_kernel(bits, S)
        return engine.wlm_fit(bits.view(1, R, -1), S, batch, y.view(1, R), k.view(1, R), w0, fit)

    rep(0)
    torch.cuda.synchronize()
    a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    a.record(stream)
    for i in range(reps):
        engine.sample_communities(5000 + i, cplan, pathways, S, dev, tables=tabs)
    b.record(stream)
    for i in range(reps):
        rep(i)
    c.record(stream)
    torch.cuda.synchronize()
    samp_ms = a.elapsed_time(b) / reps
    rep_ms = b.elapsed_time(c) / reps
    t0 = time.perf_counter()
    Mask(sub_feat.cpu(), sub_ei.cpu(), [list(p) for p in pathways], params,
         "node_prediction").generate()
    cpu_ms = (time.perf_counter() - t0) * 1e3
    return {"workload": f"c2 subgraph ({S} cols), 20 random communities, {R} rows per repeat",
            "samples_per_s": R / (rep_ms * 1e-3), "ms_per_repeat": rep_ms,
            "sampler_ms": samp_ms,
            "sampler_write_GBps": R * ((S + 31) // 32) * 4 / (samp_ms * 1e-3) / 1e9,
            "cpu_compat_sampler_ms": cpu_ms, "cpu_sampler_cores": torch.get_num_threads()}


def graph_queries_section(args, dev, n=10_000, e=100_000, f=64, queries=8):
    """graph_prediction with several queries: `Explainer.run_queries` (one mask
    set per repeat shared by all queries) against the reference's usage, one `Explainer.run` per
    query, both through the public API end to end (host orchestration included), device
    sampler, synthetic graph, random-init 2-layer GCN + Linear head + sigmoid."""
    from bikg_graph_explainability_public_amd.explainer import Explainer
    from bikg_graph_explainability_public_amd.nn import ConvStack
    g = torch.Generator().manual_seed(3)
    feat = torch.randn((n, f), generator=g)
    ei = torch.randint(0, n, (2, e), generator=g)
    torch.manual_seed(3)
    arch = ConvStack("gcn", [f, f, f], [f, 1]).eval()
    params = {"seed": 1, "interpret_samples": args.interpret_samples, "epochs": args.epochs,
              "optimizer": "adam", "lr": 0.01, "lr_patience": 10, "l1_lambda": 1e-4,
              "mask_sampler": "device"}
    names = [str(i) for i in range(n)]
    exp = Explainer(feat.to(dev), ei.to(dev), arch, params, names,
                    problem="graph_prediction")
    els = [str(7 + 97 * i) for i in range(queries)]
    exp.run_queries(els[:2], 1)
    exp.run(els[0], 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    exp.run_queries(els, 1)
    torch.cuda.synchronize()
    t_shared = time.perf_counter() - t0
    t0 = time.perf_counter()
    for el in els:
        exp.run(el, 1)
    torch.cuda.synchronize()
    t_loop = time.perf_counter() - t0
    R = args.interpret_samples * args.epochs
    return {"workload": f"graph_prediction, {n} nodes / {e} edges, {f} feats, 2-layer GCN, "
                        f"{queries} queries x {R} rows, one repeat, device sampler",
            "run_queries_ms": t_shared * 1e3, "run_per_query_ms": t_loop * 1e3,
            "samples_per_s_shared": queries * R / t_shared,
            "samples_per_s_per_query_runs": queries * R / t_loop,
            "speedup": t_loop / t_shared}


def main():
    args = parse()
    world, rank, local = setup_dist(args)
    dev = torch.device("cuda", torch.cuda.current_device())
    from bikg_graph_explainability_public_amd import _lib, engine, sharding

    _lib.load()
    arch, sub_feat, sub_ei, q, plan = build_workload(args, dev)
    S = plan.cols
    R = args.interpret_samples * args.epochs
    batch = R // args.epochs
    params = {"lr": 0.01, "l1_lambda": 1e-4}
    stream = torch.cuda.current_stream()
    ev = {k: [] for k in ("sample", "forward", "shap", "wlm")}

    T = args.repeats
    w0 = torch.zeros((T, S), device=dev)

    def step(i, record):
        marks = [torch.cuda.Event(enable_timing=True) for _ in range(5)] if record else None
        if record:
            marks[0].record(stream)
        bits = engine.sample_shapley(1000 + i * world + rank, T * R, S, dev)
        if record:
            marks[1].record(stream)
        y = plan.forward(bits)[:, 0]
        if record:
            marks[2].record(stream)
        k = engine.shap_kernel(bits, S)
        if record:
            marks[3].record(stream)
        w, _, _, _, _ = engine.wlm_fit(bits.view(T, R, -1), S, batch, y.view(T, R),
                                       k.view(T, R), w0, params)
        if record:
            marks[4].record(stream)
            for j, name in enumerate(("sample", "forward", "shap", "wlm")):
                ev[name].append((marks[j], marks[j + 1]))
        if world > 1:
            # weight_stacking (explainer.py:288-314) over every rank's repeats: one all-gather
            w = sharding.gather_rows(w.reshape(T, S), T * world)
        return w.mean(0), w.std(0, unbiased=False)

    for i in range(args.warmup):
        step(i, False)
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    phase_ms = {k: float(np.mean([a.elapsed_time(b) for a, b in v])) for k, v in ev.items()}

    if rank == 0:
        total_rows = R * T * world * args.steps
        dominant = max(phase_ms, key=phase_ms.get)
        if dominant == "wlm":
            bytes_launch = wlm_bytes(R, S, batch) * T
            kname = "surrogate fit chain (k_wlm_stats, k_wlm_colbits, k_wlm_fit, k_wlm_loss)"
            kernels = ("k_wlm_stats", "k_wlm_colbits", "k_wlm_fit", "k_wlm_loss", "k_argmin_first")
        elif dominant == "forward":
            bytes_launch = forward_bytes(plan, R * T)
            kname = "masked forward chain (k_degree, k_agg, k_dense, k_take_col)"
            kernels = ("k_degree", "k_agg", "k_dense", "k_take_col", "k_fused_forward")
        elif dominant == "shap":
            bytes_launch = T * R * (((S + 31) // 32) * 4 + 12)
            kname = "k_popcount + k_shap"
            kernels = ("k_popcount", "k_shap")
        else:
            bytes_launch = T * R * ((S + 31) // 32) * 4
            kname = "k_shapley"
            kernels = ("k_shapley",)
        achieved = bytes_launch / (phase_ms[dominant] * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(kernels, args)
        line = {
            "metric": METRIC,
            "value": total_rows / elapsed,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic",
            "config": {"workload": "c2: synthetic homogeneous 100k nodes / 1M edges, 64-dim "
                                   "feats, 2-layer GCN, interpret_samples=256, node_prediction "
                                   "(3-hop computational subgraph of node 7)",
                       "nodes": args.nodes, "edges": args.edges, "feat": args.feat,
                       "subgraph_nodes": S, "subgraph_edges": int(sub_ei.shape[1]),
                       "interpret_samples": args.interpret_samples, "epochs": args.epochs,
                       "rows_per_repeat": R, "repeats_per_rank": T,
                       "repeats_per_step": T * world,
                       "parallelism": f"repeats sharded over {world} rank(s)",
                       "mask_sampler": "device (Philox Shapley)"},
            "phases_ms": phase_ms,
            "roofline": {"kernel": kname, "bound": "hbm", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "bytes_per_launch": bytes_launch},
        }
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args, arch, sub_feat, sub_ei, q)
        if world == 1:
            comm = None if args.no_communities else communities_section(args, dev, plan, sub_feat, sub_ei)
            del plan
            torch.cuda.empty_cache()
            regimes = {}
            if not args.no_graph_prediction:
                regimes["graph_prediction_c3"] = graph_prediction_section(args, dev)
                torch.cuda.empty_cache()
            if args.full_graph_rows > 0:
                regimes["full_graph_c3"] = full_graph_section(args, dev)
                torch.cuda.empty_cache()
            if not args.no_hetero:
                regimes["hetero_c4"] = hetero_c4_section(args, dev)
                torch.cuda.empty_cache()
            if comm is not None:
                regimes["communities_c2"] = comm
            if not args.no_communities:
                regimes["graph_queries"] = graph_queries_section(args, dev)
                torch.cuda.empty_cache()
            if regimes:
                line["regimes"] = regimes
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
