"""Diagnostic (not part of the product): each stage of the c2 step replayed from a captured HIP
graph against the same stage run eagerly (max |diff|, NaN counts).

    python tools/graph_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bikg_graph_explainability_public_amd import _lib, engine  # noqa: E402


def cmp(name, a, b):
    a, b = a.double(), b.double()
    print(f"{name:10s} max|diff| {float((a - b).abs().max()):.3e}  nan graph {int(torch.isnan(a).sum())} "
          f"eager {int(torch.isnan(b).sum())}", flush=True)


REPLAYS = int(os.environ.get("PROBE_REPLAYS", "1"))


def graphed(fn, replays=None):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    for _ in range(replays or REPLAYS):
        g.replay()
    torch.cuda.synchronize()
    return out


def main():
    dev = torch.device("cuda", 0)
    _lib.load()
    args = bench.parse()
    arch, sub_feat, sub_ei, q, plan = bench.build_c2(args, dev)
    S = plan.cols
    R, B = 12800, 256
    seed_t = torch.full((1,), 1234, dtype=torch.int64, device=dev)
    bits_e = engine.sample_shapley(1234, R, S, dev)
    bits_g = graphed(lambda: engine.sample_shapley_dev(seed_t, R, S))
    cmp("bits", bits_g, bits_e)
    y_e = plan.forward(bits_e)[:, 0]
    y_g = graphed(lambda: plan.forward(bits_e)[:, 0])
    cmp("forward", y_g, y_e)
    k_e = engine.shap_kernel(bits_e, S)
    k_g = graphed(lambda: engine.shap_kernel(bits_e, S))
    cmp("shap", k_g, k_e)
    w0 = torch.zeros((1, S), device=dev)
    params = {"lr": 0.01, "l1_lambda": 1e-4}
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    w_e = engine.wlm_fit(bits_e.view(1, R, -1), S, B, y_e.view(1, R), k_e.view(1, R), w0, params)[0]
    w_g = graphed(lambda: engine.wlm_fit(bits_e.view(1, R, -1), S, B, y_e.view(1, R), k_e.view(1, R), w0,
                                         params, check=False, status=st)[0])
    cmp("fit", w_g, w_e)
    print("fit status", int(st.item()), flush=True)
    os.environ["XPG_WLM"] = "single"
    w_s = graphed(lambda: engine.wlm_fit(bits_e.view(1, R, -1), S, B, y_e.view(1, R), k_e.view(1, R), w0,
                                         params, check=False, status=st)[0])
    cmp("fit-single", w_s, w_e)
    os.environ.pop("XPG_WLM")

    # the stages chained inside one graph, fed by the device-seeded sampler
    def chain():
        b = engine.sample_shapley_dev(seed_t, R, S)
        y = plan.forward(b)[:, 0]
        k = engine.shap_kernel(b, S)
        w = engine.wlm_fit(b.view(1, R, -1), S, B, y.view(1, R), k.view(1, R), w0, params,
                           check=False, status=st)[0]
        return b, y, k, w
    for n in (1, 3):
        bg, yg, kg, wg = graphed(chain, n)
        cmp(f"chain{n}.bits", bg, bits_e)
        cmp(f"chain{n}.y", yg, y_e)
        cmp(f"chain{n}.k", kg, k_e)
        cmp(f"chain{n}.w", wg, w_e)
        print("status", int(st.item()), flush=True)


if __name__ == "__main__":
    main()
