"""Diagnostic (not part of the product): wall time of consecutive Explainer.run calls in the
bench's explainer_api order (warm-up on node 8, first call on node 7, then node 7 again and
again), with the host / device ms of each phase — does the repeated call converge, and where
does each call's host time go.

    python tools/api_repeat.py [--graph c2|c3] [--calls 8] [--times 10]
"""
import argparse
import gc
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bikg_graph_explainability_public_amd.explainer import Explainer  # noqa: E402
from bikg_graph_explainability_public_amd.nn import ConvStack  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--graph", default="c2", choices=("c2", "c3"))
    p.add_argument("--calls", type=int, default=8)
    p.add_argument("--times", type=int, default=10)
    p.add_argument("--no-gc", action="store_true", help="skip gc.collect() before each call")
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    if args.graph == "c3":
        import bench
        feat, ei, arch = bench.c3_graph(dev)
        ns = 512
    else:
        g = torch.Generator().manual_seed(0)
        n, e, f = 100_000, 1_000_000, 64
        feat = torch.randn((n, f), generator=g)
        ei = torch.randint(0, n, (2, e), generator=g)
        torch.manual_seed(0)
        arch = ConvStack("gcn", [f, 64, 64], [64, 1]).eval()
        ns = 256
    n = feat.shape[0]
    params = {"seed": 1, "interpret_samples": ns, "epochs": 50, "optimizer": "adam", "lr": 0.01,
              "lr_patience": 10, "l1_lambda": 1e-4, "mask_sampler": "device"}
    exp = Explainer(feat.to(dev), ei.to(dev), arch, params, [str(i) for i in range(n)])
    for i, q in enumerate(["8"] + ["7"] * args.calls + ["9", "10", "7"]):
        torch.cuda.synchronize()
        if not args.no_gc:
            gc.collect()
        t0 = time.perf_counter()
        exp.run(q, args.times)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        ph = exp.last_run["phases"].times()
        cells = " ".join(f"{k}={v['host_ms']:.3f}/{v['device_ms']:.3f}" for k, v in ph.items()
                         if isinstance(v, dict))
        print(f"call {i:2d} q={q:>2s} {wall:7.3f} ms  {args.times * exp.last_run['repeats'][0]['rows'] / wall / 1e3:6.1f} M/s"
              f"  [{exp.last_run['query_cache']}] {cells}", flush=True)


if __name__ == "__main__":
    main()
